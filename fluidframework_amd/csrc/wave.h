// wave.h — the handful of wave64 primitives the merge-tree engine is written against.
//
// The engine (mt_engine.h) is SPMD code for ONE wavefront. Per-lane values are `Lane<T>`, read and
// written inside `FOR_LANES(l) { ... LANE(x) ... }` bodies; everything outside those bodies is
// wave-uniform. Cross-lane movement goes only through the functions below.
//
// On gfx950 (device compilation) a Lane<T> is one register per lane, FOR_LANES runs its body once
// with l = the lane id, and the primitives are ballot / readlane / shuffles. For host compilation
// (tests only: tests/_build/libmt_emu.so) a Lane<T> is T[64] and FOR_LANES loops over the 64 lanes,
// which lets the parity suite run the exact engine source against the oracle without a GPU.
// Rule that keeps both identical: a FOR_LANES body never reads LDS that another lane writes in the
// same body (split such code into a read body and a write body).
#pragma once

#include <stdint.h>

#if defined(__HIP_DEVICE_COMPILE__)

#include <hip/hip_runtime.h>
#define FMT_DEV __device__ __forceinline__
#define FMT_GPU 1

template <class T>
struct Lane {
  T v;
};
// Eight 32-bit values per lane held in VGPRs; a wave-uniform dynamic element index lowers to
// register-relative moves (M0 / set_gpr_idx), never to scratch memory.
typedef uint32_t V8 __attribute__((ext_vector_type(8)));
typedef uint32_t V4 __attribute__((ext_vector_type(4)));
typedef uint32_t VKV __attribute__((ext_vector_type(FMT_MT_PROPS_MAX)));  // one prop set's (key, value) words
#define LANE(x) ((x).v)
#define FOR_LANES(l) for ([[maybe_unused]] int l = static_cast<int>(__lane_id()), l##_once = 1; l##_once; l##_once = 0)

FMT_DEV int waveLane() { return static_cast<int>(__lane_id()); }

// Opaque register copy: stops LLVM from folding a dynamic vector element access back into a
// variable-index load from the enclosing object's stack slot (which would put it in scratch).
FMT_DEV void launder(V8& v) { asm volatile("" : "+v"(v)); }
FMT_DEV void launder(V4& v) { asm volatile("" : "+v"(v)); }

// Large-tier rows: a plain per-lane array indexed at run time (private memory), so the row loops
// stay rolled and the 32-row engine compiles in seconds.
template <int N>
struct VecN {
  uint32_t x[N];
  FMT_DEV uint32_t& operator[](int i) { return x[i]; }
  FMT_DEV const uint32_t& operator[](int i) const { return x[i]; }
};
using V32 = VecN<32>;

// A UTF-16 unit of a global buffer that other lanes of this wave wrote: an agent-scope load is
// served by L2 (never a stale vector-L1 line).
FMT_DEV uint32_t loadCoherent(const uint16_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
FMT_DEV uint32_t loadCoherent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
FMT_DEV int32_t loadCoherent(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A store to a global buffer whose pointer was loaded from memory (so the compiler cannot infer its
// address space): written as a global store, a flat store could alias the wave's private arrays and
// would force them out of registers around it.
template <class T>
FMT_DEV void storeGlobal(T* p, T v) {
  *reinterpret_cast<__attribute__((address_space(1))) T*>(reinterpret_cast<uintptr_t>(p)) = v;
}
FMT_DEV double loadCoherentD(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}
// A global value this workgroup wrote: a workgroup-scope atomic load is a plain vector load (served by
// the CU's L1, which this CU's own stores keep current) that the compiler never turns into a scalar
// (K$) load, whose cache vector stores do not update.
FMT_DEV uint32_t loadWg(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
FMT_DEV int32_t loadWg(const int32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
FMT_DEV uint32_t loadWg(const uint16_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
// LDS add from one lane of many (ds_add_u32); the host emulation runs lanes one after another.
FMT_DEV void atomicAddLds(int32_t* p, int v) { atomicAdd(p, v); }

// Make a wave-uniform value provably uniform (lives in an SGPR afterwards).
FMT_DEV int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
FMT_DEV uint32_t uni(uint32_t x) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(x))); }
FMT_DEV double uniD(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const uint64_t u = uni(static_cast<uint32_t>(b)) | (static_cast<uint64_t>(uni(static_cast<uint32_t>(b >> 32))) << 32);
  return __builtin_bit_cast(double, u);
}

FMT_DEV uint64_t ballot(const Lane<bool>& p) { return __ballot(p.v); }

template <class T>
FMT_DEV T readlane(const Lane<T>& x, int lane) {
  return static_cast<T>(__builtin_amdgcn_readlane(static_cast<int>(x.v), lane));
}

#ifndef FMT_USE_DPP
#define FMT_USE_DPP 1
#endif

#if FMT_USE_DPP
// GFX9 DPP controls (cdna4_isa.md §DPP): row_shr:n = 0x110+n, wave_shl:1 = 0x130, wave_shr:1 = 0x138,
// row_bcast:15 = 0x142, row_bcast:31 = 0x143. Lanes whose DPP source is invalid (or whose row is
// masked off) receive `old` = 0, so every step below is an ordinary add/max.
template <int Ctrl, int RowMask = 0xF>
FMT_DEV uint32_t dppMov(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), Ctrl, RowMask, 0xF, false));
}

template <class T>
FMT_DEV Lane<T> shflUp1(const Lane<T>& x) {  // lane l receives lane l-1 (lane 0: 0)
  return Lane<T>{static_cast<T>(dppMov<0x138>(static_cast<uint32_t>(x.v)))};
}

template <class T>
FMT_DEV Lane<T> shflDown1(const Lane<T>& x) {  // lane l receives lane l+1 (lane 63: 0)
  return Lane<T>{static_cast<T>(dppMov<0x130>(static_cast<uint32_t>(x.v)))};
}

// Inclusive wave64 prefix sum: Kogge-Stone inside 16-lane rows, then row broadcasts.
FMT_DEV uint32_t waveInclusiveSum(uint32_t v) {
  v += dppMov<0x111>(v);
  v += dppMov<0x112>(v);
  v += dppMov<0x114>(v);
  v += dppMov<0x118>(v);
  v += dppMov<0x142, 0xA>(v);
  v += dppMov<0x143, 0xC>(v);
  return v;
}

FMT_DEV Lane<uint32_t> waveExclusiveSum(const Lane<uint32_t>& x, uint32_t* total) {
  const uint32_t v = waveInclusiveSum(x.v);
  *total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
  return Lane<uint32_t>{v - x.v};
}

// Exclusive prefix max (values >= -1; `init` for lane 0). Max-scan on (v + 1) as unsigned so the
// zero that invalid DPP lanes contribute is the identity.
FMT_DEV Lane<int32_t> waveExclusiveMax(const Lane<int32_t>& x, int32_t init) {
  uint32_t v = static_cast<uint32_t>(x.v + 1);
  v = max(v, dppMov<0x111>(v));
  v = max(v, dppMov<0x112>(v));
  v = max(v, dppMov<0x114>(v));
  v = max(v, dppMov<0x118>(v));
  v = max(v, dppMov<0x142, 0xA>(v));
  v = max(v, dppMov<0x143, 0xC>(v));
  const uint32_t prev = dppMov<0x138>(v);  // exclusive: value of lane l-1
  return Lane<int32_t>{waveLane() == 0 ? init : static_cast<int32_t>(prev) - 1};
}

#else

template <class T>
FMT_DEV Lane<T> shflUp1(const Lane<T>& x) {
  return Lane<T>{static_cast<T>(__shfl_up(static_cast<int>(x.v), 1))};
}

template <class T>
FMT_DEV Lane<T> shflDown1(const Lane<T>& x) {
  return Lane<T>{static_cast<T>(__shfl_down(static_cast<int>(x.v), 1))};
}

// Exclusive prefix sum across the wave; *total = sum over all lanes.
FMT_DEV Lane<uint32_t> waveExclusiveSum(const Lane<uint32_t>& x, uint32_t* total) {
  uint32_t v = x.v;
  const int lane = waveLane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = static_cast<uint32_t>(__shfl_up(static_cast<int>(v), d));
    if (lane >= d) v += o;
  }
  *total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
  return Lane<uint32_t>{v - x.v};
}

// Exclusive prefix max across the wave (identity `init` for lane 0).
FMT_DEV Lane<int32_t> waveExclusiveMax(const Lane<int32_t>& x, int32_t init) {
  int32_t v = x.v;
  const int lane = waveLane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t o = __shfl_up(v, d);
    if (lane >= d) v = v > o ? v : o;
  }
  int32_t prev = __shfl_up(v, 1);
  return Lane<int32_t>{lane == 0 ? init : prev};
}

#endif

// Lane l receives lane src[l] of x (ds_bpermute_b32: a crossbar shuffle through the LDS unit).
FMT_DEV Lane<uint32_t> gather(const Lane<uint32_t>& x, const Lane<int>& src) {
  return Lane<uint32_t>{static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src.v << 2, static_cast<int>(x.v)))};
}

FMT_DEV void waveSync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Workgroup barrier (all waves; LDS and memory ordered across it). Call only from wave-uniform
// control flow on every wave the same number of times.
FMT_DEV void groupBarrier() { __syncthreads(); }

#else  // host emulation (tests only)

#include <cstring>
#define FMT_DEV inline
#define FMT_GPU 0

template <class T>
struct Lane {
  T v[64];
};
template <int N>
struct VecN {
  uint32_t x[N];
  uint32_t& operator[](int i) { return x[i]; }
  const uint32_t& operator[](int i) const { return x[i]; }
};
using V8 = VecN<8>;
using V32 = VecN<32>;
struct V4 {
  uint32_t x[4];
  uint32_t& operator[](int i) { return x[i]; }
  const uint32_t& operator[](int i) const { return x[i]; }
};
using VKV = VecN<FMT_MT_PROPS_MAX>;
#define LANE(x) ((x).v[l])
#define FOR_LANES(l) for (int l = 0; l < 64; l++)

inline int uni(int x) { return x; }
inline uint32_t uni(uint32_t x) { return x; }

template <class T>
inline void launder(T&) {}

inline uint32_t loadCoherent(const uint16_t* p) { return *p; }
inline uint32_t loadCoherent(const uint32_t* p) { return *p; }
inline int32_t loadCoherent(const int32_t* p) { return *p; }
inline double loadCoherentD(const double* p) { return *p; }
template <class T>
inline void storeGlobal(T* p, T v) { *p = v; }
inline double uniD(double x) { return x; }
inline uint32_t loadWg(const uint32_t* p) { return *p; }
inline int32_t loadWg(const int32_t* p) { return *p; }
inline uint32_t loadWg(const uint16_t* p) { return *p; }
inline void atomicAddLds(int32_t* p, int v) { *p += v; }

inline uint64_t ballot(const Lane<bool>& p) {
  uint64_t m = 0;
  for (int l = 0; l < 64; l++)
    if (p.v[l]) m |= 1ull << l;
  return m;
}

template <class T>
inline T readlane(const Lane<T>& x, int lane) {
  return x.v[lane];
}

template <class T>
inline Lane<T> shflUp1(const Lane<T>& x) {
  Lane<T> r;
  r.v[0] = x.v[0];
  for (int l = 1; l < 64; l++) r.v[l] = x.v[l - 1];
  return r;
}

template <class T>
inline Lane<T> shflDown1(const Lane<T>& x) {
  Lane<T> r;
  for (int l = 0; l < 63; l++) r.v[l] = x.v[l + 1];
  r.v[63] = x.v[63];
  return r;
}

inline Lane<uint32_t> waveExclusiveSum(const Lane<uint32_t>& x, uint32_t* total) {
  Lane<uint32_t> r;
  uint32_t acc = 0;
  for (int l = 0; l < 64; l++) {
    r.v[l] = acc;
    acc += x.v[l];
  }
  *total = acc;
  return r;
}

inline Lane<int32_t> waveExclusiveMax(const Lane<int32_t>& x, int32_t init) {
  Lane<int32_t> r;
  int32_t acc = init;
  for (int l = 0; l < 64; l++) {
    r.v[l] = acc;
    if (l == 0) acc = x.v[0];
    else acc = acc > x.v[l] ? acc : x.v[l];
  }
  return r;
}

inline Lane<uint32_t> gather(const Lane<uint32_t>& x, const Lane<int>& src) {
  Lane<uint32_t> r;
  for (int l = 0; l < 64; l++) r.v[l] = x.v[src.v[l] & 63];
  return r;
}

inline void waveSync() {}
inline void groupBarrier() {}

#endif

FMT_DEV int ctz64(uint64_t m) { return __builtin_ctzll(m); }
FMT_DEV int ctz32(uint32_t m) { return __builtin_ctz(m); }
