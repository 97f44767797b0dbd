// map_lww.hip — SharedMap last-writer-wins replay for gfx950.
//
// Semantics (MapKernel sequenced path, packages/dds/map/src/mapKernel.ts:706-853, JS Map order):
// for every key, the converged entry is the last "set" after the last delete(key)/clear; the key is
// live iff such a set exists, and its Map insertion position (summary order for non-index keys) is
// the seq of the FIRST set after that kill. Within a document ops arrive in seq order, so
//     kill[k]  = max(seq of delete(k), seq of any clear)
//     last[k]  = max over sets of k with seq > kill[k] of (seq, value)
//     first[k] = min over sets of k with seq > kill[k] of seq
// which is two order-independent reductions per key: no per-op sequential dependency remains.
//
// Mapping: one wavefront per document, 4 documents per 256-thread workgroup, grid-stride over
// documents. Each lane owns one 16-byte op record per 64-op chunk (one coalesced dwordx4 load per
// lane, 1 KiB per wave instruction). Per-key reductions are LDS atomics (ds_max_u32, ds_max_u64,
// ds_min_u32) on a per-wave key table of key_bound entries. Pass 1 reduces kills, pass 2 reduces
// sets. A document of up to 1024 ops is read once into VGPRs (16 dwordx4 per lane, all issued
// before the first LDS update) and both passes run on registers, so HBM sees every op record once.
// Bound: HBM bandwidth — 16 B read per op, 8 B written per key slot.
#include <hip/hip_runtime.h>

#include "../../include/fmt.h"
#include "kernels.h"

namespace fmt_kernels {

constexpr int kWaves = 4;
constexpr int kUnroll = 4;  // 64-op chunks in flight per lane

struct MapKeyTables {
  uint32_t* kill;
  uint32_t* first;
  unsigned long long* last;
};

__device__ __forceinline__ uint32_t waveMax(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), off)));
  return v;
}

// Reductions of one op record (pass 1: kills, pass 2: surviving sets).
__device__ __forceinline__ void killOp(const uint4& r, uint32_t keyBound, uint32_t* kill, uint32_t& clearMax,
                                       int* error) {
  const uint32_t kind = r.w >> FMT_MAP_KIND_SHIFT;
  if (kind == FMT_MAP_DELETE) {
    if (r.y < keyBound) atomicMax(&kill[r.y], r.z);
    else atomicOr(error, 1);
  } else if (kind == FMT_MAP_CLEAR) {
    clearMax = max(clearMax, r.z);
  }
}

__device__ __forceinline__ void setOp(const uint4& r, uint32_t keyBound, const uint32_t* kill, uint32_t clearMax,
                                      unsigned long long* last, uint32_t* first, int* error) {
  if ((r.w >> FMT_MAP_KIND_SHIFT) != FMT_MAP_SET) return;
  const uint32_t key = r.y, seq = r.z;
  if (key >= keyBound) {
    atomicOr(error, 1);
    return;
  }
  if (seq > max(kill[key], clearMax)) {
    atomicMax(&last[key], (static_cast<unsigned long long>(seq) << 32) | (r.w & FMT_MAP_VALUE_MASK));
    atomicMin(&first[key], seq);
  }
}

__device__ __forceinline__ void waveSync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Records held per lane by the single-pass path: a document of up to 64 * kRegChunks ops is read
// from HBM exactly once into VGPRs, and both reductions run on the registers. Longer documents take
// the two-pass streaming path (the second pass then hits L2 only partly).
constexpr int kRegChunks = 16;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64 * kWaves) void mapLwwKernel(const fmt_map_op* __restrict__ ops,
                                                    const uint64_t* __restrict__ offsets, uint32_t nDocs,
                                                    uint32_t keyBound, fmt_map_slot* __restrict__ out,
                                                    int* __restrict__ error) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  // per wave: last[K] (8 B) | kill[K] (4 B) | first[K] (4 B)
  unsigned char* base = lds + static_cast<size_t>(wave) * keyBound * 16;
  unsigned long long* last = reinterpret_cast<unsigned long long*>(base);
  uint32_t* kill = reinterpret_cast<uint32_t*>(base + static_cast<size_t>(keyBound) * 8);
  uint32_t* first = kill + keyBound;
  const uint4* recs = reinterpret_cast<const uint4*>(ops);

  for (uint32_t doc = blockIdx.x * kWaves + wave; doc < nDocs; doc += gridDim.x * kWaves) {
    const uint64_t begin = offsets[doc], end = offsets[doc + 1];
    const uint64_t n = end - begin;
    uint32_t clearMax = 0;
    if (n <= 64u * kRegChunks) {
      // Issue every load of the document before touching LDS so they are all in flight together.
      uint4 rec[kRegChunks];
      const uint4 zero = make_uint4(0, 0, 0, 0);  // kind 0 = set of key 0 at seq 0: never survives
#pragma unroll
      for (int u = 0; u < kRegChunks; u++) {
        const uint64_t i = u * 64 + lane;
        rec[u] = zero;
        if (u * 64u < n && i < n) {
          // streamed once: non-temporal dwordx4 (6.1 vs 5.3 TB/s at M2, tools/bench_variants.py)
          const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(recs + begin + i));
          rec[u] = make_uint4(v.x, v.y, v.z, v.w);
        }
      }
      for (uint32_t k = lane; k < keyBound; k += 64) {
        last[k] = 0;
        kill[k] = 0;
        first[k] = 0xffffffffu;
      }
      waveSync();
#pragma unroll
      for (int u = 0; u < kRegChunks; u++)
        if (u * 64u < n && u * 64u + lane < n) killOp(rec[u], keyBound, kill, clearMax, error);
      clearMax = waveMax(clearMax);
      waveSync();
#pragma unroll
      for (int u = 0; u < kRegChunks; u++)
        if (u * 64u < n && u * 64u + lane < n) setOp(rec[u], keyBound, kill, clearMax, last, first, error);
    } else {
      for (uint32_t k = lane; k < keyBound; k += 64) {
        last[k] = 0;
        kill[k] = 0;
        first[k] = 0xffffffffu;
      }
      waveSync();
      for (uint64_t c = begin; c < end; c += 64 * kUnroll) {
        uint4 rec[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
          const uint64_t i = c + u * 64 + lane;
          rec[u] = i < end ? recs[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; u++)
          if (c + u * 64 + lane < end) killOp(rec[u], keyBound, kill, clearMax, error);
      }
      clearMax = waveMax(clearMax);
      waveSync();
      for (uint64_t c = begin; c < end; c += 64 * kUnroll) {
        uint4 rec[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
          const uint64_t i = c + u * 64 + lane;
          rec[u] = i < end ? recs[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; u++)
          if (c + u * 64 + lane < end) setOp(rec[u], keyBound, kill, clearMax, last, first, error);
      }
    }
    waveSync();

    fmt_map_slot* o = out + static_cast<uint64_t>(doc) * keyBound;
    for (uint32_t k = lane; k < keyBound; k += 64) {
      const unsigned long long l = last[k];
      fmt_map_slot s;
      s.value = l != 0 ? static_cast<uint32_t>(l) : FMT_MAP_ABSENT;
      s.birth_seq = l != 0 ? first[k] : 0;
      o[k] = s;
    }
    waveSync();
  }
}

size_t mapLwwLdsBytes(uint32_t keyBound) { return static_cast<size_t>(kWaves) * keyBound * 16; }

// Key pools too large for the per-wave LDS table (more than 2560 key ids): the same two reductions
// with the key tables in HBM. `last` is the output slot itself viewed as one u64 per (doc, key);
// kill and first live in a scratch slab of 2 * key_bound u32 per document (all kill rows, then all
// first rows), filled by hipMemsetAsync before the launch. One wave per document:
// pass 1 (kills) and pass 2 (surviving sets) are device-scope atomics; pass 2 reads kill[] with
// agent-scope loads, so a line another wave pulled into this CU's L1 is never read stale.
// mapLwwFinish then turns each slot's (seq << 32 | value) into (value, birth seq).
__global__ __launch_bounds__(64 * kWaves) void mapLwwHbmKernel(const fmt_map_op* __restrict__ ops,
                                                       const uint64_t* __restrict__ offsets, uint32_t nDocs,
                                                       uint32_t keyBound, unsigned long long* __restrict__ last,
                                                       uint32_t* __restrict__ killAll, uint32_t* __restrict__ firstAll,
                                                       int* __restrict__ error) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const uint4* recs = reinterpret_cast<const uint4*>(ops);
  for (uint32_t doc = blockIdx.x * kWaves + wave; doc < nDocs; doc += gridDim.x * kWaves) {
    const uint64_t begin = offsets[doc], end = offsets[doc + 1];
    const uint64_t row = static_cast<uint64_t>(doc) * keyBound;
    uint32_t* kill = killAll + row;
    uint32_t* first = firstAll + row;
    unsigned long long* lastD = last + row;
    uint32_t clearMax = 0;
    for (uint64_t i = begin + lane; i < end; i += 64) {
      const uint4 r = recs[i];
      const uint32_t kind = r.w >> FMT_MAP_KIND_SHIFT;
      if (kind == FMT_MAP_DELETE) {
        if (r.y < keyBound) atomicMax(&kill[r.y], r.z);
        else atomicOr(error, 1);
      } else if (kind == FMT_MAP_CLEAR) {
        clearMax = max(clearMax, r.z);
      }
    }
    clearMax = waveMax(clearMax);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
    for (uint64_t i = begin + lane; i < end; i += 64) {
      const uint4 r = recs[i];
      if ((r.w >> FMT_MAP_KIND_SHIFT) != FMT_MAP_SET) continue;
      if (r.y >= keyBound) {
        atomicOr(error, 1);
        continue;
      }
      const uint32_t k = __hip_atomic_load(&kill[r.y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (r.z > max(k, clearMax)) {
        atomicMax(&lastD[r.y], (static_cast<unsigned long long>(r.z) << 32) | (r.w & FMT_MAP_VALUE_MASK));
        atomicMin(&first[r.y], r.z);
      }
    }
  }
}

__global__ void mapLwwFinishKernel(uint64_t nSlots, fmt_map_slot* __restrict__ out, const uint32_t* __restrict__ first) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nSlots;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const unsigned long long l = reinterpret_cast<const unsigned long long*>(out)[i];
    fmt_map_slot s;
    s.value = l != 0 ? static_cast<uint32_t>(l) : FMT_MAP_ABSENT;
    s.birth_seq = l != 0 ? first[i] : 0;
    out[i] = s;
  }
}

bool mapLwwNeedsScratch(uint32_t keyBound) { return mapLwwLdsBytes(keyBound) > 160 * 1024; }

hipError_t launchMapLww(const fmt_map_op* ops, const uint64_t* offsets, uint32_t nDocs, uint32_t keyBound,
                        fmt_map_slot* out, int* error, int numCUs, hipStream_t stream, uint32_t* scratch) {
  if (mapLwwNeedsScratch(keyBound)) {
    const uint64_t nSlots = static_cast<uint64_t>(nDocs) * keyBound;
    uint32_t* kill = scratch;
    uint32_t* first = scratch + nSlots;
    // tables start as last = 0, kill = 0, first = 0xffffffff (fill kernels at full HBM rate)
    hipError_t e = hipMemsetAsync(out, 0, nSlots * sizeof(fmt_map_slot), stream);
    if (e == hipSuccess) e = hipMemsetAsync(kill, 0, nSlots * sizeof(uint32_t), stream);
    if (e == hipSuccess) e = hipMemsetAsync(first, 0xff, nSlots * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const uint32_t grid = nDocs == 0 ? 1 : (nDocs + kWaves - 1) / kWaves;
    hipLaunchKernelGGL(mapLwwHbmKernel, dim3(grid < 65535u * 16 ? grid : 65535u * 16), dim3(64 * kWaves), 0, stream,
                       ops, offsets, nDocs, keyBound, reinterpret_cast<unsigned long long*>(out), kill, first, error);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint64_t blocks = (nSlots + 255) / 256;
    hipLaunchKernelGGL(mapLwwFinishKernel, dim3(blocks < 65536 ? (blocks ? blocks : 1) : 65536), dim3(256), 0, stream,
                       nSlots, out, first);
    return hipGetLastError();
  }
  const size_t lds = mapLwwLdsBytes(keyBound);
  const uint32_t wanted = (nDocs + kWaves - 1) / kWaves;
  // One resident wave of workgroups (occupancy is VGPR-limited by the register-held records).
  int blocksPerCU = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocksPerCU, mapLwwKernel, 64 * kWaves, lds) != hipSuccess ||
      blocksPerCU <= 0)
    blocksPerCU = 1;
  const uint32_t cap = static_cast<uint32_t>(numCUs * blocksPerCU);
  const uint32_t grid = wanted < cap ? (wanted > 0 ? wanted : 1) : cap;
  hipLaunchKernelGGL(mapLwwKernel, dim3(grid), dim3(64 * kWaves), lds, stream, ops, offsets, nDocs, keyBound,
                     out, error);
  return hipGetLastError();
}

}  // namespace fmt_kernels
