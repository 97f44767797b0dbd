// map_sparse.hip — SharedMap last-writer-wins for key pools of any size (SURVEY §8(d)'s
// U[0, 2^20) variant), sparse output.
//
// Same result as map_lww.hip (MapKernel sequenced path, mapKernel.ts:706-853): a key is live when
// some set of it comes after its last delete and after the last clear; its value is the last such
// set's, and its JS Map insertion order (map.ts:176-246 / mapKernel.ts:545-551) is the order of the
// first such set (the set that re-created the entry). Seqs are strictly increasing within a document
// (fmt_map_op, checked by fmt_map_load_sparse), so every comparison runs on op ordinals i (1-based):
//     D[k] = last delete of k,   C = last clear,   a set i of k survives iff i > max(D[k], C)
//     first[k] = min surviving set,   last[k] = max surviving set.
// Per document the key ids are reduced by key in an LDS hash table of S = 64 .. 2048 slots (open
// addressing, linear probing, a key claimed with ds_cmpswap). Per slot two words:
//     key[s]: the key (claim phase), then last[k] (atomicMax), then the value id of op last[k]
//     w[s]:   first[k] << 16 | D[k]   (0xffff0000 when empty: pass 1 maxes the low half, pass 2
//             takes the min of (i << 16 | D[k]) over surviving sets, D[k] being final by then)
// Each op keeps its slot in a register, so a key is hashed and probed once. The output is sparse and
// driven by the ops, not the slots: the op that is first[k] writes key k's entry {key, value of
// last[k], its own seq} at rank = live keys born before it (a running ballot count over the ops in
// order), so no pass over the table and no global re-reads. Entries of document d go to
// out[doc_op_offsets[d] + rank], counts[d] = its live keys.
//
// One wave per document, kSpWaves per workgroup, grid-stride over documents. 16 KiB of LDS per wave
// (10 waves per CU: the table, not registers, sets occupancy). A document of up to 1024 ops is read
// into VGPRs once (16 dwordx4 per lane, non-temporal); longer ones (up to 16384 ops) stream, with
// the op's slot parked in its own (not yet written) output entry.
// Bound: HBM — 16 B read per op, 12 B written per live key.
#include <hip/hip_runtime.h>

#include "../../include/fmt.h"
#include "kernels.h"

namespace fmt_kernels {

constexpr int kSpWaves = 2;
constexpr uint32_t kSpSlots = 2048;                   // hash slots per wave = FMT_MAP_SPARSE_MAX_KEYS
constexpr uint32_t kSpMaxOps = 16384;                 // ops per document (ordinals fit 16 bits)
constexpr uint32_t kSpEmpty = 0xffffffffu;
constexpr uint32_t kSpWInit = 0xffff0000u;
constexpr int kSpRegChunks = 16;
typedef unsigned int spv4 __attribute__((ext_vector_type(4)));
// {key, seq, kind_value} of an op record (its doc word is not needed): one dwordx3 load at +4
typedef unsigned int spv3 __attribute__((ext_vector_type(3), aligned(4)));

struct SpWave {
  uint32_t key[kSpSlots];
  uint32_t w[kSpSlots];
};

__device__ __forceinline__ void spSync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Fibonacci hashing: the top log2(S) bits of key * 2^32/phi (one multiply; shift = 32 - log2 S).
__device__ __forceinline__ uint32_t spHash(uint32_t k, uint32_t shift) { return (k * 0x9e3779b1u) >> shift; }

template <int Ctrl, int RowMask>
__device__ __forceinline__ uint32_t spDpp(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), Ctrl, RowMask, 0xF, false));
}

// OR over the wave (row_shr 1/2/4/8 within rows, then row_bcast 15/31 into lane 63).
__device__ __forceinline__ uint32_t spWaveOr(uint32_t v) {
  v |= spDpp<0x111, 0xF>(v);
  v |= spDpp<0x112, 0xF>(v);
  v |= spDpp<0x114, 0xF>(v);
  v |= spDpp<0x118, 0xF>(v);
  v |= spDpp<0x142, 0xA>(v);
  v |= spDpp<0x143, 0xC>(v);
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

__device__ __forceinline__ uint32_t spWaveMax(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), off)));
  return v;
}

__device__ __forceinline__ uint32_t spLanesBelow(uint64_t ballot) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(ballot >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(ballot), 0u));
}

// One op of a chunk: key, seq and kind/value.
struct SpOp {
  uint32_t key, seq, kv;
};

__device__ __forceinline__ uint32_t spKind(const SpOp& o) { return o.kv >> FMT_MAP_KIND_SHIFT; }

// Whether the op takes a slot (a set or delete in range with a valid key id); bad key ids raise the
// error bit.
__device__ __forceinline__ bool spKeyed(const SpOp& o, bool inRange, uint32_t keyBound, int* error) {
  const bool keyedKind = inRange && (spKind(o) == FMT_MAP_SET || spKind(o) == FMT_MAP_DELETE);
  if (keyedKind && o.key >= keyBound) atomicOr(error, 1);
  return keyedKind && o.key < keyBound;
}

__device__ __forceinline__ SpOp spLoad(const spv4* recs, uint64_t i) {
  const spv3 v = __builtin_nontemporal_load(reinterpret_cast<const spv3*>(reinterpret_cast<const uint32_t*>(recs + i) + 1));
  return SpOp{v.x, v.y, v.z};
}

__device__ __forceinline__ void spPrefetch(SpOp (&pre)[kSpRegChunks], const spv4* recs, uint64_t begin, uint32_t n,
                                           int lane) {
#pragma unroll
  for (int u = 0; u < kSpRegChunks; u++) {
    // (lanes past the end load the last op again, so no load is predicated; every use of an op
    // checks its ordinal against n)
    const uint32_t i = min(u * 64u + lane, n - 1);
    pre[u] = SpOp{0u, 0u, FMT_MAP_CLEAR << FMT_MAP_KIND_SHIFT};
    if (u * 64u < n) pre[u] = spLoad(recs, begin + i);
  }
}

template <int R>
__device__ __forceinline__ bool spClaim(SpWave* w, const SpOp (&op)[R], uint32_t keyed, uint32_t (&slot)[R],
                                        uint32_t mask, uint32_t shift) {
  uint32_t pend = keyed;
#pragma unroll
  for (int u = 0; u < R; u++) slot[u] = spHash(op[u].key, shift);
  for (uint32_t probe = 0; probe <= mask; probe++) {
    uint32_t cur[R];
#pragma unroll
    for (int u = 0; u < R; u++) cur[u] = (pend >> u) & 1u ? atomicCAS(&w->key[slot[u]], kSpEmpty, op[u].key) : kSpEmpty;
#pragma unroll
    for (int u = 0; u < R; u++) {
      if ((pend >> u) & 1u) {
        if (cur[u] == kSpEmpty || cur[u] == op[u].key) pend &= ~(1u << u);
        else slot[u] = (slot[u] + 1) & mask;
      }
    }
    if (__ballot(pend != 0) == 0) return true;
  }
  return false;
}

__global__ __launch_bounds__(64 * kSpWaves) __attribute__((amdgpu_waves_per_eu(2))) void mapSparseKernel(
    const fmt_map_op* __restrict__ ops, const uint64_t* __restrict__ offsets, uint32_t nDocs, uint32_t keyBound,
    fmt_map_entry* __restrict__ out, uint32_t* __restrict__ counts, int* __restrict__ error) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  SpWave* w = reinterpret_cast<SpWave*>(lds) + wave;
  const spv4* recs = reinterpret_cast<const spv4*>(ops);
  // Software pipeline over the wave's documents: the next document's records (register path) and
  // the offsets of the one after it are in flight while this one is reduced (two waves per SIMD
  // cannot hide an HBM round trip per document otherwise).
  const uint32_t stride = gridDim.x * kSpWaves;
  uint32_t doc = blockIdx.x * kSpWaves + wave;
  if (doc >= nDocs) return;
  uint64_t b0 = offsets[doc], e0 = offsets[doc + 1], b1 = 0, e1 = 0;
  if (doc + stride < nDocs) {
    b1 = offsets[doc + stride];
    e1 = offsets[doc + stride + 1];
  }
  SpOp pre[kSpRegChunks];
  if (e0 - b0 <= 64u * kSpRegChunks) spPrefetch(pre, recs, b0, static_cast<uint32_t>(e0 - b0), lane);
  for (; doc < nDocs; doc += stride) {
    const uint64_t begin = b0, end = e0;
    const uint32_t n = static_cast<uint32_t>(end - begin);
    const bool inRegs = end - begin <= 64u * kSpRegChunks;
    // Only the ops after the document's last clear can leave an entry (a clear empties the map,
    // mapKernel.ts:708-760, and seqs grow with the ordinal): the rest is skipped. C = the last
    // clear's ordinal (1-based), 0 without one.
    SpOp op[kSpRegChunks];
    uint32_t keyed = 0;  // bit u: op u takes a slot (a set / delete after C with a valid key id)
    uint32_t C = 0;
    if (inRegs) {
#pragma unroll
      for (int u = 0; u < kSpRegChunks; u++) op[u] = pre[u];
#pragma unroll
      for (int u = kSpRegChunks - 1; u >= 0; u--) {
        if (C != 0 || u * 64u >= n) continue;
        const uint64_t b = __ballot(u * 64u + lane < n && spKind(op[u]) == FMT_MAP_CLEAR);
        if (b != 0) C = u * 64u + 64u - static_cast<uint32_t>(__clzll(static_cast<long long>(b)));
      }
      bool bad = false;
#pragma unroll
      for (int u = 0; u < kSpRegChunks; u++) {
        const uint32_t i1 = u * 64u + lane + 1, k = spKind(op[u]);
        const bool kk = i1 <= n && (k == FMT_MAP_SET || k == FMT_MAP_DELETE);
        bad |= kk && op[u].key >= keyBound;  // (a bad key before the last clear is still an error)
        keyed |= kk && op[u].key < keyBound && i1 > C ? 1u << u : 0u;
      }
      if (__ballot(bad) != 0 && lane == 0) atomicOr(error, 1);
    } else if (n <= kSpMaxOps) {
      for (uint32_t c = 0; c < n; c += 64) {
        const uint32_t i = c + lane;
        bool bad = false;
        if (i < n) {
          const spv4 v = recs[begin + i];
          const uint32_t k = v.w >> FMT_MAP_KIND_SHIFT;
          if (k == FMT_MAP_CLEAR) C = i + 1;
          bad = (k == FMT_MAP_SET || k == FMT_MAP_DELETE) && v.y >= keyBound;
        }
        if (__ballot(bad) != 0 && lane == 0) atomicOr(error, 1);
      }
      C = spWaveMax(C);
    }
    // the next document's records, then the offsets of the one after it (a vector load: a scalar
    // one would share lgkmcnt with the LDS traffic below and stall its first wait)
    if (doc + stride < nDocs && e1 - b1 <= 64u * kSpRegChunks) spPrefetch(pre, recs, b1, static_cast<uint32_t>(e1 - b1), lane);
    const uint32_t far = doc + 2 * stride;
    uint64_t offv = 0;
    if (far < nDocs) offv = offsets[far + (lane & 1)];
    if (n > kSpMaxOps) {  // ordinals beyond 16 bits: reported, no entries
      if (lane == 0) {
        counts[doc] = 0;
        atomicOr(error, 2);
      }
    } else {
      // table size: >= 2 slots per op after the last clear (load <= 1/2), 64 .. 2048
      const uint32_t m = n - C;
      uint32_t S = 64, shift = 26;
      while (S < 2 * m && S < kSpSlots) {
        S <<= 1;
        shift--;
      }
      const uint32_t mask = S - 1;
      for (uint32_t s = lane * 4; s < S; s += 256) {
        *reinterpret_cast<spv4*>(&w->key[s]) = spv4{kSpEmpty, kSpEmpty, kSpEmpty, kSpEmpty};
        *reinterpret_cast<spv4*>(&w->w[s]) = spv4{kSpWInit, kSpWInit, kSpWInit, kSpWInit};
      }
      fmt_map_entry* o = out + begin;
      uint32_t live = 0;
      bool full = false;
      const uint32_t u0 = C / 64;  // first chunk holding an op after the last clear
      if (inRegs) {
        uint32_t slot[kSpRegChunks], cur[kSpRegChunks];
        spSync();
#pragma unroll
        for (int u = 0; u < kSpRegChunks; u++) slot[u] = spHash(op[u].key, shift);
        // first probe of every op at once; collisions probe on, each round visiting only the
        // chunks some lane still has pending (a wave-OR of the pending masks, scalar bit tests)
#pragma unroll
        for (int u = 0; u < kSpRegChunks; u++) {
          cur[u] = kSpEmpty;
          if (u < static_cast<int>(u0) || u * 64u >= n) continue;
          if ((keyed >> u) & 1u) cur[u] = atomicCAS(&w->key[slot[u]], kSpEmpty, op[u].key);
        }
        uint32_t pend = 0;
#pragma unroll
        for (int u = 0; u < kSpRegChunks; u++) {
          const bool miss = ((keyed >> u) & 1u) && cur[u] != kSpEmpty && cur[u] != op[u].key;
          pend |= miss ? 1u << u : 0u;
          slot[u] = miss ? (slot[u] + 1) & mask : slot[u];
        }
        for (uint32_t probe = 1, any = spWaveOr(pend); any != 0; probe++, any = spWaveOr(pend)) {
          if (probe > mask) {
            full = true;
            break;
          }
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++) {
            if (((any >> u) & 1u) == 0) continue;
            if ((pend >> u) & 1u) cur[u] = atomicCAS(&w->key[slot[u]], kSpEmpty, op[u].key);
          }
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++) {
            if (((any >> u) & 1u) == 0) continue;
            if ((pend >> u) & 1u) {
              if (cur[u] == kSpEmpty || cur[u] == op[u].key) pend &= ~(1u << u);
              else slot[u] = (slot[u] + 1) & mask;
            }
          }
        }
        if (!full) {
          // the last delete of every key
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++) {
            if (u < static_cast<int>(u0) || u * 64u >= n) continue;
            if (((keyed >> u) & 1u) && spKind(op[u]) == FMT_MAP_DELETE) atomicMax(&w->w[slot[u]], kSpWInit | (u * 64u + lane + 1));
          }
          spSync();
          for (uint32_t s = lane * 4; s < S; s += 256) *reinterpret_cast<spv4*>(&w->key[s]) = spv4{0u, 0u, 0u, 0u};
          uint32_t d[kSpRegChunks];
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++) {
            d[u] = 0;
            if (u < static_cast<int>(u0) || u * 64u >= n) continue;
            d[u] = w->w[slot[u]] & 0xffffu;
          }
          spSync();
          uint32_t surv = 0;  // bit u: op u is a surviving set
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++) {
            if (u < static_cast<int>(u0) || u * 64u >= n) continue;
            const uint32_t i1 = u * 64 + lane + 1;
            if (((keyed >> u) & 1u) && spKind(op[u]) == FMT_MAP_SET && i1 > d[u]) {
              surv |= 1u << u;
              atomicMin(&w->w[slot[u]], (i1 << 16) | d[u]);
              atomicMax(&w->key[slot[u]], i1);
            }
          }
          spSync();
          uint32_t birth = 0, last = 0;
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++) {
            if (u < static_cast<int>(u0) || u * 64u >= n) continue;
            const uint32_t i1 = u * 64 + lane + 1;
            const uint32_t f = w->w[slot[u]] >> 16, l = w->key[slot[u]];
            const bool sv = (surv >> u) & 1u;
            birth |= sv && f == i1 ? 1u << u : 0u;
            last |= sv && l == i1 ? 1u << u : 0u;
          }
          spSync();
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++)
            if ((last >> u) & 1u) w->key[slot[u]] = op[u].kv & FMT_MAP_VALUE_MASK;
          spSync();
#pragma unroll
          for (int u = 0; u < kSpRegChunks; u++) {
            if (u < static_cast<int>(u0) || u * 64u >= n) continue;
            const bool b = (birth >> u) & 1u;
            const uint64_t bal = __ballot(b);
            if (bal == 0) continue;
            if (b) {
              fmt_map_entry e;
              e.key = op[u].key;
              e.value = w->key[slot[u]];
              e.birth_seq = op[u].seq;
              o[live + spLanesBelow(bal)] = e;
            }
            live += static_cast<uint32_t>(__popcll(bal));
          }
        }
      } else {
        // streaming (n > 1024): the op's slot is parked in the key word of its own output entry
        // (entries are written at ranks <= the op's ordinal, after the op's slot was read)
        uint32_t* park = reinterpret_cast<uint32_t*>(o);
        const uint32_t c0 = u0 * 64;
        spSync();
        for (uint32_t c = c0; c < n && !full; c += 64) {
          const uint32_t i = c + lane;
          const spv4 v = i < n ? recs[begin + i] : spv4{0u, 0u, 0u, FMT_MAP_CLEAR << FMT_MAP_KIND_SHIFT};
          const uint32_t k = v.w >> FMT_MAP_KIND_SHIFT;
          SpOp op1[1] = {SpOp{v.y, v.z, v.w}};
          const uint32_t keyed1 = i < n && i + 1 > C && (k == FMT_MAP_SET || k == FMT_MAP_DELETE) && v.y < keyBound ? 1u : 0u;
          uint32_t slot[1];
          full = !spClaim(w, op1, keyed1, slot, mask, shift);
          if (i < n) park[3 * i] = keyed1 ? slot[0] : 0xffffffffu;
          if (!full && keyed1 && k == FMT_MAP_DELETE) atomicMax(&w->w[slot[0]], kSpWInit | (i + 1));
        }
        if (!full) {
          spSync();
          for (uint32_t s = lane * 4; s < S; s += 256) *reinterpret_cast<spv4*>(&w->key[s]) = spv4{0u, 0u, 0u, 0u};
          spSync();
          // the low halves (D) are final: read them all before pass 2 changes any w word
          for (uint32_t c = c0; c < n; c += 64) {
            const uint32_t i = c + lane;
            if (i >= n) continue;
            const uint32_t s = park[3 * i];
            uint32_t m2 = 0;  // 0: not a surviving set
            if (s != 0xffffffffu && (recs[begin + i].w >> FMT_MAP_KIND_SHIFT) == FMT_MAP_SET) {
              const uint32_t dd = w->w[s] & 0xffffu;
              if (i + 1 > dd) m2 = ((i + 1) << 16) | dd;
            }
            park[3 * i + 1] = m2;
          }
          spSync();
          for (uint32_t c = c0; c < n; c += 64) {
            const uint32_t i = c + lane;
            if (i >= n) continue;
            const uint32_t s = park[3 * i], m2 = park[3 * i + 1];
            if (m2) {
              atomicMin(&w->w[s], m2);
              atomicMax(&w->key[s], i + 1);
            }
          }
          spSync();
          // the last set of each live key parks its value in its slot: first mark, then write, so no
          // op reads a key word that already holds a value
          for (uint32_t c = c0; c < n; c += 64) {
            const uint32_t i = c + lane;
            if (i >= n) continue;
            const uint32_t s = park[3 * i], m2 = park[3 * i + 1];
            uint32_t fl = 0;
            if (m2) fl = ((w->w[s] >> 16) == i + 1 ? 1u : 0u) | (w->key[s] == i + 1 ? 2u : 0u);
            park[3 * i + 2] = fl;
          }
          spSync();
          for (uint32_t c = c0; c < n; c += 64) {
            const uint32_t i = c + lane;
            if (i < n && (park[3 * i + 2] & 2u)) w->key[park[3 * i]] = recs[begin + i].w & FMT_MAP_VALUE_MASK;
          }
          spSync();
          for (uint32_t c = c0; c < n; c += 64) {
            const uint32_t i = c + lane;
            bool b = false;
            fmt_map_entry e;
            if (i < n && (park[3 * i + 2] & 1u)) {
              const spv4 v = recs[begin + i];
              b = true;
              e.key = v.y;
              e.value = w->key[park[3 * i]];
              e.birth_seq = v.z;
            }
            const uint64_t bal = __ballot(b);
            if (b) o[live + spLanesBelow(bal)] = e;  // rank <= i: never a parked word still to be read
            live += static_cast<uint32_t>(__popcll(bal));
          }
        }
      }
      if (full) {  // more distinct keys than the table holds: reported, no entries
        live = 0;
        if (lane == 0) atomicOr(error, 2);
      }
      if (lane == 0) counts[doc] = live;
      spSync();
    }
    b0 = b1;
    e0 = e1;
    b1 = static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(offv), 0))) |
         (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(offv >> 32), 0))) << 32);
    e1 = static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(offv), 1))) |
         (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(offv >> 32), 1))) << 32);
  }
}

// Packs each document's entries (out[doc_op_offsets[d] ..]) into consecutive ranges (packedOff[d]).
__global__ void mapSparsePackKernel(const fmt_map_entry* __restrict__ in, const uint64_t* __restrict__ offsets,
                                    const uint32_t* __restrict__ counts, const uint64_t* __restrict__ packedOff,
                                    uint32_t nDocs, fmt_map_entry* __restrict__ packed) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t d = blockIdx.x * 4 + wave; d < nDocs; d += gridDim.x * 4) {
    const uint64_t src = offsets[d], dst = packedOff[d];
    for (uint32_t i = lane; i < counts[d]; i += 64) packed[dst + i] = in[src + i];
  }
}

size_t mapSparseLdsBytes() { return sizeof(SpWave) * kSpWaves; }

hipError_t launchMapSparse(const fmt_map_op* ops, const uint64_t* offsets, uint32_t nDocs, uint32_t keyBound,
                           fmt_map_entry* out, uint32_t* counts, int* error, int numCUs, hipStream_t stream) {
  const size_t lds = mapSparseLdsBytes();
  int blocksPerCU = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocksPerCU, mapSparseKernel, 64 * kSpWaves, lds) != hipSuccess ||
      blocksPerCU <= 0)
    blocksPerCU = 1;
  const uint32_t wanted = (nDocs + kSpWaves - 1) / kSpWaves;
  const uint32_t cap = static_cast<uint32_t>(numCUs * blocksPerCU);
  const uint32_t grid = wanted < cap ? (wanted > 0 ? wanted : 1) : cap;
  hipLaunchKernelGGL(mapSparseKernel, dim3(grid), dim3(64 * kSpWaves), lds, stream, ops, offsets, nDocs, keyBound, out,
                     counts, error);
  return hipGetLastError();
}

hipError_t launchMapSparsePack(const fmt_map_entry* in, const uint64_t* offsets, const uint32_t* counts,
                               const uint64_t* packedOff, uint32_t nDocs, fmt_map_entry* packed, hipStream_t stream) {
  const uint32_t blocks = nDocs / 4 + 1;
  hipLaunchKernelGGL(mapSparsePackKernel, dim3(blocks < 65536 ? blocks : 65536), dim3(256), 0, stream, in, offsets,
                     counts, packedOff, nDocs, packed);
  return hipGetLastError();
}

static_assert(sizeof(SpWave) * kSpWaves <= 160 * 1024, "the sparse map tables must fit one CU's LDS");

}  // namespace fmt_kernels
