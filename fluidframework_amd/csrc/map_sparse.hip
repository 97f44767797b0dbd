// map_sparse.hip — SharedMap last-writer-wins for key pools of any size (SURVEY §8(d)'s
// U[0, 2^20) variant), sparse output.
//
// Same reductions as map_lww.hip (MapKernel sequenced path, mapKernel.ts:706-853):
//     kill[k]  = max(seq of delete(k), seq of any clear)
//     last[k]  = the last set of k with seq > kill[k];   first[k] = the first such set
// but per document the key ids are first reduced by key in an LDS hash table (open addressing,
// linear probing, key claimed with ds_cmpswap), so the table is sized by the document's distinct
// keys, not by the key pool. The output is sparse: one fmt_map_entry per live key, written in JS
// Map insertion order (birth seq ascending, map.ts:176-246 / mapKernel.ts:545-551) — each entry's
// rank is the number of live keys born before it, from a bitmap over op ordinals (births are
// distinct ops) and one wave prefix scan. Entries of document d go to out[doc_op_offsets[d] + rank]
// (a document has at most as many live keys as ops), counts[d] = its live keys.
//
// One wave per document, kWaves per workgroup, grid-stride over documents; a document of up to
// 1024 ops is read into VGPRs once (16 dwordx4 per lane, non-temporal), longer ones stream twice.
// Bound: HBM — 16 B read per op, 12 B written per live key.
#include <hip/hip_runtime.h>

#include "../../include/fmt.h"
#include "kernels.h"

namespace fmt_kernels {

constexpr int kSpWaves = 4;
constexpr uint32_t kSpSlots = 2048;                   // hash slots per wave = FMT_MAP_SPARSE_MAX_KEYS
constexpr uint32_t kSpMaxOps = 16384;                 // ops per document (birth bitmap)
constexpr uint32_t kSpEmpty = 0xffffffffu;
constexpr int kSpRegChunks = 16;
typedef unsigned int spv4 __attribute__((ext_vector_type(4)));

struct SpWave {
  uint32_t key[kSpSlots];
  uint32_t kill[kSpSlots];   // kill seq
  uint32_t first[kSpSlots];  // op ordinal of the first surviving set (0xffffffff: none)
  uint32_t last[kSpSlots];   // op ordinal of the last surviving set
  uint32_t born[kSpMaxOps / 32];     // bit i: op ordinal i is a live key's birth
  uint32_t wordBase[kSpMaxOps / 32]; // live births before word w
  uint32_t overflow;
};

__device__ __forceinline__ void spSync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t spHash(uint32_t k) {  // murmur3 finalizer
  k ^= k >> 16;
  k *= 0x85ebca6bu;
  k ^= k >> 13;
  k *= 0xc2b2ae35u;
  k ^= k >> 16;
  return k & (kSpSlots - 1);
}

// The slot holding `key` (claimed if new); kSpEmpty when the table is full.
__device__ __forceinline__ uint32_t spSlot(SpWave* w, uint32_t key) {
  uint32_t h = spHash(key);
  for (uint32_t probe = 0; probe < kSpSlots; probe++) {
    const uint32_t cur = atomicCAS(&w->key[h], kSpEmpty, key);
    if (cur == kSpEmpty || cur == key) return h;
    h = (h + 1) & (kSpSlots - 1);
  }
  return kSpEmpty;
}

__device__ __forceinline__ uint32_t spWaveMax(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), off)));
  return v;
}

__device__ __forceinline__ void spKill(SpWave* w, const uint4& r, uint32_t keyBound, uint32_t& clearMax, int* error) {
  const uint32_t kind = r.w >> FMT_MAP_KIND_SHIFT;
  if (kind == FMT_MAP_DELETE) {
    if (r.y >= keyBound) {
      atomicOr(error, 1);
      return;
    }
    const uint32_t s = spSlot(w, r.y);
    if (s == kSpEmpty) w->overflow = 1u;
    else atomicMax(&w->kill[s], r.z);
  } else if (kind == FMT_MAP_CLEAR) {
    clearMax = max(clearMax, r.z);
  }
}

__device__ __forceinline__ void spSet(SpWave* w, const uint4& r, uint32_t idx, uint32_t keyBound, uint32_t clearMax,
                                      int* error) {
  if ((r.w >> FMT_MAP_KIND_SHIFT) != FMT_MAP_SET) return;
  if (r.y >= keyBound) {
    atomicOr(error, 1);
    return;
  }
  const uint32_t s = spSlot(w, r.y);
  if (s == kSpEmpty) {
    w->overflow = 1u;
    return;
  }
  if (r.z > max(w->kill[s], clearMax)) {  // (kills are final: pass 1 is complete)
    atomicMax(&w->last[s], idx);
    atomicMin(&w->first[s], idx);
  }
}

__global__ __launch_bounds__(64 * kSpWaves) void mapSparseKernel(const fmt_map_op* __restrict__ ops,
                                                           const uint64_t* __restrict__ offsets, uint32_t nDocs,
                                                           uint32_t keyBound, fmt_map_entry* __restrict__ out,
                                                           uint32_t* __restrict__ counts, int* __restrict__ error) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  SpWave* w = reinterpret_cast<SpWave*>(lds) + wave;
  const uint4* recs = reinterpret_cast<const uint4*>(ops);
  for (uint32_t doc = blockIdx.x * kSpWaves + wave; doc < nDocs; doc += gridDim.x * kSpWaves) {
    const uint64_t begin = offsets[doc], end = offsets[doc + 1];
    const uint32_t n = static_cast<uint32_t>(end - begin);
    if (end - begin > kSpMaxOps) {  // beyond the birth bitmap: reported, no entries
      if (lane == 0) {
        counts[doc] = 0;
        atomicOr(error, 2);
      }
      continue;
    }
    for (uint32_t s = lane; s < kSpSlots; s += 64) {
      w->key[s] = kSpEmpty;
      w->kill[s] = 0;
      w->first[s] = kSpEmpty;
      w->last[s] = 0;
    }
    for (uint32_t i = lane; i < (n + 31) / 32; i += 64) w->born[i] = 0;
    if (lane == 0) w->overflow = 0;
    uint32_t clearMax = 0;
    if (n <= 64u * kSpRegChunks) {
      uint4 rec[kSpRegChunks];
#pragma unroll
      for (int u = 0; u < kSpRegChunks; u++) {
        const uint32_t i = u * 64 + lane;
        rec[u] = make_uint4(0, 0, 0, 0);
        if (u * 64u < n && i < n) {
          const spv4 v = __builtin_nontemporal_load(reinterpret_cast<const spv4*>(recs + begin + i));
          rec[u] = make_uint4(v.x, v.y, v.z, v.w);
        }
      }
      spSync();
#pragma unroll
      for (int u = 0; u < kSpRegChunks; u++)
        if (u * 64u < n && u * 64u + lane < n) spKill(w, rec[u], keyBound, clearMax, error);
      clearMax = spWaveMax(clearMax);
      spSync();
#pragma unroll
      for (int u = 0; u < kSpRegChunks; u++)
        if (u * 64u < n && u * 64u + lane < n) spSet(w, rec[u], u * 64 + lane, keyBound, clearMax, error);
    } else {
      spSync();
      for (uint32_t i = lane; i < n; i += 64) spKill(w, recs[begin + i], keyBound, clearMax, error);
      clearMax = spWaveMax(clearMax);
      spSync();
      for (uint32_t i = lane; i < n; i += 64) spSet(w, recs[begin + i], i, keyBound, clearMax, error);
    }
    spSync();
    if (w->overflow) {  // more distinct keys than the table holds: reported, no entries
      if (lane == 0) {
        counts[doc] = 0;
        atomicOr(error, 2);
      }
      spSync();
      continue;
    }
    // every slot of this lane (kSlotsPerLane, unrolled): live keys mark their births in the bitmap,
    // and the value / birth-seq loads of all of them are issued before any is used
    constexpr int kPer = kSpSlots / 64;
    uint32_t sk[kPer], sf[kPer], sl[kPer];
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      const uint32_t sl0 = lane + 64 * i;
      sk[i] = w->key[sl0];
      sf[i] = w->first[sl0];
      sl[i] = w->last[sl0];
    }
#pragma unroll
    for (int i = 0; i < kPer; i++)
      if (sk[i] != kSpEmpty && sf[i] != kSpEmpty) atomicOr(&w->born[sf[i] >> 5], 1u << (sf[i] & 31));
    uint32_t val[kPer], bseq[kPer];
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      const bool live = sk[i] != kSpEmpty && sf[i] != kSpEmpty;
      val[i] = live ? recs[begin + sl[i]].w : 0u;
      bseq[i] = live ? recs[begin + sf[i]].z : 0u;
    }
    spSync();
    // word prefixes of the birth bitmap (one wave scan over per-lane sums)
    const uint32_t nWords = (n + 31) / 32, per = (nWords + 63) / 64;
    uint32_t mine = 0;
    for (uint32_t k = 0; k < per; k++) {
      const uint32_t wi = lane * per + k;
      if (wi < nWords) mine += __popc(w->born[wi]);
    }
    uint32_t incl = mine;  // inclusive wave prefix sum
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = static_cast<uint32_t>(__shfl_up(static_cast<int>(incl), off));
      if (lane >= off) incl += t;
    }
    const uint32_t total = static_cast<uint32_t>(__shfl(static_cast<int>(incl), 63));
    uint32_t run = incl - mine;
    for (uint32_t k = 0; k < per; k++) {
      const uint32_t wi = lane * per + k;
      if (wi < nWords) {
        w->wordBase[wi] = run;
        run += __popc(w->born[wi]);
      }
    }
    spSync();
    fmt_map_entry* o = out + begin;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      if (sk[i] == kSpEmpty || sf[i] == kSpEmpty) continue;
      const uint32_t f = sf[i];
      const uint32_t rank = w->wordBase[f >> 5] + __popc(w->born[f >> 5] & ((1u << (f & 31)) - 1u));
      fmt_map_entry e;
      e.key = sk[i];
      e.value = val[i] & FMT_MAP_VALUE_MASK;
      e.birth_seq = bseq[i];
      o[rank] = e;
    }
    if (lane == 0) counts[doc] = total;
    spSync();
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
