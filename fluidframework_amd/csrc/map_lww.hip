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
// sets; pass 2 re-reads the document's ops, which are L2-resident after pass 1 (HBM traffic stays
// one read of every op). Bound: HBM bandwidth — 16 B read per op, 8 B written per key slot.
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

__global__ __launch_bounds__(256) void mapLwwKernel(const fmt_map_op* __restrict__ ops,
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

  for (uint32_t doc = blockIdx.x * kWaves + wave; doc < nDocs; doc += gridDim.x * kWaves) {
    for (uint32_t k = lane; k < keyBound; k += 64) {
      last[k] = 0;
      kill[k] = 0;
      first[k] = 0xffffffffu;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint64_t begin = offsets[doc], end = offsets[doc + 1];

    // Pass 1: kills.
    uint32_t clearMax = 0;
    for (uint64_t c = begin; c < end; c += 64 * kUnroll) {
      uint4 rec[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const uint64_t i = c + u * 64 + lane;
        rec[u] = i < end ? *reinterpret_cast<const uint4*>(ops + i) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const uint64_t i = c + u * 64 + lane;
        if (i >= end) continue;
        const uint32_t kind = rec[u].w >> FMT_MAP_KIND_SHIFT;
        if (kind == FMT_MAP_DELETE) {
          if (rec[u].y < keyBound) atomicMax(&kill[rec[u].y], rec[u].z);
          else atomicOr(error, 1);
        } else if (kind == FMT_MAP_CLEAR) {
          clearMax = max(clearMax, rec[u].z);
        }
      }
    }
    clearMax = waveMax(clearMax);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();

    // Pass 2: surviving sets.
    for (uint64_t c = begin; c < end; c += 64 * kUnroll) {
      uint4 rec[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const uint64_t i = c + u * 64 + lane;
        rec[u] = i < end ? *reinterpret_cast<const uint4*>(ops + i) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const uint64_t i = c + u * 64 + lane;
        if (i >= end) continue;
        const uint32_t kind = rec[u].w >> FMT_MAP_KIND_SHIFT;
        if (kind != FMT_MAP_SET) continue;
        const uint32_t key = rec[u].y, seq = rec[u].z;
        if (key >= keyBound) {
          atomicOr(error, 1);
          continue;
        }
        if (seq > max(kill[key], clearMax)) {
          atomicMax(&last[key], (static_cast<unsigned long long>(seq) << 32) | (rec[u].w & FMT_MAP_VALUE_MASK));
          atomicMin(&first[key], seq);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();

    fmt_map_slot* o = out + static_cast<uint64_t>(doc) * keyBound;
    for (uint32_t k = lane; k < keyBound; k += 64) {
      const unsigned long long l = last[k];
      fmt_map_slot s;
      s.value = l != 0 ? static_cast<uint32_t>(l) : FMT_MAP_ABSENT;
      s.birth_seq = l != 0 ? first[k] : 0;
      o[k] = s;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

size_t mapLwwLdsBytes(uint32_t keyBound) { return static_cast<size_t>(kWaves) * keyBound * 16; }

hipError_t launchMapLww(const fmt_map_op* ops, const uint64_t* offsets, uint32_t nDocs, uint32_t keyBound,
                        fmt_map_slot* out, int* error, int numCUs, hipStream_t stream) {
  const size_t lds = mapLwwLdsBytes(keyBound);
  const uint32_t wanted = (nDocs + kWaves - 1) / kWaves;
  const int blocksPerCU = lds <= 20 * 1024 ? 8 : static_cast<int>(160 * 1024 / lds);
  const uint32_t cap = static_cast<uint32_t>(numCUs * (blocksPerCU > 0 ? blocksPerCU : 1));
  const uint32_t grid = wanted < cap ? (wanted > 0 ? wanted : 1) : cap;
  hipLaunchKernelGGL(mapLwwKernel, dim3(grid), dim3(64 * kWaves), lds, stream, ops, offsets, nDocs, keyBound,
                     out, error);
  return hipGetLastError();
}

}  // namespace fmt_kernels
