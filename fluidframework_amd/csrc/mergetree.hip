// mergetree.hip — merge-tree replay, small tier (8 register rows: 512 leaves, 2 waves/SIMD), the
// overflow-list kernel and the tier cascade (kernel template: mergetree_kernel.h).
//
// A plain batch replays every document in the compact tier first (mergetree_compact.hip: 4 rows,
// 3 waves/SIMD); the documents it overflows replay in this tier from a device-side list; those this
// tier overflows go to the large tier (mergetree_large.hip) after the host reads the list length.
// Batches holding obliterates or remove-order recording start in this tier.
#define FMT_MT_COLLECT_DEFINE 1
#include "mergetree_kernel.h"

namespace fmt_kernels {

constexpr int kMtWaves = 4;  // small tier: 4 documents per workgroup, 2 waves/SIMD

int mergeTreeProfileCompact(uint64_t* out, int n, bool reset);
int mergeTreeProfileLarge(uint64_t* out, int n, bool reset);

int mergeTreeProfile(uint64_t* out, int n, bool reset) {
  for (int c = 0; c < n; c++) out[c] = 0;
  if (addTuProfile(out, n, reset) < 0 || mergeTreeProfileCompact(out, n, reset) < 0 ||
      mergeTreeProfileLarge(out, n, reset) < 0)
    return -1;
  return fmt_mt::kPfCount;
}

MtCaps mergeTreeCaps(bool large) {
  if (large)
    return MtCaps{static_cast<uint32_t>(Slab<fmt_mt::LargeTier>::kLeaves), static_cast<uint32_t>(Slab<fmt_mt::LargeTier>::kChars),
                  static_cast<uint32_t>(Slab<fmt_mt::LargeTier>::kProps)};
  return MtCaps{static_cast<uint32_t>(Slab<fmt_mt::SmallTier>::kLeaves), static_cast<uint32_t>(Slab<fmt_mt::SmallTier>::kChars),
                static_cast<uint32_t>(Slab<fmt_mt::SmallTier>::kProps)};
}

size_t mergeTreeCheckpointBytes() { return sizeof(uint32_t) * fmt_mt::Doc<false, fmt_mt::CompactTier>::kCkptWords; }

hipError_t launchMergeTreeCompact(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                                  uint32_t count, uint32_t* esc, int numCUs, hipStream_t stream, uint32_t* next,
                                  bool obliterate);

// The compact tier's overflow list in[0] = n, in[1..n] reordered into out by remaining ops,
// longest first (64 buckets between 0 and the largest remainder): with documents dealt to waves
// in list order, the small-tier pass then ends on short documents (longest-processing-time first).
// A checkpointed document has ops [ckpt next, end) left, any other one its whole stream.
constexpr int kOrderBuckets = 64;
__global__ __launch_bounds__(1024) void orderByRemainingKernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                               const fmt_mt_doc_result* __restrict__ headers,
                                                               const uint64_t* __restrict__ offs,
                                                               const uint32_t* __restrict__ ckpt, uint32_t ckptWords) {
  __shared__ uint32_t cnt[kOrderBuckets], base[kOrderBuckets], maxRem;
  const uint32_t n = in[0];
  if (threadIdx.x < kOrderBuckets) cnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) maxRem = 0;
  __syncthreads();
  auto remaining = [&](uint32_t d) -> uint32_t {
    uint64_t first = offs[d];
    if (headers[d].status == fmt_mt::kCkptEscalate) {
      const uint32_t* h = ckpt + static_cast<size_t>(d) * ckptWords;
      first = h[0] | (static_cast<uint64_t>(h[1]) << 32);
    }
    const uint64_t r = offs[d + 1] - first;
    return r > 0xffffffffull ? 0xffffffffu : static_cast<uint32_t>(r);
  };
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicMax(&maxRem, remaining(in[1 + i]));
  __syncthreads();
  const uint64_t span = static_cast<uint64_t>(maxRem) + 1;
  auto bucket = [&](uint32_t r) -> uint32_t {  // 0 = the longest remainders
    return kOrderBuckets - 1 - static_cast<uint32_t>(static_cast<uint64_t>(r) * kOrderBuckets / span);
  };
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[bucket(remaining(in[1 + i]))], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int b = 0; b < kOrderBuckets; b++) {
      base[b] = s;
      s += cnt[b];
    }
    out[0] = n;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t d = in[1 + i];
    out[1 + atomicAdd(&base[bucket(remaining(d))], 1u)] = d;
  }
}

// Variants: obliterates (Ob) and/or the remove-order recording of SnapshotV1 batches (Rm).
hipError_t launchMergeTree(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                           uint32_t count, uint32_t* esc, uint32_t* esc2, uint32_t* esc3, int numCUs,
                           hipStream_t stream, bool obliterate, bool removeOrder, uint32_t* sched, bool adjust) {
  using S = fmt_mt::SmallTier;
  uint32_t* n1 = sched ? sched + 1 : nullptr;
  if (adjust) {  // annotate-adjust batches: the Adj variants, small tier over every document (no checkpoints)
    // (1 wave/SIMD: 512 registers a wave; at 2 the property-manager code spilled 3710 VGPRs to scratch,
    // at 1 the overflow lives in AGPRs)
    if (removeOrder)
      return launchTier<true, S, true, kMtWaves, 1, true>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
    return launchTier<true, S, false, kMtWaves, 1, true>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  }
  if (obliterate && removeOrder)
    return launchTier<true, S, true, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  if (obliterate && (esc == nullptr || esc2 == nullptr))
    return launchTier<true, S, false, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  if (removeOrder)
    return launchTier<false, S, true, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  if (esc == nullptr || esc2 == nullptr)
    return launchTier<false, S, false, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  // compact tier over everything → overflow list esc2 → this tier over that list → overflow list esc
  hipError_t e = launchMergeTreeCompact(batch, out, docList, count, esc2, numCUs, stream, sched, obliterate);
  if (e != hipSuccess) return e;
  if (esc3 != nullptr && out.ckpt != nullptr) {  // longest remaining streams first
    hipLaunchKernelGGL(orderByRemainingKernel, dim3(1), dim3(1024), 0, stream, esc2, esc3, out.headers,
                       batch.docOpOffsets, out.ckpt,
                       static_cast<uint32_t>(fmt_mt::Doc<false, fmt_mt::CompactTier>::kCkptWords));
    esc2 = esc3;
  }
  if (obliterate)
    return launchTier<true, S, false, kMtWaves, 2>(batch, out, esc2 + 1, count, esc, numCUs, stream, esc2, n1);
  return launchTier<false, S, false, kMtWaves, 2>(batch, out, esc2 + 1, count, esc, numCUs, stream, esc2, n1);
}

}  // namespace fmt_kernels
