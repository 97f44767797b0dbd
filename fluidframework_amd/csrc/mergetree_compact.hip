// mergetree_compact.hip — merge-tree replay, compact tier (4 register rows: 256 leaves). Plain batches
// start here; see mergetree.hip for the cascade. Plain batches run it at 4 waves/SIMD (128 VGPRs, 14
// spilled; 16 waves × 9312 B of LDS per CU): A/B at full T1 449 -> 395 ms against 3 waves/SIMD at
// 152 VGPRs (profiles/r3/cw4/). Obliterate batches keep 3 (168 VGPRs, the full Scratch).
#include "mergetree_kernel.h"

namespace fmt_kernels {

constexpr int kMtWavesCompact = 4;  // 4 documents per workgroup

int mergeTreeProfileCompact(uint64_t* out, int n, bool reset) { return addTuProfile(out, n, reset); }

hipError_t launchMergeTreeCompact(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                                  uint32_t count, uint32_t* esc, int numCUs, hipStream_t stream, uint32_t* next,
                                  bool obliterate) {
  if (obliterate)  // Doc<true>: the same 4 rows plus the live-obliterate table (163 VGPRs)
    return launchTier<true, fmt_mt::CompactTier, false, kMtWavesCompact, 3>(batch, out, docList, count, esc, numCUs,
                                                                           stream, nullptr, next);
  return launchTier<false, fmt_mt::CompactTier, false, kMtWavesCompact, 4>(batch, out, docList, count, esc, numCUs,
                                                                          stream, nullptr, next);
}

}  // namespace fmt_kernels
