// mergetree_large.hip — merge-tree replay, large tier (32 rows in private memory: 2048 leaves,
// 131071 UTF-16 units in HBM; one document per workgroup) for the documents the small tier overflows.
#include "mergetree_kernel.h"

namespace fmt_kernels {

constexpr int kMtWavesLarge = 1;  // large tier: one document per workgroup, 1 wave/SIMD (VGPRs)

int mergeTreeProfileLarge(uint64_t* out, int n, bool reset) { return addTuProfile(out, n, reset); }

hipError_t launchMergeTreeLarge(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                                uint32_t count, int numCUs, hipStream_t stream, bool obliterate, bool removeOrder,
                                uint32_t* next, bool adjust, bool local) {
  using G = fmt_mt::LargeTier;
  if (local && adjust)  // f4 with annotate-adjust
    return launchTier<false, G, false, kMtWavesLarge, 1, true, true>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
  if (local)  // f4: the local client's submissions, acks, rollbacks and reconnects (plain ops otherwise)
    return launchTier<false, G, false, kMtWavesLarge, 1, false, true>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
  if (adjust && removeOrder)
    return launchTier<true, G, true, kMtWavesLarge, 1, true>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
  if (adjust)
    return launchTier<true, G, false, kMtWavesLarge, 1, true>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
  if (obliterate && removeOrder)
    return launchTier<true, G, true, kMtWavesLarge, 1>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
  if (obliterate)
    return launchTier<true, G, false, kMtWavesLarge, 1>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
  if (removeOrder)
    return launchTier<false, G, true, kMtWavesLarge, 1>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
  return launchTier<false, G, false, kMtWavesLarge, 1>(batch, out, docList, count, nullptr, numCUs, stream, nullptr, next);
}

}  // namespace fmt_kernels
