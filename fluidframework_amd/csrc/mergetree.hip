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
                                  uint32_t count, uint32_t* esc, int numCUs, hipStream_t stream, uint32_t* next);

// Variants: obliterates (Ob) and/or the remove-order recording of SnapshotV1 batches (Rm).
hipError_t launchMergeTree(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                           uint32_t count, uint32_t* esc, uint32_t* esc2, int numCUs, hipStream_t stream,
                           bool obliterate, bool removeOrder, uint32_t* sched) {
  using S = fmt_mt::SmallTier;
  uint32_t* n1 = sched ? sched + 1 : nullptr;
  if (obliterate && removeOrder)
    return launchTier<true, S, true, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  if (obliterate)
    return launchTier<true, S, false, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  if (removeOrder)
    return launchTier<false, S, true, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  if (esc == nullptr || esc2 == nullptr)
    return launchTier<false, S, false, kMtWaves, 2>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  // compact tier over everything → overflow list esc2 → this tier over that list → overflow list esc
  hipError_t e = launchMergeTreeCompact(batch, out, docList, count, esc2, numCUs, stream, sched);
  if (e != hipSuccess) return e;
  return launchTier<false, S, false, kMtWaves, 2>(batch, out, esc2 + 1, count, esc, numCUs, stream, esc2, n1);
}

}  // namespace fmt_kernels
