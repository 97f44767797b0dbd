// mergetree_local.hip — f4 local-client batches (FMT_MT_F_LOCAL / ACK / ROLLBACK / REGEN records),
// the tiers below the large one (round 6). Round 5 ran every local document in the large tier (one
// wave per workgroup, leaf rows in private memory). Now a local batch takes a register tier first, as
// plain batches do, but without checkpoints: the small tier's local variant
// (Doc<false, SmallTier, false, false, true>: 8 register rows, 512 leaves, 6144 UTF-16 units in LDS,
// the pending-group count as a sixth leaf word) replays every document, and the ones it cannot hold
// (FMT_E_CAPACITY) replay again, from their first op, in the large tier's local variant
// (mergetree_large.hip). The compact tier's local variant (4 rows) can go first instead
// (FMT_LOCAL_PATH). The local state itself — pending segment groups, group records,
// PropertiesManager records, regenerated ops, normalization scratch — lives in per-document HBM slabs
// (mt_engine.h LocalTables) in every tier, so a restart simply rewrites them.
#include "mergetree_kernel.h"

namespace fmt_kernels {

constexpr int kMtWavesLocal = 4;  // 4 documents per workgroup
// 0: compact → large; 1: small → large (kept: the reference farms' writer views overflow the compact
// tier in 17 of 28 streams; A/B at 20k documents 383 ms against 410 for 2 and 1379 for 0,
// profiles/r6/local2/ab_local.json); 2: compact → small → large (tools/build_variants.py loc*)
#ifndef FMT_LOCAL_PATH
#define FMT_LOCAL_PATH 1
#endif

hipError_t launchMergeTreeLocal(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                                uint32_t count, uint32_t* esc, uint32_t* esc2, int numCUs, hipStream_t stream,
                                uint32_t* sched, bool adjust) {
  using K = fmt_mt::CompactTier;
  using S = fmt_mt::SmallTier;
  uint32_t* n0 = sched, * n1 = sched ? sched + 1 : nullptr;
  // annotate-adjust batches (round 6): the PropertiesManager's remote and local change lists with
  // adjust folding (Doc<..., Adj, Loc>), small tier first whatever FMT_LOCAL_PATH says
  if (adjust)
    return launchTier<false, S, false, kMtWavesLocal, 2, true, true>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  if constexpr (FMT_LOCAL_PATH == 0)
    return launchTier<false, K, false, kMtWavesLocal, 3, false, true>(batch, out, docList, count, esc, numCUs, stream, nullptr, n0);
  if constexpr (FMT_LOCAL_PATH == 1)
    return launchTier<false, S, false, kMtWavesLocal, 2, false, true>(batch, out, docList, count, esc, numCUs, stream, nullptr, n1);
  // compact over everything → overflow list esc2 → the small tier over that list → overflow list esc
  if constexpr (FMT_LOCAL_PATH != 2) return hipErrorInvalidValue;
  hipError_t e = launchTier<false, K, false, kMtWavesLocal, 3, false, true>(batch, out, docList, count, esc2, numCUs, stream,
                                                                            nullptr, n0);
  if (e != hipSuccess) return e;
  return launchTier<false, S, false, kMtWavesLocal, 2, false, true>(batch, out, esc2 + 1, count, esc, numCUs, stream, esc2, n1);
}

}  // namespace fmt_kernels
