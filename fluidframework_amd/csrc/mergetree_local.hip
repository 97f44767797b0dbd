// mergetree_local.hip — f4 local-client batches (FMT_MT_F_LOCAL / ACK / ROLLBACK / REGEN records),
// first tier (round 6). Every document replays in the compact tier's local variant
// (Doc<false, CompactTier, false, false, true>: 4 register rows, 256 leaves, 2048 UTF-16 units in
// LDS, the pending-group count as a sixth leaf word); the documents it cannot hold (FMT_E_CAPACITY:
// leaves, text, blocks, prop sets, writers past 31) are listed in esc and replay again, from their
// first op, in the large tier's local variant (mergetree_large.hip). Round 5 ran every local document
// in the large tier (one wave per workgroup, leaf rows in private memory). The local state itself —
// pending segment groups, group records, PropertiesManager records, regenerated ops, normalization
// scratch — lives in per-document HBM slabs (mt_engine.h LocalTables) in both tiers, so a restart
// simply rewrites them.
#include "mergetree_kernel.h"

namespace fmt_kernels {

constexpr int kMtWavesLocal = 4;  // 4 documents per workgroup

hipError_t launchMergeTreeLocal(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                                uint32_t count, uint32_t* esc, int numCUs, hipStream_t stream, uint32_t* next) {
  return launchTier<false, fmt_mt::CompactTier, false, kMtWavesLocal, 3, false, true>(batch, out, docList, count, esc,
                                                                                      numCUs, stream, nullptr, next);
}

}  // namespace fmt_kernels
