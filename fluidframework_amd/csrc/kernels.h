// kernels.h — host-side launchers of the gfx950 kernels (one .hip translation unit each).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/fmt.h"

namespace fmt_mt {
struct AdjustTables;  // mt_engine.h
struct LocalTables;   // mt_engine.h (f4)
}

namespace fmt_kernels {

// ---- SharedMap LWW (map_lww.hip)
size_t mapLwwLdsBytes(uint32_t keyBound);
// key pools beyond the LDS table take the HBM-table path, which needs 2 * key_bound u32 of scratch
// per document (nullptr otherwise)
bool mapLwwNeedsScratch(uint32_t keyBound);
size_t mapSparseLdsBytes();
hipError_t launchMapSparse(const fmt_map_op* ops, const uint64_t* offsets, uint32_t nDocs, uint32_t keyBound,
                           fmt_map_entry* out, uint32_t* counts, int* error, int numCUs, hipStream_t stream);
hipError_t launchMapSparsePack(const fmt_map_entry* in, const uint64_t* offsets, const uint32_t* counts,
                               const uint64_t* packedOff, uint32_t nDocs, fmt_map_entry* packed, hipStream_t stream);
// ---- SharedMap local-client pending state (map_pending.hip)
size_t mapPendingScratchBytes(uint64_t nEvents);
hipError_t launchMapPending(const fmt_map_local_op* events, const uint64_t* evOffs, const fmt_map_entry* seqEntries,
                            const uint64_t* seqOffs, const uint32_t* seqCounts, uint32_t nDocs, void* scratch,
                            const uint64_t* outBase, fmt_map_entry* out, uint32_t* outCounts, int32_t* outStatus,
                            hipStream_t stream);
hipError_t launchMapLww(const fmt_map_op* ops, const uint64_t* offsets, uint32_t nDocs, uint32_t keyBound,
                        fmt_map_slot* out, int* error, int numCUs, hipStream_t stream, uint32_t* scratch);

// ---- merge-tree replay (mergetree.hip)
struct MtDeviceBatch {
  const fmt_mt_op* ops;
  const uint64_t* docOpOffsets;
  uint32_t nDocs;
  const uint16_t* text;
  const uint32_t* docInit;  // (offset, len) per doc or nullptr
  const uint32_t* propsOff;
  const uint32_t* propsKv;
  uint32_t nPropsOps;
  const uint64_t* catchupOffsets;  // per-doc catch-up slab offsets (nDocs + 1), or nullptr
  const fmt_mt_snapshot_doc* snapshots;  // per-doc summary loads, or nullptr
  const fmt_mt_snapshot_seg* snapshotSegs;
  const uint64_t* rmOrderOffsets;  // per-doc remove-order slab offsets (nDocs + 1), or nullptr
  const fmt_mt_snapshot_info* snapshotInfo;  // SnapshotV1 merge info per snapshot segment, or nullptr
  const fmt_mt_stamp* snapshotStamps;
  uint64_t nSnapshotInfo;
  const fmt_mt_relpos* relpos;     // relative positions (FMT_MT_F_REL1/REL2 ops), or nullptr
  uint32_t nRelpos;
  uint32_t markerKey;              // key id of "markerId", FMT_MT_NO_MARKER if none
  const fmt_mt::AdjustTables* adj;  // annotate-adjust tables (device memory), nullptr when none
  const fmt_mt::LocalTables* loc = nullptr;  // f4 local-client slabs (device memory), nullptr when none
};

struct MtDeviceOut {
  fmt_mt_doc_result* headers;  // nDocs
  fmt_mt_leaf* leaves;         // nDocs * capLeaves
  uint16_t* chars;             // nDocs * capChars
  fmt_mt_propset* props;       // nDocs * capProps
  fmt_mt_catchup_range* catchup;  // slabs at catchupOffsets, or nullptr
  fmt_mt_remove_order* rmOrder;   // slabs at rmOrderOffsets, or nullptr
  uint32_t* ckpt;                 // plain batches: per-document compact → small tier checkpoints, or nullptr
  // large tier over a plain batch: the small tier's result slabs, where it left its checkpoints
  const fmt_mt_leaf* smallLeaves;
  const uint16_t* smallChars;
  // annotate-adjust batches: per leaf the prop set of getAtSeq(minSeq) (legacy summaries), at the
  // leaves slab's stride; nullptr otherwise
  uint16_t* legacyProps;
  // large tier over a plain batch: per large-tier slot, its large → huge checkpoint record
  // (huge_ckpt.h, fmt_ckpt::kWords words), or nullptr
  uint32_t* hugeCkpt = nullptr;
};
// Bytes of one document's tier checkpoint (mt_engine.h Doc::kCkptWords).
size_t mergeTreeCheckpointBytes();

// Per-document capacities of the small (LDS-text) and large (HBM-text) engine tiers.
// Bulk legacy summaries (summary.hip): a document's result buffers, its runs and its output spans.
struct SumView {
  const fmt_mt_leaf* leaves;
  const uint16_t* chars;
  const fmt_mt_propset* props;
  const uint16_t* legacyProps;  // per leaf: the prop set the legacy summary reads, or nullptr (leaf.props)
  const uint32_t* cls;          // per prop set its match class as the engine interned it (huge documents,
                                // up to 65534 sets), or nullptr: the summary kernel derives it in LDS
  const uint64_t* rmHi;         // per leaf its remove clients 64..253 (3 words: 64..127, 128..191, 192..253;
                                // huge documents of batches with such clients), or nullptr: none
};
struct SumRun {
  uint32_t len;    // UTF-16 units of the merged segment
  uint16_t props;  // prop set id of its head leaf (0xffff: undefined)
  uint16_t flags;  // 1: a Marker (its one unit is the refType)
};
struct SumDocOut {
  unsigned long long run_off, text_off;
  uint32_t n_runs, n_units, status, pad;
};
hipError_t launchSummaryRuns(const fmt_mt_doc_result* hdrs, const SumView* views, uint32_t nDocs, SumRun* runs,
                             uint16_t* text, unsigned long long* cursors, SumDocOut* docOut, int numCUs,
                             hipStream_t stream);
// Packing before a D2H copy (transfer.hip): span i's `words` dwords from src to dst + dstWord.
struct GatherSpan {
  const uint32_t* src;
  uint64_t dstWord;
  uint32_t words, pad;
};
hipError_t launchGatherSpans(const GatherSpan* spans, uint32_t n, uint32_t* dst, int numCUs, hipStream_t stream);
// Per-document content digest of the converged state (digest.hip).
hipError_t launchStateDigest(const fmt_mt_doc_result* hdrs, const SumView* views, uint32_t nDocs, uint64_t* out,
                             int numCUs, hipStream_t stream);

struct MtCaps {
  uint32_t leaves, chars, props;
};
MtCaps mergeTreeCaps(bool large);

// Compact + small tiers: replays documents docList[0..count) (or all docs when docList == nullptr);
// documents that overflow the small tier are listed in esc (esc[0] = count, then ids) when esc !=
// nullptr. A plain batch (no obliterates, no remove order) with esc2 != nullptr starts in the compact
// tier and lists its overflow in esc2 (count + 1 entries) for the small tier. esc[0] and esc2[0] must
// be zero before the call. sched: 3 zeroed device counters (compact, small, large) from which the
// tiers deal documents to waves dynamically (nullptr: static grid-stride shares). adjust: the batch
// holds annotate-adjust entries (the Adj engine variants, small tier first, no checkpoints).
hipError_t launchMergeTree(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                           uint32_t count, uint32_t* esc, uint32_t* esc2, uint32_t* esc3, int numCUs,
                           hipStream_t stream, bool obliterate, bool removeOrder, uint32_t* sched, bool adjust);

// Large tier over docList[0..count): out.leaves/chars/props are slabs indexed by list position.
hipError_t launchMergeTreeLarge(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                                uint32_t count, int numCUs, hipStream_t stream, bool obliterate, bool removeOrder,
                                uint32_t* next, bool adjust, bool local = false);

// f4 local-client batches (round 6): the small tier's local variant over docList[0..count) (or every
// document; FMT_LOCAL_PATH selects a compact-tier pass first, documents it cannot hold listed in esc2),
// the ones it cannot hold listed in esc (esc[0] = count, then ids) for launchMergeTreeLarge(..., local =
// true). esc[0] and esc2[0] zeroed by the caller; sched: zeroed dealing counters (compact, small).
// adjust: annotate-adjust batches, the small tier's Adj local variant.
hipError_t launchMergeTreeLocal(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                                uint32_t count, uint32_t* esc, uint32_t* esc2, int numCUs, hipStream_t stream,
                                uint32_t* sched, bool adjust = false);

// Diagnostic: per-phase cycle totals of a FMT_PROFILE=1 build (all zero otherwise).
int mergeTreeProfile(uint64_t* out, int n, bool reset);

}  // namespace fmt_kernels

// ---- huge documents (hugedoc.hip, huge_engine.h): one wave per document, state in HBM
namespace fmt_huge {
struct HugeState;
struct HugeInputs;
}  // namespace fmt_huge

namespace fmt_kernels {

struct HugeOut {
  fmt_mt_doc_result* header;
  fmt_mt_leaf* leaves;
  uint64_t capLeaves;
  uint16_t* chars;
  uint64_t capChars;
  fmt_mt_propset* props;
  uint16_t* legacy;          // annotate-adjust batches: per leaf the getAtSeq(minSeq) prop set, else nullptr
  const uint32_t* cls;       // the engine's match class per prop set (HugeState::pClass)
  unsigned long long* prof;  // [24] shader-clock totals per phase (huge_engine.h HugeDoc::prof)
  uint64_t* leavesHi;        // per leaf its remove clients 64..253 (3 words, bit (c - 64) % 64 of word (c - 64) / 64;
                             // fmt_mt_fetch_rm_clients_hi / _hi2), or nullptr
};
size_t hugeLdsBytes();
hipError_t launchHugeDocs(const fmt_huge::HugeState* states, const fmt_huge::HugeInputs* inputs, const HugeOut* outs,
                          uint32_t count, bool adjust, bool rmOrder, hipStream_t stream);

}  // namespace fmt_kernels
