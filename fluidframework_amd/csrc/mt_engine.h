// mt_engine.h — merge-tree observer replay for ONE document on ONE wavefront (gfx950 wave64).
//
// Reference semantics (packages/dds/merge-tree/src): Client.applyMsg → applyRemoteOp
// (client.ts:1291-1379) → MergeTree.insertSegments / markRangeRemoved / annotateRange
// (mergeTree.ts:1484-1517, 2292-2383, 2009-2081), the inserting walk (mergeTree.ts:1811-1987),
// zamboni (zamboni.ts:33-213) with its LRU heap (core-utils/src/heap.ts:54-182), and
// updateSeqNumbers / setMinSeq (client.ts:1381-1391, mergeTree.ts:1147-1166).
//
// MI355X data layout (what replaces the JS object tree):
//   * Leaves live in VGPRs, in document order, row-major: leaf j is element j >> 6 ("row") of
//     lane j & 63, five 32-bit words each (W0 len|block|props, W1 insert seq, W2 first-remove seq,
//     W3 remove-client mask, W4 leaf id|insert client). 40 VGPRs hold up to 512 leaves; passes
//     visit only the rows that hold leaves (wave-uniform guard). A perspective's visible length
//     of every leaf, its prefix sums, and every "which leaf holds position p" question are then
//     lane-local arithmetic plus one wave scan / ballot: no tree walk and no partial-lengths index
//     (the reference's PartialSequenceLengths is only an index whose value must equal the sum of
//     leaf lengths, partialLengths.ts:1189-1240). Insert/delete of a leaf is a one-lane DPP shift
//     (wave_shr / wave_shl) of the rows at and above it, with a one-lane carry between rows.
//   * The B+tree above the leaves is kept exactly (it decides zamboni scope and therefore the
//     segmentation that summaries expose): leaf blocks are contiguous runs of leaves tagged with a
//     block id; interior blocks store child lists. Block table, LRU heap, prop-set table and the
//     document's UTF-16 text in document order (tombstones included) live in LDS (~8.5 KiB/wave).
// Every decision that the reference makes by walking the tree is reproduced from these arrays:
//   ensureIntervalBoundary: split the unique leaf that strictly contains pos in the op's view;
//   insert: the new leaf goes before the first leaf whose view-prefix equals pos, skipping leaves
//           removed at/below minSeq except the very last leaf (mergeTree.ts:1862-1875, breakTie
//           :1811-1826 is always true at remaining position 0 for a remote op), into that leaf's
//           block; past the end it is appended to the last leaf's block;
//   nodeMap: the leaves of positive view length inside [start, end).
#pragma once

#include "../../include/fmt.h"
#include "wave.h"
#include "adjust.h"
#include "huge_ckpt.h"

#include <cstddef>
#include <type_traits>

#if FMT_GPU
#define FMT_LDS __attribute__((address_space(3)))
#else
#define FMT_LDS
#endif

namespace fmt_mt {

constexpr int kMaxNodes = 8;         // MaxNodesInBlock (mergeTreeNodes.ts:248)
constexpr int kGranularity = 256;    // TextSegmentGranularity (textSegment.ts:21)
constexpr int kObCap = 64;           // obliterates alive in the collab window (seq > minSeq)
constexpr int kKeysMax = FMT_MT_PROPS_KEYS_MAX;  // keys of one prop set (working-set slots)
constexpr int kKeyChunks = kKeysMax / 64;        // slot k = chunk k / 64, lane k % 64
static_assert(kKeysMax % 64 == 0, "prop-set slots come in whole waves");
constexpr int32_t kNotRemoved = 0x7fffffff;
constexpr int kCapacityFinal = -33;  // internal status (small tier only), never leaves the runtime
constexpr int kCkptEscalate = -34;   // internal status: the compact tier stopped at a checkpoint (Doc::saveCkpt)

// Capacity tiers. Every document first replays in the small tier (leaves in 40 VGPRs, text in
// LDS, 2 waves/SIMD). A document that overflows it (FMT_E_CAPACITY) is replayed again from its
// inputs in the large tier: 32 rows of 2048 leaves in per-lane private memory, 10-bit block ids,
// 63 writers, 64 prop sets, and the text in the document's HBM output slab instead of LDS. Same
// engine source. Small: W0 = len | block << kLenBits | props << (kLenBits + kBlkBits); large:
// W0 = len | block << kLenBits, props in W6.
struct SmallTier {
  static constexpr int kRows = 8;          // rows of 64 leaves (one VR element per row)
  // UTF-16 units per document (tombstones included): the LDS left per wave at 2 waves/SIMD (8 per
  // CU: 8 × 19424 B of Scratch fits the 160 KiB)
  static constexpr int kCapChars = 6144;
  static constexpr int kMaxBlocks = 128;
  static constexpr int kHeapCap = 255;
  static constexpr int kPropCap = 32;
  static constexpr int kLenBits = 16, kBlkBits = 8;  // props: the remaining 8 bits
  static constexpr bool kHbmChars = false;
  static constexpr bool kUnroll = true;     // rows are compile-time VGPR elements
  static constexpr int kWords = 5;          // remove-client set: W3 (writers 1..31)
  static constexpr int kMaxClient = 31;
  static constexpr bool kPropsWord = false; // prop-set id in W0
  using BId = uint8_t;
  using VR = V8;
};

// The compact tier: the small tier's layout with 4 register rows (256 leaves), so the replay kernel
// fits 168 VGPRs and runs 3 waves per SIMD instead of 2 (more waves to cover the LDS and readlane
// latency of each wave's dependent op chain). Plain batches replay in it first; a document that
// outgrows it replays again in the small tier (runtime cascade).
struct CompactTier : SmallTier {
  static constexpr int kRows = 4;
  static constexpr int kCapChars = 2048;  // 12 waves/CU × 11232 B of Scratch
  using VR = V4;
};

struct LargeTier {
  static constexpr int kRows = 32;
  static constexpr int kCapChars = 131071;  // a leaf length (17 bits) can hold all of them
  static constexpr int kMaxBlocks = 1023;   // ids 0..1022; 1023 = no block
  static constexpr int kHeapCap = 1023;     // at most one heap entry per block (needsScour)
  static constexpr int kPropCap = 1024;     // prop-set ids in their own word W6; 0xFFFF = undefined
  static constexpr int kLenBits = 17, kBlkBits = 10;
  static constexpr bool kHbmChars = true;
  static constexpr bool kUnroll = false;    // rows indexed at run time (private memory)
  static constexpr int kWords = 7;          // remove-client set: W3 (ids 0..31) + W5 (ids 32..63); W6 props
  static constexpr int kMaxClient = 63;
  static constexpr bool kPropsWord = true;  // prop-set id in W6
  using BId = uint16_t;
  using VR = V32;
};

// Uniform row loops: unrolled so that the row is a compile-time V8 element, with a wave-uniform
// guard so rows outside [lo, hi) cost one scalar branch.
#define FMT_PRAGMA(x) _Pragma(#x)
// (Large tier: rolled loops over exactly [lo, hi), rows indexed at run time.)
#define FOR_ROWS(r, lo, hi)                                                                            \
  FMT_PRAGMA(unroll kRowUnroll)                                                                      \
  for (int r = kRowUnroll > 1 ? 0 : (lo); r < (kRowUnroll > 1 ? kRows : ((hi) < kRows ? (hi) : kRows)); r++) \
    if (r >= (lo) && r < (hi))
#define FOR_ROWS_DOWN(r, lo, hi)                                                                          \
  FMT_PRAGMA(unroll kRowUnroll)                                                                        \
  for (int r = kRowUnroll > 1 ? kRows - 1 : ((hi) < kRows ? (hi) : kRows) - 1; r >= (kRowUnroll > 1 ? 0 : (lo)); r--) \
    if (r >= (lo) && r < (hi))

template <class BId>
struct Blk {
  uint8_t count;
  BId parent;
  uint8_t leaf;        // children are leaves
  int8_t needsScour;   // -1 undefined, 0 false, 1 true
  BId child[kMaxNodes];
};

struct HeapEnt {
  int32_t maxSeq;
  uint32_t leafId;
};

struct PropSet {
  uint32_t n;
  uint32_t kv[FMT_MT_PROPS_MAX];
};

// One live obliterate (mergeTree.ts ObliterateInfo): its endpoint references as (leaf id, offset)
// — id 0 once the reference is removed — and its stamp.
struct ObEnt {
  uint32_t startId, endId;
  int32_t startOff, endOff;
  int32_t seq, client;
};

// Per-wave LDS state (the large tier keeps its text in HBM: chars[] is then a stub).
template <class C>
struct Scratch {
  uint16_t chars[C::kHbmChars ? 2 : C::kCapChars];
  Blk<typename C::BId> blk[C::kMaxBlocks];
  HeapEnt heap[C::kHeapCap + 1];  // 1-based
  PropSet props[C::kPropCap];
  uint16_t propCls[C::kPropCap];  // match class: the first interned set with the same content (empty: 0xFFFF)
  uint32_t kvWork[FMT_MT_PROPS_KEYS_MAX];  // applyProps' working set (slot k = entry k)
  typename C::BId freeList[C::kMaxBlocks];
  uint32_t tmp[64];
  ObEnt ob[kObCap];          // slots
  uint8_t obSeq[kObCap];     // Obliterates.seqOrdered: slots in seq order
  uint8_t obStart[kObCap];   // Obliterates.startOrdered: slots in SortedSegmentSet order
};

// Leaf word fields (W0's packing is per tier, see Doc).
// W4 = leaf id (23 bits) | Marker flag << 23 | insert client << 24
constexpr uint32_t kW4Marker = 1u << 23;
constexpr uint32_t kIdLimit = 1u << 23;  // leaf ids are 23-bit: a document allocating more fails (FMT_E_CAPACITY)
FMT_DEV uint32_t fId(uint32_t w4) { return w4 & 0x7FFFFFu; }
FMT_DEV bool fMarker(uint32_t w4) { return (w4 & kW4Marker) != 0; }
FMT_DEV int32_t fClient(uint32_t w4) { return static_cast<int32_t>(static_cast<int8_t>(w4 >> 24)); }
FMT_DEV uint32_t mkW4(uint32_t id, int32_t client) { return (id & 0x7FFFFFu) | (static_cast<uint32_t>(client & 0xFF) << 24); }

struct LeafRec {
  uint32_t w[8];  // W0..W4, and W5, W6 in the large tier; W7: the local variant's pending-group count
};

struct AdjustTables;

// f4: the local client's per-document slabs (device memory), each at its offset table's entry for the
// document (nDocs + 1 entries, in records): the pending segment groups (4 words: localSeq, type |
// marker flag << 8, payload, pos2 — the op's, what acks, rollbacks and regeneration read), the group
// records (2 words: leaf id, group serial; a SegmentGroup's segments in order, a segment's groups in
// order), PropertiesManager records (4 words, Doc::pm*), the regenerated ops and their text, and a
// scratch area for segment normalization (leaf records + text of the runs it reorders).
// f4 (Doc<..., Loc = true>): per-document slabs of the local client's state, each document's at
// xOffs[doc] .. xOffs[doc + 1] (units: groups of 8 words, records of 2 words, PropertiesManager records of
// 4 words, ops, UTF-16 units, words).
struct LocalTables {
  uint32_t* groups;  // pending SegmentGroups, in queue order (Doc::groupPush)
  const uint64_t* groupOffs;
  uint32_t* recs;    // (leaf id, group serial): the segments of each group in the order they joined
  const uint64_t* recOffs;
  uint32_t* pm;
  const uint64_t* pmOffs;
  fmt_mt_op* regen;
  const uint64_t* regenOffs;
  uint16_t* regenText;
  const uint64_t* regenTextOffs;
  uint32_t* regenCount;  // per document: regenerated ops, their text units
  uint32_t* scratch;
  const uint64_t* scratchOffs;
};

struct DocInputs {
  const fmt_mt_op* ops;
  uint64_t begin, end;
  const uint16_t* text;
  uint32_t initOff, initLen;
  const uint32_t* propsOff;
  const uint32_t* propsKv;
  uint32_t nPropsOps;
  const fmt_mt_snapshot_seg* snapSegs;  // this document's summary segments (loaded != 0)
  uint32_t nHeader, nBody;
  int32_t snapMinSeq, snapSeq;
  uint32_t loaded;
  const fmt_mt_snapshot_info* snapInfo;  // SnapshotV1 merge info parallel to snapSegs, or nullptr
  const fmt_mt_stamp* snapStamps;
  // the batch's whole merge-info table (FMT_MT_F_LOADSEG ops name rows of it), or nullptr
  const fmt_mt_snapshot_info* infoAll;
  const fmt_mt_stamp* stampsAll;
  uint64_t nInfoAll;
  const fmt_mt_relpos* relpos;  // FMT_MT_F_REL1/REL2 ops index it (nullptr: none in the batch)
  uint32_t nRelpos;
  uint32_t markerKey;           // key id of "markerId"
  // annotate-adjust (nullptr: none in the batch), see Doc::adjustValue; read on demand, so the rare
  // path keeps no registers across the op loop
  const AdjustTables* adj;
  uint32_t doc;                 // this document's index (its number slab and count)
  const LocalTables* loc = nullptr;  // f4 slabs (Loc variants only)
};

struct DocOutputs {
  fmt_mt_doc_result* header;
  fmt_mt_leaf* leaves;    // kCapLeaves entries
  uint16_t* chars;        // kCapChars entries (the large tier's working text)
  fmt_mt_propset* props;  // kPropCap entries
  fmt_mt_catchup_range* catchup;  // catchupCap entries (nullptr: no FMT_MT_F_CATCHUP ops)
  uint32_t catchupCap;
  fmt_mt_remove_order* rmOrder;   // rmOrderCap entries (nullptr: no FMT_MT_F_RMORDER ops)
  uint32_t rmOrderCap;
  uint32_t* ckpt;                 // the document's tier checkpoint (kCkptWords), or nullptr
  bool ckptResume;                // resume from the checkpoint the tier below left
  // small → large tier: the small tier leaves its checkpoint in its own result slabs (leaves slab:
  // head, leaf words, scratch; chars slab: the text), where the large tier reads it
  uint32_t* bigCkpt;              // small tier: its leaves slab; large tier: the small slab to read
  uint16_t* bigCkptChars;
  // annotate-adjust batches: per leaf, the prop-set id of getAtSeq(properties, minSeq), what the legacy
  // summary reads (snapshotlegacy.ts:211-212); nullptr otherwise
  uint16_t* legacyProps;
  // large tier, plain batches: the document's large → huge checkpoint record (huge_ckpt.h), or nullptr
  uint32_t* hugeCkpt = nullptr;
};

// Diagnostic build only (FMT_PROFILE=1): per-phase shader-clock totals, see stamp().
#ifndef FMT_PROFILE
#define FMT_PROFILE 0
#endif
// Diagnostic / A-B switch: op records through scalar loads (see Doc::fetchOp).
#ifndef FMT_SCALAR_OPS
#define FMT_SCALAR_OPS 0
#endif
enum ProfCat {
  kPfOpLoad, kPfScan, kPfSplit, kPfInsert, kPfRange, kPfLru, kPfZamboniOp, kPfWindow, kPfOutput,
  kPfInsChars, kPfInsShift, kPfZFind, kPfZChars, kPfZSerial, kPfZDelete, kPfZPack, kPfCount
};

// Ob: the engine variant that also replays obliterates (f1). Without obliterates in a batch the
// runtime launches Doc<false>, whose code is exactly the obliterate-free engine.
// Rm: the variant that records the remove order for SnapshotV1 summaries (FMT_MT_F_RMORDER ops);
// batches without such ops run the Rm = false code, which has none of it.
// Adj: the variant that folds annotate-adjust entries (batches with adjusts; always with Ob, whose
// runtime path restarts overflowing documents in the next tier instead of checkpointing them).
// Loc: the local-client variant (f4, batches with FMT_MT_F_LOCAL / ACK / ROLLBACK / REGEN records):
// local stamps, pending segment groups, acks, rollbacks and regeneration (large tier only).
template <bool Ob, class C = SmallTier, bool Rm = false, bool Adj = false, bool Loc = false>
class Doc {
 public:
  using VR = typename C::VR;
  using BId = typename C::BId;
  static constexpr int kRows = C::kRows;
  static constexpr int kRowUnroll = C::kUnroll ? C::kRows : 1;
  static constexpr int kCapLeaves = 64 * kRows;
  static constexpr int kCapChars = C::kCapChars;
  static constexpr int kMaxBlocks = C::kMaxBlocks;
  static constexpr int kHeapCap = C::kHeapCap;
  static constexpr int kPropCap = C::kPropCap;
  static constexpr uint32_t kLenMask = (1u << C::kLenBits) - 1u;
  static constexpr uint32_t kNoBlk = (1u << C::kBlkBits) - 1u;
  static constexpr bool kPW = C::kPropsWord;
  // A limit both tiers share (keys per prop set, catch-up / remove-order slabs, live obliterates):
  // the small tier reports it as kCapacityFinal so that the overflow list does not replay the
  // document in the large tier only to fail again; collectOverflowKernel turns it into
  // FMT_E_CAPACITY. Every other capacity failure of the small tier escalates.
  static constexpr int kCapFinal = C::kHbmChars ? FMT_E_CAPACITY : kCapacityFinal;
  static constexpr uint32_t kPropsUndef = kPW ? 0xFFFFu : (1u << (32 - C::kLenBits - C::kBlkBits)) - 1u;
  static_assert(kMaxBlocks <= static_cast<int>(kNoBlk) && kPropCap <= static_cast<int>(kPropsUndef), "W0 field widths");
  static_assert(kRows <= 32, "row bitmasks are 32-bit");
  FMT_DEV static uint32_t fLen(uint32_t w0) { return w0 & kLenMask; }
  FMT_DEV static uint32_t fBlk(uint32_t w0) { return (w0 >> C::kLenBits) & kNoBlk; }
  // (large tier: W0 holds no props; mkW0 ignores them and W6 keeps them)
  FMT_DEV static uint32_t fProps(uint32_t w0) { return kPW ? 0u : w0 >> (C::kLenBits + C::kBlkBits); }
  FMT_DEV static uint32_t mkW0(uint32_t len, uint32_t blk, uint32_t props) {
    return kPW ? len | (blk << C::kLenBits) : len | (blk << C::kLenBits) | (props << (C::kLenBits + C::kBlkBits));
  }

#if FMT_PROFILE && FMT_GPU
  uint64_t profT = 0;
  uint64_t prof[kPfCount] = {};
  FMT_DEV void stamp(int cat) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    prof[cat] += t - profT;
    profT = t;
  }
#else
  FMT_DEV void stamp(int) {}
#endif
  // Loc (f4): one more leaf word, W[kPendW] = the number of the local client's pending segment groups
  // holding the leaf (segmentGroupCollection.ts); the prop-set word stays W[kPropW]
  static constexpr int kWords = C::kWords + (Loc ? 1 : 0);
  static constexpr int kPropW = C::kWords - 1;
  static constexpr int kPendW = C::kWords;
  static constexpr int kMaxClient = C::kMaxClient;
  static constexpr int kTopClient = 253;  // the huge tier's writer ceiling (huge_engine.h kMaxClient)
  Lane<VR> W[kWords];  // W[f] element r of lane l = field f of leaf 64 r + l
  FMT_LDS Scratch<C>* s;  // (an LDS-space pointer: per-lane LDS addresses stay 32-bit)
  uint16_t* gch = nullptr;  // large tier: the document's text, in its HBM output slab
  int n = 0;          // leaves
  int nChars = 0;
  int root = 0;
  int nFree = 0;
  int heapN = 0;
  int nProps = 0;
  int curSeq = 0;
  int minSeq = 0;
  int status = FMT_OK;
  int failSeq = 0;
  uint32_t nextId = 1;
  uint32_t opIdx = 0;   // index of the current op within the document
  int obSeqN = 0;       // live obliterates (seqOrdered length)
  int obStartN = 0;     // startOrdered length (can exceed obSeqN: a failed SortedSet.remove)
  uint64_t obUsed = 0;  // slot bitmap
  uint32_t cuN = 0;     // catch-up ranges recorded
  DocInputs in;
  fmt_mt_catchup_range* cuOut = nullptr;
  uint32_t cuCap = 0;
  uint32_t rmN = 0;     // remove-order entries recorded (HBM slab, leaf ids until writeOutputs)
  fmt_mt_remove_order* rmOut = nullptr;
  uint32_t rmCap = 0;
  int rmPendN = 0;      // split copies waiting for rmFlush (at most two splits per op)
  uint32_t rmPendFrom0 = 0, rmPendTo0 = 0, rmPendFrom1 = 0, rmPendTo1 = 0;
  bool rmHitsSet = false;
  Lane<uint32_t> rmHits;  // leaves a flagged REMOVE found already removed (row bitmask per lane)

  // ------------------------------------------------------------------ tier checkpoint
  // A document without remove-order recording in the compact tier that is about to outgrow its 4
  // register rows stops before the op (one op adds at most two leaves: an insert's split plus the
  // new leaf, or a range op's — obliterate's too — two boundary splits) and leaves its whole state
  // in its HBM checkpoint: the scalars, the leaf words of the compact rows and the LDS scratch (same
  // layout in both tiers). The small tier resumes it from that op instead of replaying it from its
  // first op.
  static constexpr bool kSavesCkpt = !C::kHbmChars && C::kRows < SmallTier::kRows && !Rm && !Loc;
  static constexpr bool kResumesCkpt = !C::kHbmChars && C::kRows == SmallTier::kRows && !Rm && !Loc;
  // layout: 16 head words | leaf words of the compact rows | the compact tier's chars | the rest of
  // the scratch (blk .. tmp: the same fields in both tiers; only the chars array differs in size) |
  // the live obliterates (ob .. obStart; Ob only, head words 13..15 hold their counts and bitmap)
  static constexpr int kCkptRows = CompactTier::kRows;
  static constexpr int kCkptHead = 16;
  static constexpr int kCkptCharWords = CompactTier::kCapChars / 2;
  static constexpr int kCkptRestWords =
      static_cast<int>((offsetof(Scratch<CompactTier>, tmp) - offsetof(Scratch<CompactTier>, blk) + 3) / 4);
  static_assert(offsetof(Scratch<CompactTier>, tmp) - offsetof(Scratch<CompactTier>, blk) ==
                    offsetof(Scratch<SmallTier>, tmp) - offsetof(Scratch<SmallTier>, blk),
                "checkpointed scratch fields");
  static constexpr int kCkptObWords =
      static_cast<int>((offsetof(Scratch<CompactTier>, obStart) + kObCap - offsetof(Scratch<CompactTier>, ob) + 3) / 4);
  static_assert(offsetof(Scratch<CompactTier>, obStart) - offsetof(Scratch<CompactTier>, ob) ==
                    offsetof(Scratch<SmallTier>, obStart) - offsetof(Scratch<SmallTier>, ob),
                "checkpointed obliterate fields");
  static constexpr int kCkptWords = kCkptHead + 5 * kCkptRows * 64 + kCkptCharWords + kCkptRestWords + kCkptObWords;
  uint32_t* ckpt = nullptr;
  uint64_t ckptNext = 0;  // the op a tier checkpoint resumes at

  // small → large (plain batches): the small tier stops before an op that could outgrow its 512
  // leaves or 6144 units, or that comes from a writer past its 31; the large tier converts its state
  // (W0 packing and 8-bit block ids of the small tier, text into the HBM slab).
  // (Ob: the live-obliterate table goes to the end of the document's compact checkpoint slot, free
  // once the small tier has resumed from it; head words 13..15 of the slab hold its counts and bitmap)
  static constexpr bool kSavesBig = !C::kHbmChars && C::kRows == SmallTier::kRows && !Rm && !Loc;
  static constexpr bool kResumesBig = C::kHbmChars && !Rm && !Loc;
  static constexpr int kCkptObOff = kCkptWords - kCkptObWords;
  static constexpr int kBigRows = SmallTier::kRows;
  static constexpr int kBigRestWords =
      static_cast<int>((offsetof(Scratch<SmallTier>, tmp) - offsetof(Scratch<SmallTier>, blk) + 3) / 4);
  static_assert(kCkptHead + 5 * kBigRows * 64 + kBigRestWords <= 64 * SmallTier::kRows * 8,
                "the small tier's checkpoint fits its leaves slab");
  uint32_t* bigCkpt = nullptr;
  uint16_t* bigCkptChars = nullptr;

  // large → huge (round 5; huge_ckpt.h): a plain document the large tier is about to outgrow stops
  // before the op, writes its result slabs and the checkpoint record, and the huge tier replays on
  // from that op with the same tree.
  // (annotate-adjust and remove-order documents too: their PropertiesManager records, computed
  // numbers and remove-order entries stay in the batch's HBM slabs, which the huge tier reads with the
  // same layout; the record carries pmN and rmN, the entries keep their leaf ids)
  static constexpr bool kSavesHuge = C::kHbmChars && !Loc;
  uint32_t* hugeCkpt = nullptr;
  bool savingHuge = false;  // (writeOutputs: no legacy getAtSeq view, it would mark the records; no
                            // remove-order index conversion)
  FMT_DEV void saveHuge(uint64_t next) {
    namespace K = fmt_ckpt;
    uint32_t* ck = hugeCkpt;
    FOR_LANES(l) {
      if (l == 0) {
        ck[K::kNextLo] = static_cast<uint32_t>(next);
        ck[K::kNextHi] = static_cast<uint32_t>(next >> 32);
        ck[K::kN] = static_cast<uint32_t>(n);
        ck[K::kNChars] = static_cast<uint32_t>(nChars);
        ck[K::kRoot] = static_cast<uint32_t>(root);
        ck[K::kNFree] = static_cast<uint32_t>(nFree);
        ck[K::kHeapN] = static_cast<uint32_t>(heapN);
        ck[K::kNProps] = static_cast<uint32_t>(nProps);
        ck[K::kCurSeq] = static_cast<uint32_t>(curSeq);
        ck[K::kMinSeq] = static_cast<uint32_t>(minSeq);
        ck[K::kNextId] = nextId;
        ck[K::kCuN] = cuN;
        ck[K::kObCounts] = Ob ? static_cast<uint32_t>(obSeqN) | (static_cast<uint32_t>(obStartN) << 16) : 0u;
        ck[K::kObUsedLo] = Ob ? static_cast<uint32_t>(obUsed) : 0u;
        ck[K::kObUsedHi] = Ob ? static_cast<uint32_t>(obUsed >> 32) : 0u;
        ck[K::kPmN] = Adj ? static_cast<uint32_t>(pmN) : 0u;
        ck[K::kRmN] = Rm ? rmN : 0u;
      }
    }
    static_assert(!kSavesHuge || (kCapLeaves == K::kLeaves && kMaxBlocks == K::kBlocks && kHeapCap + 1 == K::kHeap &&
                                  kObCap == K::kObSlots), "huge_ckpt.h layout");
    const int nr = rows();
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        const int j = r * 64 + l;
        if (j < n) {
          ck[K::kLeafW4 + j] = LANE(W[4])[r];
          ck[K::kLeafBlk + j] = fBlk(LANE(W[0])[r]);
        }
      }
    }
    FOR_LANES(l) {
      for (int b = l; b < kMaxBlocks; b += 64) {
        const Blk<BId> k = s->blk[b];
        uint32_t* o = ck + K::kBlk + K::kBlkWords * b;
        o[0] = static_cast<uint32_t>(k.count) | (static_cast<uint32_t>(k.leaf) << 8) |
               (static_cast<uint32_t>(static_cast<uint8_t>(k.needsScour)) << 16);
        o[1] = static_cast<uint32_t>(k.parent) == kNoBlk ? K::kNoParent : static_cast<uint32_t>(k.parent);
        for (int c = 0; c < kMaxNodes; c++) o[2 + c] = static_cast<uint32_t>(k.child[c]);
      }
      for (int k = l; k <= heapN; k += 64) {
        ck[K::kHeapOff + 2 * k] = static_cast<uint32_t>(s->heap[k].maxSeq);
        ck[K::kHeapOff + 2 * k + 1] = s->heap[k].leafId;
      }
      for (int k = l; k < nFree; k += 64) ck[K::kFree + k] = static_cast<uint32_t>(s->freeList[k]);
      if constexpr (Ob) {
        for (int k = l; k < kObCap; k += 64) {
          const ObEnt e = s->ob[k];
          uint32_t* o = ck + K::kOb + 6 * k;
          o[0] = e.startId;
          o[1] = e.endId;
          o[2] = static_cast<uint32_t>(e.startOff);
          o[3] = static_cast<uint32_t>(e.endOff);
          o[4] = static_cast<uint32_t>(e.seq);
          o[5] = static_cast<uint32_t>(e.client);
          ck[K::kObSeq + k] = s->obSeq[k];
          ck[K::kObStart + k] = s->obStart[k];
        }
      }
    }
    waveSync();
  }

  FMT_DEV void saveBig(uint64_t next) {
    uint32_t* ck = bigCkpt;
    FOR_LANES(l) {
      if (l == 0) {
        ck[0] = static_cast<uint32_t>(next);
        ck[1] = static_cast<uint32_t>(next >> 32);
        ck[2] = static_cast<uint32_t>(n);
        ck[3] = static_cast<uint32_t>(nChars);
        ck[4] = static_cast<uint32_t>(root);
        ck[5] = static_cast<uint32_t>(nFree);
        ck[6] = static_cast<uint32_t>(heapN);
        ck[7] = static_cast<uint32_t>(nProps);
        ck[8] = static_cast<uint32_t>(curSeq);
        ck[9] = static_cast<uint32_t>(minSeq);
        ck[10] = static_cast<uint32_t>(failSeq);
        ck[11] = nextId;
        ck[12] = cuN;
        if constexpr (Ob) {
          ck[13] = static_cast<uint32_t>(obSeqN) | (static_cast<uint32_t>(obStartN) << 16);
          ck[14] = static_cast<uint32_t>(obUsed);
          ck[15] = static_cast<uint32_t>(obUsed >> 32);
        }
      }
    }
    if constexpr (Ob) {
      const uint32_t* obw = reinterpret_cast<const FMT_LDS uint32_t*>(s->ob);
      FOR_LANES(l) {
        for (int t = l; t < kCkptObWords; t += 64) ckpt[kCkptObOff + t] = obw[t];
      }
    }
    FOR_LANES(l) {
#pragma unroll
      for (int f = 0; f < 5; f++) {
#pragma unroll
        for (int r = 0; r < kBigRows && r < kRows; r++) ck[kCkptHead + (f * kBigRows + r) * 64 + l] = LANE(W[f])[r];
      }
    }
    waveSync();
    const uint32_t* rest = reinterpret_cast<const uint32_t*>(reinterpret_cast<const unsigned char*>(s) + offsetof(Scratch<C>, blk));
    uint32_t* dst = ck + kCkptHead + 5 * kBigRows * 64;
    FOR_LANES(l) {
      for (int t = l; t < kBigRestWords; t += 64) dst[t] = rest[t];
      if constexpr (!C::kHbmChars)
        for (int t = l; t < nChars; t += 64) bigCkptChars[t] = s->chars[t];
    }
  }

  // The large tier takes over a document the small tier checkpointed. Returns the op to resume at.
  FMT_DEV uint64_t restoreBig() {
    const uint32_t* ck = bigCkpt;
    const uint64_t next = uni(ck[0]) | (static_cast<uint64_t>(uni(ck[1])) << 32);
    n = static_cast<int>(uni(ck[2]));
    nChars = static_cast<int>(uni(ck[3]));
    root = static_cast<int>(uni(ck[4]));
    const int smallFree = static_cast<int>(uni(ck[5]));
    heapN = static_cast<int>(uni(ck[6]));
    nProps = static_cast<int>(uni(ck[7]));
    curSeq = static_cast<int>(uni(ck[8]));
    minSeq = static_cast<int>(uni(ck[9]));
    failSeq = static_cast<int>(uni(ck[10]));
    nextId = uni(ck[11]);
    cuN = uni(ck[12]);
    if constexpr (Ob) {
      const uint32_t c13 = uni(ck[13]);
      obSeqN = static_cast<int>(c13 & 0xFFFFu);
      obStartN = static_cast<int>(c13 >> 16);
      obUsed = uni(ck[14]) | (static_cast<uint64_t>(uni(ck[15])) << 32);
      uint32_t* obw = reinterpret_cast<FMT_LDS uint32_t*>(s->ob);
      FOR_LANES(l) {
        for (int t = l; t < kCkptObWords; t += 64) obw[t] = ckpt[kCkptObOff + t];
      }
    }
    status = FMT_OK;
    // small-tier W0 = len (16 bits) | block (8) | props (8, 255 undefined)
    constexpr uint32_t kSmallNoProps = 255u, kSmallNoBlk = 255u;
    FOR_ROWS(r, 0, kRows) {
      FOR_LANES(l) {
        uint32_t w[5] = {0u, 0u, 0u, 0u, 0u};
        if (r < kBigRows)
          for (int f = 0; f < 5; f++) w[f] = ck[kCkptHead + (f * kBigRows + r) * 64 + l];
        const bool live = r * 64 + l < n;
        const uint32_t sp = w[0] >> 24;
        LANE(W[0])[r] = live ? mkW0(w[0] & 0xFFFFu, (w[0] >> 16) & 0xFFu, 0u) : 0u;
        LANE(W[1])[r] = w[1];
        LANE(W[2])[r] = w[2];
        LANE(W[3])[r] = w[3];
        LANE(W[4])[r] = w[4];
        if constexpr (C::kWords > 5) {
          LANE(W[5])[r] = 0u;
          LANE(W[kPropW])[r] = live ? (sp == kSmallNoProps ? kPropsUndef : sp) : 0u;
        }
      }
    }
    // the small scratch image from its blk field on: blocks, heap, prop sets, match classes, free list
    const unsigned char* img = reinterpret_cast<const unsigned char*>(ck + kCkptHead + 5 * kBigRows * 64) -
                               offsetof(Scratch<SmallTier>, blk);
    const Scratch<SmallTier>* sm = reinterpret_cast<const Scratch<SmallTier>*>(img);
    const auto blkId = [&](uint32_t b) -> BId { return static_cast<BId>(b == kSmallNoBlk ? kNoBlk : b); };
    FOR_LANES(l) {
      for (int b = l; b < SmallTier::kMaxBlocks; b += 64) {
        const Blk<uint8_t> src = sm->blk[b];
        Blk<BId>& d = s->blk[b];
        d.count = src.count;
        d.parent = blkId(src.parent);
        d.leaf = src.leaf;
        d.needsScour = src.needsScour;
        for (int c = 0; c < kMaxNodes; c++) d.child[c] = blkId(src.child[c]);
      }
      for (int k = l; k <= heapN; k += 64) s->heap[k] = sm->heap[k];
      for (int k = l; k < nProps; k += 64) {
        s->props[k] = sm->props[k];
        s->propCls[k] = sm->propCls[k];
      }
      // free list: the ids the small tier never had at the bottom, its own free ids on top (popped first)
      const int extra = kMaxBlocks - SmallTier::kMaxBlocks;
      for (int k = l; k < extra; k += 64) s->freeList[k] = static_cast<BId>(kMaxBlocks - 1 - k);
      for (int k = l; k < smallFree; k += 64) s->freeList[extra + k] = static_cast<BId>(sm->freeList[k]);
      if constexpr (C::kHbmChars)
        for (int t = l; t < nChars; t += 64) gch[t] = bigCkptChars[t];
    }
    nFree = kMaxBlocks - SmallTier::kMaxBlocks + smallFree;
    waveSync();
    return next;
  }

  FMT_DEV void saveCkpt(uint64_t next) {
    uint32_t* ck = ckpt;
    FOR_LANES(l) {
      if (l == 0) {
        ck[0] = static_cast<uint32_t>(next);
        ck[1] = static_cast<uint32_t>(next >> 32);
        ck[2] = static_cast<uint32_t>(n);
        ck[3] = static_cast<uint32_t>(nChars);
        ck[4] = static_cast<uint32_t>(root);
        ck[5] = static_cast<uint32_t>(nFree);
        ck[6] = static_cast<uint32_t>(heapN);
        ck[7] = static_cast<uint32_t>(nProps);
        ck[8] = static_cast<uint32_t>(curSeq);
        ck[9] = static_cast<uint32_t>(minSeq);
        ck[10] = static_cast<uint32_t>(failSeq);
        ck[11] = nextId;
        ck[12] = cuN;
        if constexpr (Ob) {
          ck[13] = static_cast<uint32_t>(obSeqN) | (static_cast<uint32_t>(obStartN) << 16);
          ck[14] = static_cast<uint32_t>(obUsed);
          ck[15] = static_cast<uint32_t>(obUsed >> 32);
        }
      }
    }
    FOR_LANES(l) {
#pragma unroll
      for (int f = 0; f < 5; f++) {
#pragma unroll
        for (int r = 0; r < kCkptRows && r < kRows; r++) ck[kCkptHead + (f * kCkptRows + r) * 64 + l] = LANE(W[f])[r];
      }
    }
    waveSync();  // every LDS write of the op stream has landed
    const uint32_t* chars = reinterpret_cast<const FMT_LDS uint32_t*>(s->chars);
    const uint32_t* rest = reinterpret_cast<const uint32_t*>(reinterpret_cast<const unsigned char*>(s) + offsetof(Scratch<C>, blk));
    uint32_t* dst = ck + kCkptHead + 5 * kCkptRows * 64;
    const int charWords = (nChars + 1) / 2;
    FOR_LANES(l) {
      for (int t = l; t < charWords; t += 64) dst[t] = chars[t];
      for (int t = l; t < kCkptRestWords; t += 64) dst[kCkptCharWords + t] = rest[t];
    }
    if constexpr (Ob) {
      const uint32_t* obw = reinterpret_cast<const FMT_LDS uint32_t*>(s->ob);
      FOR_LANES(l) {
        for (int t = l; t < kCkptObWords; t += 64) dst[kCkptCharWords + kCkptRestWords + t] = obw[t];
      }
    }
  }

  // Returns the op index to resume at.
  FMT_DEV uint64_t restoreCkpt() {
    const uint32_t* ck = ckpt;
    const uint64_t next = uni(ck[0]) | (static_cast<uint64_t>(uni(ck[1])) << 32);
    n = static_cast<int>(uni(ck[2]));
    nChars = static_cast<int>(uni(ck[3]));
    root = static_cast<int>(uni(ck[4]));
    nFree = static_cast<int>(uni(ck[5]));
    heapN = static_cast<int>(uni(ck[6]));
    nProps = static_cast<int>(uni(ck[7]));
    curSeq = static_cast<int>(uni(ck[8]));
    minSeq = static_cast<int>(uni(ck[9]));
    failSeq = static_cast<int>(uni(ck[10]));
    nextId = uni(ck[11]);
    cuN = uni(ck[12]);
    if constexpr (Ob) {
      const uint32_t c13 = uni(ck[13]);
      obSeqN = static_cast<int>(c13 & 0xFFFFu);
      obStartN = static_cast<int>(c13 >> 16);
      obUsed = uni(ck[14]) | (static_cast<uint64_t>(uni(ck[15])) << 32);
    }
    status = FMT_OK;
    FOR_LANES(l) {
#pragma unroll
      for (int f = 0; f < 5; f++) {
        VR z;
#pragma unroll
        for (int r = 0; r < kRows; r++) z[r] = r < kCkptRows ? ck[kCkptHead + (f * kCkptRows + r) * 64 + l] : 0u;
        LANE(W[f]) = z;
      }
    }
    const uint32_t* src = ck + kCkptHead + 5 * kCkptRows * 64;
    uint32_t* chars = reinterpret_cast<FMT_LDS uint32_t*>(s->chars);
    uint32_t* rest = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(s) + offsetof(Scratch<C>, blk));
    const int charWords = (nChars + 1) / 2;
    FOR_LANES(l) {
      for (int t = l; t < charWords; t += 64) chars[t] = src[t];
      for (int t = l; t < kCkptRestWords; t += 64) rest[t] = src[kCkptCharWords + t];
    }
    if constexpr (Ob) {
      uint32_t* obw = reinterpret_cast<FMT_LDS uint32_t*>(s->ob);
      FOR_LANES(l) {
        for (int t = l; t < kCkptObWords; t += 64) obw[t] = src[kCkptCharWords + kCkptRestWords + t];
      }
    }
    waveSync();
    return next;
  }

  // ------------------------------------------------------------------ leaf array primitives
  // Leaf j lives in row j >> 6 (element of the V8) of lane j & 63: document order runs along a
  // row's lanes, then to the next row. Rows at or above rows() hold only empty (all-zero) slots,
  // and every pass below visits rows [0, rows()) only, so its cost follows the live leaf count.
  FMT_DEV int rows() const { return (n + 63) >> 6; }

  FMT_DEV static Lane<uint32_t> row(const Lane<VR>& a, int r) {  // r compile-time after unrolling
    Lane<uint32_t> x;
    FOR_LANES(l) { LANE(x) = LANE(a)[r]; }
    return x;
  }

  FMT_DEV static Lane<uint32_t> selectRow(const Lane<VR>& arr, int r) {  // r wave-uniform, dynamic
    Lane<uint32_t> x;
    FOR_LANES(l) {
      if constexpr (C::kUnroll) {
        VR t = LANE(arr);
        launder(t);  // keep the dynamic index on a register value (v_movrels), never a scratch GEP
        LANE(x) = t[r];
      } else {
        LANE(x) = LANE(arr)[r];
      }
    }
    return x;
  }

  FMT_DEV uint32_t readField(int j, int f) const { return readlane(selectRow(W[f], j >> 6), j & 63); }

  // Prop-set id of leaf j / of leaf 64 r + l inside a FOR_LANES body, and setting it.
  FMT_DEV uint32_t propsAt(int j) const {
    if constexpr (kPW) return readField(j, kPropW);
    else return fProps(readField(j, 0));
  }
  FMT_DEV uint32_t propsL(int l, int r) const {
    if constexpr (kPW) return LANE(W[kPropW])[r];
    else return fProps(LANE(W[0])[r]);
  }
  FMT_DEV void setPropsL(int l, int r, uint32_t p) {
    if constexpr (kPW) {
      LANE(W[kPropW])[r] = p;
    } else {
      const uint32_t w0 = LANE(W[0])[r];
      LANE(W[0])[r] = mkW0(fLen(w0), fBlk(w0), p);
    }
  }

  FMT_DEV LeafRec readLeaf(int j) const {
    LeafRec r;
#pragma unroll
    for (int f = 0; f < kWords; f++) r.w[f] = readField(j, f);
    return r;
  }

  FMT_DEV void writeField(int j, int f, uint32_t v) {
    const int rj = j >> 6, lane = j & 63;
    FOR_ROWS(r, rj, rj + 1) {
      FOR_LANES(l) {
        if (l == lane) LANE(W[f])[r] = v;
      }
    }
  }

  // Insert `rec` at index k: rows from k's row up are shifted one lane up (DPP wave_shr), each
  // row's lane 0 taking the previous row's lane 63. Top-down, so that carry is still the old value.
  FMT_DEV bool insertLeafAt(int k, const LeafRec& rec) {
    if (n >= kCapLeaves) return fail(FMT_E_CAPACITY);
    const int rk = k >> 6, kl = k & 63, nr = (n + 64) >> 6;
    FOR_ROWS_DOWN(r, rk, nr) {
#pragma unroll
      for (int f = 0; f < kWords; f++) {
        const Lane<uint32_t> cur = row(W[f], r);
        const Lane<uint32_t> up = shflUp1(cur);
        if (r > rk) {
          const uint32_t carry = readlane(row(W[f], r > 0 ? r - 1 : 0), 63);
          FOR_LANES(l) { LANE(W[f])[r] = l == 0 ? carry : LANE(up); }
        } else {
          const uint32_t rv = rec.w[f];
          FOR_LANES(l) { LANE(W[f])[r] = l > kl ? LANE(up) : (l == kl ? rv : LANE(cur)); }
        }
      }
    }
    n++;
    return true;
  }

  // Remove the leaf at index k: rows from k's row up shift one lane down (DPP wave_shl), lane 63
  // taking the next row's lane 0 (zero past the last row, which keeps empty slots zero).
  FMT_DEV void deleteLeafAt(int k) {
    const int rk = k >> 6, kl = k & 63, nr = rows();
    FOR_ROWS(r, rk, nr) {
#pragma unroll
      for (int f = 0; f < kWords; f++) {
        const Lane<uint32_t> cur = row(W[f], r);
        const Lane<uint32_t> dn = shflDown1(cur);
        const uint32_t carry = r + 1 < nr ? readlane(row(W[f], r + 1 < kRows ? r + 1 : r), 0) : 0u;
        if (r > rk) {
          FOR_LANES(l) { LANE(W[f])[r] = l == 63 ? carry : LANE(dn); }
        } else {
          FOR_LANES(l) { LANE(W[f])[r] = l < kl ? LANE(cur) : (l == 63 ? carry : LANE(dn)); }
        }
      }
    }
    n--;
  }

  // Delete the leaves first + k for every bit k < cnt of `dead` in one pass: leaf i of the result
  // comes from the (i - first)-th surviving leaf of the block, or from i + d after it (d = deleted
  // count <= 7, so from the same row or the next). Empty slots past the new end stay zero.
  FMT_DEV void deleteLeaves(int first, int cnt, uint32_t dead) {
    const int d = __builtin_popcount(dead);
    if (d == 0) return;
    const int nr = rows(), nNew = n - d, keptEnd = first + cnt - d;
    FOR_ROWS(r, first >> 6, nr) {
      Lane<int> src;
      Lane<bool> fromNext, live;
      FOR_LANES(l) {
        const int i = r * 64 + l;
        int from = i + d;
        if (i < first) {
          from = i;
        } else if (i < keptEnd) {
          int seen = 0;
#pragma unroll
          for (int k = 0; k < kMaxNodes; k++) {
            if (k < cnt && ((dead >> k) & 1u) == 0) {
              if (seen == i - first) from = first + k;
              seen++;
            }
          }
        }
        LANE(src) = from & 63;
        LANE(fromNext) = (from >> 6) > r;
        LANE(live) = i < nNew;
      }
#pragma unroll
      for (int f = 0; f < kWords; f++) {
        const Lane<uint32_t> a = gather(row(W[f], r), src);
        const Lane<uint32_t> b = gather(row(W[f], r + 1 < kRows ? r + 1 : r), src);
        FOR_LANES(l) { LANE(W[f])[r] = LANE(live) ? (LANE(fromNext) && r + 1 < kRows ? LANE(b) : LANE(a)) : 0u; }
      }
    }
    n = nNew;
  }

  // Exclusive prefix (document order) of per-leaf values over rows [0, nr); returns the total.
  // Rows >= nr of `excl` are left unset.
  FMT_DEV static uint32_t scanRows(const Lane<VR>& vals, Lane<VR>& excl, int nr) {
    uint32_t base = 0;
    FOR_ROWS(r, 0, nr) {
      uint32_t tot;
      const Lane<uint32_t> ex = waveExclusiveSum(row(vals, r), &tot);
      FOR_LANES(l) { LANE(excl)[r] = LANE(ex) + base; }
      base += tot;
    }
    return base;
  }

  // Whether `client` holds a remove stamp on leaf 64 r + l (the remove-client set: W3, plus W5 for
  // ids 32..63 in the large tier).
  FMT_DEV bool removedBy(int l, int r, int client) const {
    if (client < 0) return false;  // NonCollabClient / LocalClientId never hold a remove stamp here
    if constexpr (C::kWords > 5) {
      if (client >= 32) return ((LANE(W[5])[r] >> (client - 32)) & 1u) != 0;
    }
    return ((LANE(W[3])[r] >> client) & 1u) != 0;
  }

  // Visible length of every leaf from PriorPerspective(refSeq, client) (perspective.ts:80-93).
  // Leaves removed at/below minSeq are never present for such a perspective (refSeq >= minSeq).
  // Empty slots have length 0.
  FMT_DEV void visLengths(int refSeq, int client, Lane<VR>& vis, int nr) const {
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        const uint32_t w0 = LANE(W[0])[r];
        const int32_t ins = static_cast<int32_t>(LANE(W[1])[r]);
        const int32_t rm = static_cast<int32_t>(LANE(W[2])[r]);
        const int32_t ic = fClient(LANE(W[4])[r]);
        const bool present = (ins <= refSeq || ic == client) && !(rm <= refSeq || removedBy(l, r, client));
        LANE(vis)[r] = present ? fLen(w0) : 0u;
      }
    }
  }

  // Char offset of every leaf (all leaves, tombstones included).
  FMT_DEV void charStarts(Lane<VR>& cst, int nr) const {
    Lane<VR> lens;
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) { LANE(lens)[r] = fLen(LANE(W[0])[r]); }
    }
    scanRows(lens, cst, nr);
  }

  // Char offset of leaf j: the lengths of the leaves before it, summed per lane over the rows and
  // then once across the wave (no per-row scans).
  FMT_DEV uint32_t charOffsetOf(int j) const {
    if (j >= n) return static_cast<uint32_t>(nChars);
    Lane<uint32_t> acc;
    FOR_LANES(l) { LANE(acc) = 0u; }
    FOR_ROWS(r, 0, (j >> 6) + 1) {
      FOR_LANES(l) {
        if (r * 64 + l < j) LANE(acc) += fLen(LANE(W[0])[r]);
      }
    }
    uint32_t total;
    waveExclusiveSum(acc, &total);
    return total;
  }

  FMT_DEV uint32_t charStartOf(int j) const {
    if (j >= n) return static_cast<uint32_t>(nChars);
    Lane<VR> cst;
    charStarts(cst, (j >> 6) + 1);
    return readlane(selectRow(cst, j >> 6), j & 63);
  }

  // First leaf (document order) whose row bit is set in a per-lane row bitmask, or -1.
  FMT_DEV static int firstSet(const Lane<uint32_t>& bits, int nr) {
    FOR_ROWS(r, 0, nr) {
      Lane<bool> p;
      FOR_LANES(l) { LANE(p) = ((LANE(bits) >> r) & 1u) != 0; }
      const uint64_t m = ballot(p);
      if (m != 0) return r * 64 + ctz64(m);
    }
    return -1;
  }

  // First leaf index with block id b (leaf blocks are contiguous runs), or -1.
  FMT_DEV int firstLeafOf(uint32_t b) const {
    const int nr = rows();
    FOR_ROWS(r, 0, nr) {
      Lane<bool> p;
      FOR_LANES(l) { LANE(p) = r * 64 + l < n && fBlk(LANE(W[0])[r]) == b; }
      const uint64_t m = ballot(p);
      if (m != 0) return r * 64 + ctz64(m);
    }
    return -1;
  }

  FMT_DEV int findLeafById(uint32_t id) const {  // ids start at 1, so empty slots never match
    const int nr = rows();
    FOR_ROWS(r, 0, nr) {
      Lane<bool> p;
      FOR_LANES(l) { LANE(p) = fId(LANE(W[4])[r]) == id; }
      const uint64_t m = ballot(p);
      if (m != 0) return r * 64 + ctz64(m);
    }
    return -1;
  }

  // ------------------------------------------------------------------ chars (doc order)
  // Small tier: LDS. Large tier: the document's HBM output slab (written by this wave only).
  FMT_DEV uint32_t chRead(int i) const {
    if constexpr (C::kHbmChars) return loadCoherent(gch + i);
    else return s->chars[i];
  }
  FMT_DEV void chWrite(int i, uint32_t v) {
    if constexpr (C::kHbmChars) gch[i] = static_cast<uint16_t>(v);
    else s->chars[i] = static_cast<uint16_t>(v);
  }

  FMT_DEV void charsShiftUp(int from, int by) {  // chars[from..nChars) → chars[from+by..)
    const int count = nChars - from;
    for (int top = count - 1; top >= 0; top -= 64) {
      Lane<uint32_t> v;
      FOR_LANES(l) {
        const int t = top - l;
        LANE(v) = t >= 0 ? chRead(from + t) : 0u;
      }
      waveSync();
      FOR_LANES(l) {
        const int t = top - l;
        if (t >= 0) chWrite(from + t + by, LANE(v));
      }
      waveSync();
    }
  }

  FMT_DEV void charsShiftDown(int from, int by) {  // chars[from..nChars) → chars[from-by..)
    for (int base = from; base < nChars; base += 64) {
      Lane<uint32_t> v;
      FOR_LANES(l) {
        const int t = base + l;
        LANE(v) = t < nChars ? chRead(t) : 0u;
      }
      waveSync();
      FOR_LANES(l) {
        const int t = base + l;
        if (t < nChars) chWrite(t - by, LANE(v));
      }
      waveSync();
    }
  }

  // ------------------------------------------------------------------ status
  FMT_DEV bool fail(int code) {
    if (status == FMT_OK) status = code;
    return false;
  }

  // ------------------------------------------------------------------ blocks
  FMT_DEV int allocBlk(uint8_t leafType) {
    if (nFree == 0) {
      fail(FMT_E_CAPACITY);
      return -1;
    }
    const int id = s->freeList[--nFree];
    auto& b = s->blk[id];
    b.count = 0;
    b.parent = kNoBlk;
    b.leaf = leafType;
    b.needsScour = -1;
    waveSync();
    return id;
  }

  FMT_DEV void freeBlk(int id) {
    s->freeList[nFree++] = static_cast<BId>(id);
    waveSync();
  }

  // Re-tag leaves [first, first+count) with block id b.
  FMT_DEV void tagLeaves(int first, int count, uint32_t b) {
    if (count <= 0) return;
    const int r0 = first >> 6, r1 = ((first + count - 1) >> 6) + 1;
    FOR_ROWS(r, r0, r1) {
      FOR_LANES(l) {
        const int idx = r * 64 + l;
        if (idx >= first && idx < first + count) {
          const uint32_t w0 = LANE(W[0])[r];
          LANE(W[0])[r] = mkW0(fLen(w0), b, fProps(w0));
        }
      }
    }
  }

  // A child was inserted into block b; split on overflow and propagate (mergeTree.ts:1946-1987,
  // root growth :1313-1320). The new right half always gets needsScour = undefined.
  FMT_DEV void childAdded(int b) {
    int cnt = uni(static_cast<int>(s->blk[b].count)) + 1;
    s->blk[b].count = static_cast<uint8_t>(cnt);
    waveSync();
    while (cnt >= kMaxNodes) {
      const int leafType = uni(static_cast<int>(s->blk[b].leaf));
      const int nb = allocBlk(static_cast<uint8_t>(leafType));
      if (nb < 0) return;
      constexpr int half = kMaxNodes / 2;
      if (leafType) {
        const int first = firstLeafOf(static_cast<uint32_t>(b));
        tagLeaves(first + half, half, static_cast<uint32_t>(nb));
      } else {
        for (int i = 0; i < half; i++) {
          const int c = uni(static_cast<int>(s->blk[b].child[half + i]));
          s->blk[nb].child[i] = static_cast<BId>(c);
          s->blk[c].parent = static_cast<BId>(nb);
        }
      }
      s->blk[b].count = half;
      s->blk[nb].count = half;
      waveSync();
      const int p = uni(static_cast<int>(s->blk[b].parent));
      if (p == static_cast<int>(kNoBlk)) {
        const int r = allocBlk(0);
        if (r < 0) return;
        s->blk[r].count = 2;
        s->blk[r].child[0] = static_cast<BId>(b);
        s->blk[r].child[1] = static_cast<BId>(nb);
        s->blk[b].parent = static_cast<BId>(r);
        s->blk[nb].parent = static_cast<BId>(r);
        waveSync();
        root = r;
        return;
      }
      const int pc = uni(static_cast<int>(s->blk[p].count));
      int idx = 0;
      while (idx < pc && uni(static_cast<int>(s->blk[p].child[idx])) != b) idx++;
      for (int i = pc; i > idx + 1; i--) {
        const int c = uni(static_cast<int>(s->blk[p].child[i - 1]));
        waveSync();
        s->blk[p].child[i] = static_cast<BId>(c);
      }
      s->blk[p].child[idx + 1] = static_cast<BId>(nb);
      s->blk[nb].parent = static_cast<BId>(p);
      s->blk[p].count = static_cast<uint8_t>(pc + 1);
      waveSync();
      cnt = pc + 1;
      b = p;
    }
  }

  // ------------------------------------------------------------------ LRU heap (heap.ts)
  FMT_DEV int heapSeq(int k) const { return uni(s->heap[k].maxSeq); }

  // heap.ts sift order (add: fixUp; get: swap root and last, fixDown), moving a hole instead of
  // swapping entries: the same arrangement, with one LDS round trip per level (going down, both
  // children are read together; entry heapN + 1 is inside the array and never chosen)
  FMT_DEV void heapAdd(int maxSeq, uint32_t leafId) {
    if (heapN >= kHeapCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    int k = ++heapN;
    while (k > 1) {
      const HeapEnt up = s->heap[k >> 1];
      if (!(uni(up.maxSeq) - maxSeq > 0)) break;
      waveSync();
      s->heap[k] = up;
      k >>= 1;
    }
    waveSync();
    s->heap[k].maxSeq = maxSeq;
    s->heap[k].leafId = leafId;
    waveSync();
  }

  FMT_DEV HeapEnt heapGet() {
    HeapEnt top;
    top.maxSeq = uni(s->heap[1].maxSeq);
    top.leafId = uni(s->heap[1].leafId);
    const HeapEnt y = s->heap[heapN];  // the last entry sifts down from the root
    const int ys = uni(y.maxSeq);
    waveSync();
    heapN--;
    int k = 1;
    while ((k << 1) <= heapN) {
      int j = k << 1;
      const HeapEnt a = s->heap[j], b = s->heap[j + 1];
      HeapEnt c = a;
      if (j < heapN && uni(a.maxSeq) - uni(b.maxSeq) > 0) {
        j++;
        c = b;
      }
      if (ys - uni(c.maxSeq) <= 0) break;
      waveSync();
      s->heap[k] = c;
      k = j;
    }
    waveSync();
    if (heapN >= 1) s->heap[k] = y;
    waveSync();
    return top;
  }

  // ------------------------------------------------------------------ prop sets
  // matchProperties (properties.ts:32-61; undefined ≡ {}) as equality of match classes, kept when
  // sets are interned: sets with the same (key, value) content in any key order share the class of
  // the first of them; the empty set's class is undefined's.
  FMT_DEV uint32_t propCls(uint32_t a) const { return a == kPropsUndef ? 0xFFFFu : static_cast<uint32_t>(uni(static_cast<uint32_t>(s->propCls[a]))); }
  FMT_DEV bool propsMatch(uint32_t a, uint32_t b) const { return a == b || propCls(a) == propCls(b); }

  // The class of a new set q (s->kvWork[0..cnt)): lane p < q compares set p with it as maps (same
  // size, every key of one present with the same value in the other); the first match names it.
  FMT_DEV void propsIndex(int q, uint32_t cnt) {
    uint32_t cls = cnt == 0 ? 0xFFFFu : static_cast<uint32_t>(q);
    for (int base = 0; cnt > 0 && base < q && cls == static_cast<uint32_t>(q); base += 64) {
      Lane<bool> eq;
      FOR_LANES(l) {
        const int p = base + l;
        bool m = p < q && s->props[p].n == cnt;
        for (uint32_t i = 0; m && i < cnt; i++) {
          const uint32_t x = s->kvWork[i];
          bool found = false;
          for (uint32_t k = 0; k < cnt; k++)
            if ((setKv(p, k) >> 16) == (x >> 16)) found = setKv(p, k) == x;
          m = found;
        }
        LANE(eq) = m;
      }
      const uint64_t mq = ballot(eq);
      if (mq) cls = static_cast<uint32_t>(base + ctz64(mq));
    }
    waveSync();
    FOR_LANES(l) {
      if (l == 0) s->propCls[q] = static_cast<uint16_t>(cls);
    }
    waveSync();
  }

  // `seg.properties ??= {}` then raw LWW per key, null deletes (segmentPropertiesManager.ts:188-238).
  // The working set lives in LDS (kvWork, slot k = lane k % 64 of chunk k / 64), so the sets' width
  // costs no registers; the chunks past the set's entries are skipped.
  // (AdjSite: the annotate call site, the only one whose props ops can hold annotate-adjust entries)
  template <bool AdjSite = false>
  FMT_DEV uint32_t applyProps(uint32_t old, uint32_t opId) {
    uint32_t cnt = loadWork(old);
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a; t < b; t++) {
      uint32_t e = uni(in.propsKv[t]);
      const uint32_t key = e >> 16;
      uint32_t pos = cnt;
      for (int c = 0; c < kKeyChunks && pos == cnt && c * 64 < static_cast<int>(cnt); c++) {
        Lane<bool> hit;
        FOR_LANES(l) {
          const int k = c * 64 + l;
          LANE(hit) = k < static_cast<int>(cnt) && (s->kvWork[k] >> 16) == key;
        }
        const uint64_t m = ballot(hit);
        if (m) pos = static_cast<uint32_t>(c * 64 + ctz64(m));
      }
      if ((e & 0xFFFFu) == FMT_MT_VALUE_ADJUST) {  // annotate-adjust: fold into the current value
        // (an insert's or a loaded segment's props hold raw values only; batches with adjusts run the
        // Adj variant)
        if constexpr (AdjSite && Adj) {
          if (++t >= b) {
            fail(FMT_E_DATA);
            return 0;
          }
          const uint32_t cur = pos < cnt ? uni(s->kvWork[pos]) & 0xFFFFu : 0u;  // absent: null
          const uint32_t v = adjustFold(in.adj, in.doc, cur, uni(in.propsKv[t]));
          if (v == kAdjFailData || v == kAdjFailCap) {
            fail(v == kAdjFailData ? FMT_E_DATA : kCapFinal);
            return 0;
          }
          e = (key << 16) | v;
        } else {
          fail(AdjSite ? FMT_E_UNSUPPORTED : FMT_E_DATA);
          return 0;
        }
      }
      if ((e & 0xFFFFu) == 0) {  // null: delete the key
        if (pos < cnt) {  // entries pos+1 .. cnt-1 move down one slot, a chunk at a time in slot order
          for (int c = static_cast<int>(pos) / 64; c < kKeyChunks && c * 64 < static_cast<int>(cnt); c++) {
            Lane<uint32_t> v;
            FOR_LANES(l) {
              const int k = c * 64 + l;
              LANE(v) = (k < kKeysMax - 1 && k >= static_cast<int>(pos)) ? s->kvWork[k + 1] : 0u;
            }
            waveSync();
            FOR_LANES(l) {
              const int k = c * 64 + l;
              if (k >= static_cast<int>(pos) && k + 1 < static_cast<int>(cnt)) s->kvWork[k] = LANE(v);
            }
            waveSync();
          }
          cnt--;
        }
      } else if (pos < cnt) {
        FOR_LANES(l) {
          if (l == static_cast<int>(pos % 64)) s->kvWork[pos] = e;
        }
      } else {
        if (cnt >= static_cast<uint32_t>(kKeysMax)) {
          fail(kCapFinal);
          return 0;
        }
        FOR_LANES(l) {
          if (l == static_cast<int>(cnt % 64)) s->kvWork[cnt] = e;
        }
        cnt++;
      }
      waveSync();
    }
    return internWork(cnt);
  }

  // The prop set s->kvWork[0 .. cnt) (key order kept) as an interned set id: an equal set already in
  // the table, else a new one.
  // (a set wider than FMT_MT_PROPS_MAX takes consecutive records, fmt.h fmt_mt_propset)
  FMT_DEV uint32_t internWork(uint32_t cnt) {
    for (int base = 0; base < nProps; base += 64) {  // interned already? lane p checks prop set base + p
      Lane<bool> same;
      FOR_LANES(l) {
        const int p = base + l;
        bool eq = p < nProps && s->props[p].n == cnt;
        for (uint32_t i = 0; eq && i < cnt; i++) eq = setKv(p, i) == s->kvWork[i];
        LANE(same) = eq;
      }
      const uint64_t m = ballot(same);
      if (m != 0) return static_cast<uint32_t>(base + ctz64(m));
    }
    const int rec = cnt > FMT_MT_PROPS_MAX ? static_cast<int>((cnt + FMT_MT_PROPS_MAX - 1) / FMT_MT_PROPS_MAX) : 1;
    if (nProps + rec > kPropCap) {
      fail(FMT_E_CAPACITY);
      return 0;
    }
    propsIndex(nProps, cnt);
    for (int c = 0; c * 64 < rec * FMT_MT_PROPS_MAX; c++) {  // (slots past cnt: the record's unused entries, 0)
      FOR_LANES(l) {
        const int j = c * 64 + l, q = j / FMT_MT_PROPS_MAX, k = j % FMT_MT_PROPS_MAX;
        if (q < rec) {
          if (k == 0) s->props[nProps + q].n = q == 0 ? cnt : FMT_MT_PROPS_CONT;
          s->props[nProps + q].kv[k] = j < static_cast<int>(cnt) ? s->kvWork[j] : 0u;
          if (k == 0 && q > 0) s->propCls[nProps + q] = 0xFFFEu;  // (a continuation: no leaf names it)
        }
      }
    }
    waveSync();
    const int id = nProps;
    nProps += rec;
    return static_cast<uint32_t>(id);
  }
  // entry k of the prop set whose first record is p
  FMT_DEV uint32_t setKv(int p, uint32_t k) const { return s->props[p + static_cast<int>(k / FMT_MT_PROPS_MAX)].kv[k % FMT_MT_PROPS_MAX]; }
  // the working set = the entries of set `old` (kPropsUndef: none); returns their count (slots past
  // it are never read)
  FMT_DEV uint32_t loadWork(uint32_t old) {
    const uint32_t cnt = old != kPropsUndef ? uni(s->props[old].n) : 0u;
    for (int c = 0; c < kKeyChunks && c * 64 < static_cast<int>(cnt); c++) {
      FOR_LANES(l) {
        const int k = c * 64 + l;
        if (k < static_cast<int>(cnt)) s->kvWork[k] = setKv(static_cast<int>(old), static_cast<uint32_t>(k));
      }
    }
    waveSync();
    return cnt;
  }

  // ------------------------------------------------------------------ property managers (Adj)
  // segment.propertyManager (segmentPropertiesManager.ts:140-345) of every leaf, kept for the legacy
  // summary's getAtSeq(properties, minSeq) (snapshotlegacy.ts:211-212), as records in the document's
  // HBM slab, in creation order: a head {leaf id, key, kind 0, value = msnConsensus} per (leaf, key)
  // that has pending remote changes (the manager's Map order), and the pending changes {leaf id, key,
  // kind 1, seq, value after the change}. A change's value after it is all a later fold needs: the
  // fold of msnConsensus with a prefix of the list equals the value the last change of that prefix
  // produced when it applied. A raw change folds straight into msnConsensus while its key has nothing
  // pending (:213-221); updateMsn(msn) (:275-291) folds the changes at or below msn and drops a key
  // left with none. Record words: leaf id (0: deleted), key | kind << 16, seq, value.
  int pmN = 0;  // records in use (deleted ones included)
  // (Loc: the local client's managers, in its own slab: heads {leaf, key, 0, msnConsensus} and local
  // changes {leaf, key | 0x20000, group serial, value}, segmentPropertiesManager.ts:48-52 `local`)
  FMT_DEV uint32_t* pmBase() const {
    if constexpr (Loc) return in.loc->pm + 4 * in.loc->pmOffs[in.doc];
    else return in.adj->pm + 4 * in.adj->pmOffsets[in.doc];
  }
  FMT_DEV int pmCap() const {
    if constexpr (Loc) return static_cast<int>(in.loc->pmOffs[in.doc + 1] - in.loc->pmOffs[in.doc]);
    else return static_cast<int>(in.adj->pmOffsets[in.doc + 1] - in.adj->pmOffsets[in.doc]);
  }
  FMT_DEV uint32_t pmWord(int i, int w) const { return uni(loadCoherent(pmBase() + 4 * i + w)); }

  // First record at or after `from` whose (leaf id, key | kind) match (~0u: any key / kind), or -1.
  FMT_DEV int pmFind(uint32_t leaf, uint32_t keyKind, uint32_t mask, int from = 0) const {
    const uint32_t* R = pmBase();
    for (int base = from; base < pmN; base += 64) {
      Lane<bool> p;
      FOR_LANES(l) {
        const int i = base + l;
        LANE(p) = i < pmN && loadCoherent(R + 4 * i) == leaf && (loadCoherent(R + 4 * i + 1) & mask) == (keyKind & mask);
      }
      const uint64_t m = ballot(p);
      if (m != 0) return base + ctz64(m);
    }
    return -1;
  }

  // Drops deleted records, keeping the order (a wave stream compaction in place).
  FMT_DEV void pmCompact() {
    uint32_t* R = pmBase();
    int out = 0;
    for (int base = 0; base < pmN; base += 64) {
      Lane<uint32_t> w0, w1, w2, w3;
      Lane<bool> live;
      FOR_LANES(l) {
        const int i = base + l;
        LANE(w0) = i < pmN ? loadCoherent(R + 4 * i) : 0u;
        LANE(w1) = i < pmN ? loadCoherent(R + 4 * i + 1) : 0u;
        LANE(w2) = i < pmN ? loadCoherent(R + 4 * i + 2) : 0u;
        LANE(w3) = i < pmN ? loadCoherent(R + 4 * i + 3) : 0u;
        LANE(live) = LANE(w0) != 0u;
      }
      const uint64_t m = ballot(live);
      FOR_LANES(l) {
        if (LANE(live)) {
          const int at = out + __builtin_popcountll(m & ((1ull << l) - 1ull));
          storeGlobal(R + 4 * at, LANE(w0));
          storeGlobal(R + 4 * at + 1, LANE(w1));
          storeGlobal(R + 4 * at + 2, LANE(w2));
          storeGlobal(R + 4 * at + 3, LANE(w3));
        }
      }
      out += __builtin_popcountll(m);
    }
    pmN = out;
  }

  FMT_DEV bool pmAppend(uint32_t leaf, uint32_t keyKind, int seq, uint32_t value) {
    if (pmN >= pmCap()) pmCompact();
    if (pmN >= pmCap()) return fail(kCapFinal);
    uint32_t* R = pmBase() + 4 * pmN;
    FOR_LANES(l) {
      if (l < 4) storeGlobal(R + l, l == 0 ? leaf : l == 1 ? keyKind : l == 2 ? static_cast<uint32_t>(seq) : value);
    }
    pmN++;
    return true;
  }

  FMT_DEV void pmSet(int i, int w, uint32_t v) {
    uint32_t* R = pmBase() + 4 * i + w;
    FOR_LANES(l) {
      if (l == 0) storeGlobal(R, v);
    }
  }

  // updateMsn(msn) on the manager of leaf `leaf`.
  FMT_DEV void pmUpdateMsn(uint32_t leaf, int msn) {
    // (heads: records of kind 0; Loc's local changes, kind 2, are neither heads nor folded)
    for (int h = pmFind(leaf, 0u, 0x30000u); h >= 0 && status == FMT_OK; h = pmFind(leaf, 0u, 0x30000u, h + 1)) {
      const uint32_t key = pmWord(h, 1) & 0xFFFFu;
      const uint32_t* R = pmBase();
      int last = -1;
      bool pending = false;
      for (int base = h + 1; base < pmN; base += 64) {  // (a head precedes its key's changes)
        Lane<bool> fold, keep;
        FOR_LANES(l) {
          const int i = base + l;
          const bool mine = i < pmN && loadCoherent(R + 4 * i) == leaf && loadCoherent(R + 4 * i + 1) == (key | 0x10000u);
          const int sq = mine ? static_cast<int>(loadCoherent(R + 4 * i + 2)) : 0;
          LANE(fold) = mine && sq <= msn;
          LANE(keep) = mine && sq > msn;
        }
        const uint64_t mf = ballot(fold), mk = ballot(keep);
        if (mf != 0) last = base + 63 - __builtin_clzll(mf);
        pending = pending || mk != 0;
        FOR_LANES(l) {
          if (LANE(fold)) storeGlobal(pmBase() + 4 * (base + l), 0u);  // folded: deleted
        }
      }
      if (last >= 0) pmSet(h, 3, pmWord(last, 3));  // (a deleted record keeps its value word)
      if constexpr (Loc) pending = pending || pmFind(leaf, key | 0x20000u, 0x3FFFFu, h + 1) >= 0;
      if (!pending) pmSet(h, 0, 0u);
    }
  }

  // copyTo (segmentPropertiesManager.ts:300-316): a split's right part gets the left's records.
  FMT_DEV void pmCopy(uint32_t from, uint32_t to) {
    if (pmFind(from, 0u, 0u) < 0) return;
    pmCompact();  // (no compaction while copying: record indices stay put)
    const int end = pmN;
    for (int i = pmFind(from, 0u, 0u); i >= 0 && i < end && status == FMT_OK; i = pmFind(from, 0u, 0u, i + 1)) {
      if (pmN >= pmCap()) {
        fail(kCapFinal);
        return;
      }
      pmAppend(to, pmWord(i, 1), static_cast<int>(pmWord(i, 2)), pmWord(i, 3));
    }
  }

  FMT_DEV void pmDropLeaf(uint32_t leaf) {  // the leaf left the tree (zamboni): its manager is unreachable
    const uint32_t* R = pmBase();
    for (int base = 0; base < pmN; base += 64) {
      FOR_LANES(l) {
        const int i = base + l;
        if (i < pmN && loadCoherent(R + 4 * i) == leaf) storeGlobal(pmBase() + 4 * i, 0u);
      }
    }
  }

  // handleProperties (segmentPropertiesManager.ts:188-238) of an annotate op on leaf j, before the
  // leaf's prop set changes: every change of the op in opToChanges order, then updateMsn(minSeq).
  FMT_DEV void pmAnnotate(int j, uint32_t opId, int seq) {
    const uint32_t leaf = fId(readField(j, 4));
    const uint32_t old = propsAt(j);
    uint32_t cnt = loadWork(old);
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a; t < b && status == FMT_OK; t++) {
      const uint32_t e = uni(in.propsKv[t]);
      const uint32_t key = e >> 16;
      const bool adjust = (e & 0xFFFFu) == FMT_MT_VALUE_ADJUST;
      uint32_t pos = cnt;
      for (uint32_t k = 0; k < cnt; k++)
        if ((uni(s->kvWork[k]) >> 16) == key) pos = k;
      const uint32_t before = pos < cnt ? uni(s->kvWork[pos]) & 0xFFFFu : 0u;
      uint32_t after = e & 0xFFFFu;
      if (adjust) {
        if (++t >= b) {
          fail(FMT_E_DATA);
          return;
        }
        after = adjustFold(in.adj, in.doc, before, uni(in.propsKv[t]));
        if (after == kAdjFailData || after == kAdjFailCap) {
          fail(after == kAdjFailData ? FMT_E_DATA : kCapFinal);
          return;
        }
      }
      int h = pmFind(leaf, key, 0x1FFFFu);
      if (h < 0) {
        if (!pmAppend(leaf, key, 0, before)) return;
        h = pmN - 1;
      }
      if (!adjust && pmFind(leaf, key | 0x10000u, 0x1FFFFu, h + 1) < 0) pmSet(h, 3, after);
      else if (!pmAppend(leaf, key | 0x10000u, seq, after)) return;
      // the working set follows the change (null deletes the key)
      if (after == 0u) {
        if (pos < cnt) {
          for (uint32_t k = pos; k + 1 < cnt; k++) {
            const uint32_t v = uni(s->kvWork[k + 1]);
            waveSync();
            FOR_LANES(l) {
              if (l == 0) s->kvWork[k] = v;
            }
          }
          cnt--;
        }
      } else if (pos < cnt) {
        FOR_LANES(l) {
          if (l == 0) s->kvWork[pos] = (key << 16) | after;
        }
      } else if (cnt < static_cast<uint32_t>(kKeysMax)) {
        FOR_LANES(l) {
          if (l == 0) s->kvWork[cnt] = (key << 16) | after;
        }
        cnt++;
      }
      waveSync();
    }
    pmUpdateMsn(leaf, minSeq);
  }

  // getAtSeq(properties, minSeq) of every leaf (segmentPropertiesManager.ts:328-344): leaves with a
  // pending key get the interned set of their current properties with each pending key set to the
  // value its changes at or below minSeq leave (null: deleted; a key the properties lack goes last, in
  // the manager's key order); the others keep their set.
  FMT_DEV void pmLegacyProps(uint16_t* out) {
    const int nr = rows();
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        const int idx = r * 64 + l;
        if (idx < n) {
          const uint32_t pid = propsL(l, r);
          out[idx] = pid == kPropsUndef ? 0xFFFFu : static_cast<uint16_t>(pid);
        }
      }
    }
    const uint32_t* R = pmBase();
    for (int h0 = 0; h0 < pmN && status == FMT_OK;) {
      // the next head of a leaf not handled yet (a handled head's seq word gets bit 31)
      int h = -1;
      for (int base = h0; base < pmN && h < 0; base += 64) {
        Lane<bool> p;
        FOR_LANES(l) {
          const int i = base + l;
          LANE(p) = i < pmN && loadCoherent(R + 4 * i) != 0u && (loadCoherent(R + 4 * i + 1) & 0x30000u) == 0u &&
                    (loadCoherent(R + 4 * i + 2) & 0x80000000u) == 0u;
        }
        const uint64_t m = ballot(p);
        if (m != 0) h = base + ctz64(m);
      }
      if (h < 0) break;
      const uint32_t leaf = pmWord(h, 0);
      const int j = findLeafById(leaf);
      uint32_t cnt = 0;
      if (j >= 0) {
        cnt = loadWork(propsAt(j));
      }
      for (int g = h; g >= 0 && status == FMT_OK; g = pmFind(leaf, 0u, 0x30000u, g + 1)) {
        pmSet(g, 2, 0x80000000u);  // (done: a head's seq word is otherwise unused)
        if (j < 0) continue;
        const uint32_t key = pmWord(g, 1) & 0xFFFFu;
        uint32_t v = pmWord(g, 3);
        for (int c = pmFind(leaf, key | 0x10000u, 0x1FFFFu, g + 1); c >= 0; c = pmFind(leaf, key | 0x10000u, 0x1FFFFu, c + 1)) {
          if (static_cast<int>(pmWord(c, 2)) > minSeq) break;  // (a key's changes are in seq order)
          v = pmWord(c, 3);
        }
        uint32_t pos = cnt;
        for (uint32_t k = 0; k < cnt; k++)
          if ((uni(s->kvWork[k]) >> 16) == key) pos = k;
        if (v == 0u) {
          if (pos < cnt) {
            for (uint32_t k = pos; k + 1 < cnt; k++) {
              const uint32_t x = uni(s->kvWork[k + 1]);
              waveSync();
              FOR_LANES(l) {
                if (l == 0) s->kvWork[k] = x;
              }
            }
            cnt--;
          }
        } else if (pos < cnt) {
          FOR_LANES(l) {
            if (l == 0) s->kvWork[pos] = (key << 16) | v;
          }
        } else if (cnt < static_cast<uint32_t>(kKeysMax)) {
          FOR_LANES(l) {
            if (l == 0) s->kvWork[cnt] = (key << 16) | v;
          }
          cnt++;
        } else {
          fail(kCapFinal);
        }
        waveSync();
      }
      if (j >= 0 && status == FMT_OK) {
        const uint32_t id = internWork(cnt);
        if (status != FMT_OK) break;
        FOR_LANES(l) {
          if (l == 0) out[j] = static_cast<uint16_t>(id);
        }
      }
      h0 = h + 1;
    }
  }

  // ------------------------------------------------------------------ annotate-adjust
  // computePropertyValue for one adjust change (segmentPropertiesManager.ts:54-78): the current
  // value's number (typeof "number", else 0) + delta, then max clamps, else min, in IEEE double.
  // A change's current value is always the running fold of the key's changes in seq order (every
  // remote change folds into properties[key] when it applies, :199-235), so the replay state needs
  // no per-segment change lists. Returns the result's value id (0: null, the key is deleted).
  // ------------------------------------------------------------------ catch-up ranges
  // The ranges of the op's sequenceDelta event, merged as createOpsFromDelta merges them
  // (sequence/src/sequence.ts:395-452) and recorded for the legacy summary's catch-up ops. `delta`
  // is a per-lane row bitmask of the delta segments: the inserted leaf, the newly removed leaves, or
  // the annotated leaves not removed. Each one's position is Client.getPosition in the local view
  // right after the op (before its zamboni): the prefix of not-removed leaf lengths. A REMOVE range
  // absorbs a segment starting where it starts (removed text has no local length); an ANNOTATE
  // range one starting where it ends (the props always match: every delta segment now holds the
  // op's own raw values for exactly the op's keys).
  FMT_DEV void recordCatchup(const Lane<uint32_t>& delta, int type) {
    const int nr = rows();
    uint32_t base = 0;  // local length of the rows before r (row by row: no per-leaf prefix array)
    int p1 = 0, p2 = 0;
    bool open = false;
    FOR_ROWS(r, 0, nr) {
      Lane<uint32_t> loc;
      Lane<bool> p;
      FOR_LANES(l) {
        LANE(loc) = static_cast<int32_t>(LANE(W[2])[r]) == kNotRemoved ? fLen(LANE(W[0])[r]) : 0u;
        LANE(p) = ((LANE(delta) >> r) & 1u) != 0;
      }
      uint32_t tot;
      const Lane<uint32_t> ex = waveExclusiveSum(loc, &tot);
      uint64_t m = ballot(p);
      while (m) {
        const int lane = ctz64(m);
        m &= m - 1;
        const int pos = static_cast<int>(readlane(ex, lane) + base);
        const int len = static_cast<int>(fLen(readlane(row(W[0], r), lane)));
        if (open && (((type == FMT_MT_REMOVE || type == FMT_MT_OBLITERATE) && p1 == pos) ||
                     (type == FMT_MT_ANNOTATE && p2 == pos))) {
          p2 += len;
          continue;
        }
        if (open) emitCatchup(p1, p2, type);
        p1 = pos;
        p2 = pos + len;
        open = true;
      }
      base += tot;
    }
    if (open) emitCatchup(p1, p2, type);
  }

  FMT_DEV void emitCatchup(int p1, int p2, int type) {
    if (cuN >= cuCap) {
      fail(kCapFinal);
      return;
    }
    FOR_LANES(l) {
      if (l == 0) {
        fmt_mt_catchup_range c;
        c.op = opIdx;
        c.pos1 = p1;
        c.pos2 = p2;
        c.type = static_cast<uint32_t>(type);
        cuOut[cuN] = c;
      }
    }
    cuN++;
  }

  // ------------------------------------------------------------------ remove order (SnapshotV1)
  // A flagged REMOVE or obliterate that hits an already-removed leaf adds a later remove stamp to it
  // (spliceIntoList, stamps.ts:144-158: remote stamps arrive in seq order, so they append), and an
  // obliterate-on-insert can give a new leaf several. The summary's removedClientIds and
  // movedSeqs / movedClientIds (snapshotV1.ts:235-264) need them in order, by kind, which the
  // remove-client mask W3 does not keep: each such stamp is appended to the document's HBM slab as
  // (leaf id, client, seq, kind). Rare (concurrent overlapping removes), so lane 0 writes one entry
  // at a time.
  FMT_DEV void rmAppend(uint32_t id, int client, int seq, uint32_t kind) {
    if (rmN >= rmCap) {
      fail(kCapFinal);
      return;
    }
    FOR_LANES(l) {
      if (l == 0) {
        fmt_mt_remove_order e;
        e.leaf = id;
        e.client = client;
        e.seq = seq;
        e.kind = kind;
        rmOut[rmN] = e;
      }
    }
    rmN++;
  }

  // Deferred to one call site per op (replay, before zamboni), so the rare recording code is inlined
  // once: the right parts of split multi-removed leaves inherit their entries (splitLeafSegment
  // copies the remove stamps, mergeTreeNodes.ts:389-435), in split order; then every leaf the
  // flagged REMOVE found already removed gets the op's stamp.
  FMT_DEV void rmFlush(int client, int seq, uint32_t kind) {
    for (int q = 0; q < rmPendN && status == FMT_OK; q++) {
      const uint32_t from = q == 0 ? rmPendFrom0 : rmPendFrom1, to = q == 0 ? rmPendTo0 : rmPendTo1;
      const uint32_t n0 = rmN;
      for (uint32_t k = 0; k < n0 && status == FMT_OK; k++) {
        if (uni(loadCoherent(&rmOut[k].leaf)) == from)
          rmAppend(to, static_cast<int>(uni(loadCoherent(reinterpret_cast<const uint32_t*>(&rmOut[k].client)))),
                   static_cast<int>(uni(loadCoherent(reinterpret_cast<const uint32_t*>(&rmOut[k].seq)))),
                   uni(loadCoherent(&rmOut[k].kind)));
      }
    }
    rmPendN = 0;
    if (rmHitsSet) {
      rmHitsSet = false;
      Lane<uint32_t> todo = rmHits;
      const int nr = rows();
      for (;;) {
        const int j = firstSet(todo, nr);
        if (j < 0 || status != FMT_OK) break;
        FOR_LANES(l) {
          if (l == (j & 63)) LANE(todo) &= ~(1u << (j >> 6));
        }
        rmAppend(fId(readField(j, 4)), client, seq, kind);
      }
    }
  }

  // ------------------------------------------------------------------ ops
  // addToLRUSet (mergeTree.ts:812-822) for leaf j: the first registration of a block sets
  // needsScour; later leaves of that block are no-ops until zamboni clears it.
  FMT_DEV void lruForLeaf(int j, int b, int seq) {
    if (uni(static_cast<int>(s->blk[b].needsScour)) != 1 && seq > curSeq) {
      s->blk[b].needsScour = 1;
      waveSync();
      heapAdd(seq, fId(readField(j, 4)));
    }
  }

  // addToLRUSet for every hit leaf in document order. Leaf blocks are contiguous runs, so only the
  // first hit of each block can register: take the first remaining hit, register its block, clear
  // that block's hits, repeat (one pass per distinct block instead of one step per hit leaf).
  FMT_DEV void lruForHits(const Lane<uint32_t>& hits, int seq, int nr) {
    Lane<uint32_t> todo = hits;
    for (;;) {
      const int j = firstSet(todo, nr);
      if (j < 0) return;
      const uint32_t b = fBlk(readField(j, 0));
      lruForLeaf(j, static_cast<int>(b), seq);
      if (status != FMT_OK) return;
      FOR_ROWS(r, 0, nr) {
        FOR_LANES(l) {
          if (fBlk(LANE(W[0])[r]) == b) LANE(todo) &= ~(1u << r);
        }
      }
    }
  }

  // splitLeafSegment (mergeTree.ts:1768-1796) of leaf j at `offset` (0 < offset < len): the right
  // part becomes leaf j + 1 of the same block, with a fresh id and the same stamps and props.
  FMT_DEV bool splitLeafAt(int j, int offset) {
    if (nextId >= kIdLimit) return fail(kCapFinal);
    LeafRec rec;
    const uint32_t w0 = readField(j, 0);
    const uint32_t w4 = readField(j, 4);
    rec.w[0] = mkW0(fLen(w0) - static_cast<uint32_t>(offset), fBlk(w0), fProps(w0));
    rec.w[1] = readField(j, 1);
    rec.w[2] = readField(j, 2);
    rec.w[3] = readField(j, 3);
    rec.w[4] = mkW4(nextId++, fClient(w4));
    rec.w[5] = C::kWords > 5 ? readField(j, 5) : 0u;
    rec.w[6] = kPW ? readField(j, kPropW) : 0u;
    rec.w[7] = 0u;
    if constexpr (Loc) {  // SegmentGroupCollection.copyTo (splitLeafSegment, mergeTree.ts:1779-1782)
      rec.w[kPendW] = readField(j, kPendW);
      if (rec.w[kPendW] != 0u) recCopy(fId(w4), fId(rec.w[4]));
    }
    if constexpr (Ob) {  // LocalReferenceCollection.split (localReference.ts:464-483)
      if (obUsed != 0) obRefsMove(fId(w4), fId(rec.w[4]), offset, -offset);
    }
    if constexpr (Rm) {
      if (rmN > 0 && static_cast<int32_t>(rec.w[2]) != kNotRemoved) {  // its entries, if any: copied in rmFlush
        if (rmPendN >= 2) return fail(FMT_E_DATA);  // an op splits at most twice: a broken invariant
        if (rmPendN == 0) {
          rmPendFrom0 = fId(w4);
          rmPendTo0 = fId(rec.w[4]);
        } else {
          rmPendFrom1 = fId(w4);
          rmPendTo1 = fId(rec.w[4]);
        }
        rmPendN++;
      }
    }
    if constexpr (Adj || Loc) {  // copyPropertiesAndManager (mergeTree.ts:1784)
      if (pmN > 0) pmCopy(fId(w4), fId(rec.w[4]));
    }
    writeField(j, 0, mkW0(static_cast<uint32_t>(offset), fBlk(w0), fProps(w0)));
    if (!insertLeafAt(j + 1, rec)) return false;
    childAdded(static_cast<int>(fBlk(w0)));
    stamp(kPfSplit);
    return status == FMT_OK;
  }

  // The leaf that strictly contains view position pos (st < pos < st + vis), or -1; *stOut = its st.
  FMT_DEV static int containing(const Lane<VR>& vis, const Lane<VR>& st, int pos, int nr, int* stOut) {
    FOR_ROWS(r, 0, nr) {
      Lane<bool> p;
      FOR_LANES(l) {
        const int sp = static_cast<int>(LANE(st)[r]);
        LANE(p) = sp < pos && pos < sp + static_cast<int>(LANE(vis)[r]);
      }
      const uint64_t m = ballot(p);
      if (m != 0) {
        *stOut = static_cast<int>(readlane(row(st, r), ctz64(m)));
        return r * 64 + ctz64(m);
      }
    }
    return -1;
  }

  // ensureIntervalBoundary (mergeTree.ts:1798-1808): split the unique leaf that strictly contains
  // pos in the op's view. Returns false only on failure. (Obliterate's path; inserts and
  // remove/annotate resolve their boundaries from their one view scan instead.)
  FMT_DEV bool splitAt(int pos, int refSeq, int client) {
    const int nr = rows();
    Lane<VR> vis, st;
    visLengths(refSeq, client, vis, nr);
    scanRows(vis, st, nr);
    stamp(kPfScan);
    int sp = 0;
    const int j = containing(vis, st, pos, nr, &sp);
    if (j < 0) {
      stamp(kPfSplit);
      return true;
    }
    return splitLeafAt(j, pos - sp);
  }

  // A row bitmask (bit r of lane l = leaf 64 r + l) after inserting a leaf at index k with bit b:
  // bits at k and above move up one leaf, exactly like insertLeafAt moves the leaves.
  FMT_DEV static Lane<uint32_t> maskInsert(const Lane<uint32_t>& m, int k, bool b) {
    const Lane<uint32_t> up = shflUp1(m);
    const uint32_t carry = readlane(m, 63) << 1;
    const int rk = k >> 6, kl = k & 63;
    Lane<uint32_t> out;
    FOR_LANES(l) {
      const int keepRows = k > l ? (k - l + 63) >> 6 : 0;  // rows r with 64 r + l < k
      const uint32_t keep = keepRows >= 32 ? ~0u : (1u << keepRows) - 1u;
      const uint32_t shifted = l == 0 ? carry : LANE(up);
      uint32_t v = (LANE(m) & keep) | (shifted & ~keep);
      if (l == kl) v = (v & ~(1u << rk)) | (b ? 1u << rk : 0u);
      LANE(out) = v;
    }
    return out;
  }

  // insertSegments (mergeTree.ts:1484-1517) after the boundary split: the new leaf goes before the
  // first leaf whose view prefix equals pos, leaves removed at/below minSeq skipped except the very
  // last leaf (mergeTree.ts:1862-1875); past the end it is appended to the last leaf's block.
  // Returns the new leaf's index, or -1 (nothing inserted, or failure).
  // (localOp, Loc: the local client's submission — local perspective, local stamp, no LRU entry)
  FMT_DEV int insertText(const fmt_mt_op& op, const Lane<uint32_t>& text0, int clientArg = 0x7fff, bool boundary = true,
                         bool localOp = false) {
    const int refSeq = op.ref_seq, client = clientArg != 0x7fff ? clientArg : op.client, seq = op.seq;
    const int pos = op.pos1, len = static_cast<int>(opLen(op));
    const int nr = rows();
    Lane<VR> vis, st;
    visLengths(refSeq, client, vis, nr);
    const uint32_t total = scanRows(vis, st, nr);
    stamp(kPfScan);
    // ensureIntervalBoundary(pos) from the same scan: a split leaves every view start in place, and
    // the right part (view start pos) is then the first leaf at pos.
    int sp = 0;
    const int js = containing(vis, st, pos, nr, &sp);
    if (boundary && js >= 0 && !splitLeafAt(js, pos - sp)) return -1;
    if (len <= 0) return -1;
    // seg {text, props}: the new segment's properties = clone(props) (textSegment.ts:41-52,
    // mergeTreeNodes.ts:343-347): raw LWW of the props op onto an empty set
    uint32_t insProps = kPropsUndef;
    if (op.pos2 > 0) {
      if (static_cast<uint32_t>(op.pos2 - 1) >= in.nPropsOps) {
        fail(FMT_E_DATA);
        return -1;
      }
      insProps = applyProps(kPropsUndef, static_cast<uint32_t>(op.pos2 - 1));
      if (status != FMT_OK) return -1;
    }
    // (without the boundary — a loader batch's later segment — the walk stops at the leaf holding
    // pos and inserts before it, mergeTree.ts:1876-1882)
    int insIdx = js >= 0 ? (boundary ? js + 1 : js) : -1;
    FOR_ROWS(r, 0, nr) {
      if (insIdx < 0) {
        Lane<bool> p;
        FOR_LANES(l) {
          const int idx = r * 64 + l;
          const bool undefinedLen = static_cast<int32_t>(LANE(W[2])[r]) <= minSeq;
          const bool skipped = undefinedLen && idx != n - 1;
          // breakTie (mergeTree.ts:1811-1826) of a remote insert against a leaf the local client
          // inserted and has not had acked: the remote stamp is older, so the walk passes it
          const bool tie = !Loc || localOp || LANE(vis)[r] > 0u || static_cast<int32_t>(LANE(W[1])[r]) < FMT_MT_LOCAL_SEQ_BASE;
          LANE(p) = idx < n && !skipped && tie && static_cast<int>(LANE(st)[r]) == pos;
        }
        const uint64_t m = ballot(p);
        if (m != 0) insIdx = r * 64 + ctz64(m);
      }
    }
    int blk;
    if (insIdx >= 0) {
      blk = static_cast<int>(fBlk(readField(insIdx, 0)));
    } else {
      if (pos != static_cast<int>(total)) {  // "MergeTree insert failed" (mergeTree.ts:1629)
        fail(FMT_E_DATA);
        return -1;
      }
      insIdx = n;
      blk = n > 0 ? static_cast<int>(fBlk(readField(n - 1, 0))) : root;
    }
    if (nChars + len > kCapChars) {
      fail(FMT_E_CAPACITY);
      return -1;
    }
    if (nextId >= kIdLimit) {
      fail(kCapFinal);
      return -1;
    }
    const int cpos = static_cast<int>(charOffsetOf(insIdx));
    charsShiftUp(cpos, len);
    FOR_LANES(l) {
      if (l < len) chWrite(cpos + l, LANE(text0));
      for (int t = l + 64; t < len; t += 64) chWrite(cpos + t, in.text[op.payload + t]);
    }
    waveSync();
    nChars += len;
    stamp(kPfInsChars);
    LeafRec rec;
    rec.w[0] = mkW0(static_cast<uint32_t>(len), static_cast<uint32_t>(blk), insProps);
    rec.w[1] = static_cast<uint32_t>(seq);
    rec.w[2] = static_cast<uint32_t>(kNotRemoved);
    rec.w[3] = 0;
    rec.w[4] = mkW4(nextId++, client) | ((op.flags & FMT_MT_F_MARKER) != 0 ? kW4Marker : 0u);  // Marker.make
    rec.w[5] = 0;
    rec.w[6] = insProps;
    rec.w[7] = 0;
    if (uni(static_cast<int>(s->blk[blk].count)) == 0) {
      s->blk[blk].leaf = 1;  // an empty root becomes a leaf block
      waveSync();
    }
    if (!insertLeafAt(insIdx, rec)) return -1;
    stamp(kPfInsShift);
    childAdded(blk);
    if (status != FMT_OK) return -1;
    stamp(kPfInsert);
    if constexpr (Ob) {
      if (obStartN > 0) obliterateOnInsert(insIdx, refSeq, client, Rm && (op.flags & FMT_MT_F_RMORDER) != 0);
    }
    if (!localOp) lruForLeaf(insIdx, static_cast<int>(fBlk(readField(insIdx, 0))), seq);
    stamp(kPfLru);
    return status == FMT_OK ? insIdx : -1;
  }

  // ------------------------------------------------------------------ obliterates (f1)
  // Obliterates (mergeTree.ts:515-625). A reference's "ordinal" is its leaf's document index, or
  // "" (smallest) once the leaf is gone from the tree or the reference was removed.
  FMT_DEV int leafOf(uint32_t id) const { return id == 0 ? -1 : findLeafById(id); }

  FMT_DEV static int ordinalCompare(int ia, int ib) {
    if (ia < 0 || ib < 0) return (ia < 0) == (ib < 0) ? 0 : (ia < 0 ? -1 : 1);
    return ia < ib ? -1 : (ia > ib ? 1 : 0);
  }

  FMT_DEV int startCompare(int a, int b) const {  // SortedSegmentSet.compare on start references
    const int c = ordinalCompare(leafOf(uni(s->ob[a].startId)), leafOf(uni(s->ob[b].startId)));
    return c != 0 ? c : uni(s->ob[a].startOff) - uni(s->ob[b].startOff);
  }

  // SortedSet.findItemPosition + SortedSegmentSet.onFindEquivalent (sortedSet.ts,
  // sortedSegmentSet.ts), verbatim: the array is only as sorted as the ordinals were at insertion.
  FMT_DEV int findStart(int slot, bool* exists) const {
    *exists = false;
    if (obStartN == 0) return 0;
    int start = 0, end = obStartN - 1, index = -1;
    while (start <= end) {
      index = start + (end - start) / 2;
      const int at = uni(static_cast<int>(s->obStart[index]));
      const int c = startCompare(slot, at);
      if (c < 0) {
        if (start == index) return index;
        end = index - 1;
      } else if (c > 0) {
        if (index == end) return index + 1;
        start = index + 1;
      } else {
        if (at == slot) {
          *exists = true;
          return index;
        }
        for (int b = index - 1; b >= 0 && startCompare(slot, uni(static_cast<int>(s->obStart[b]))) == 0; b--)
          if (uni(static_cast<int>(s->obStart[b])) == slot) {
            *exists = true;
            return b;
          }
        for (; index < obStartN && startCompare(slot, uni(static_cast<int>(s->obStart[index]))) == 0; index++)
          if (uni(static_cast<int>(s->obStart[index])) == slot) {
            *exists = true;
            return index;
          }
        return index;
      }
    }
    return index;
  }

  // References on leaf `from` at offset >= minOff move to leaf `to`, offset += add (split: the
  // right part; zamboni append: every reference of the appended leaf).
  FMT_DEV void obRefsMove(uint32_t from, uint32_t to, int minOff, int add) {
    for (int k = 0; k < kObCap; k++) {
      if (((obUsed >> k) & 1ull) == 0) continue;
      const uint32_t sid = uni(s->ob[k].startId), eid = uni(s->ob[k].endId);
      const int so = uni(s->ob[k].startOff), eo = uni(s->ob[k].endOff);
      waveSync();
      if (sid == from && so >= minOff) {
        s->ob[k].startId = to;
        s->ob[k].startOff = so + add;
      }
      if (eid == from && eo >= minOff) {
        s->ob[k].endId = to;
        s->ob[k].endOff = eo + add;
      }
      waveSync();
    }
  }

  FMT_DEV bool obAdd(uint32_t sId, int sOff, uint32_t eId, int eOff, int seq, int client) {
    // (more live obliterates than this table holds: the document grows, up to the huge tier's HBM table)
    if (obUsed == ~0ull) return fail(FMT_E_CAPACITY);
    const int slot = ctz64(~obUsed);
    obUsed |= 1ull << slot;
    s->ob[slot].startId = sId;
    s->ob[slot].startOff = sOff;
    s->ob[slot].endId = eId;
    s->ob[slot].endOff = eOff;
    s->ob[slot].seq = seq;
    s->ob[slot].client = client;
    s->obSeq[obSeqN] = static_cast<uint8_t>(slot);
    waveSync();
    obSeqN++;
    bool exists;
    const int at = findStart(slot, &exists);
    if (!exists) {
      if (obStartN >= kObCap) return fail(FMT_E_CAPACITY);
      for (int i = obStartN; i > at; i--) {
        const uint8_t v = s->obStart[i - 1];
        waveSync();
        s->obStart[i] = v;
      }
      s->obStart[at] = static_cast<uint8_t>(slot);
      waveSync();
      obStartN++;
    }
    return true;
  }

  // Obliterates.setMinSeq (mergeTree.ts:537-545), before zamboni: drop obliterates at/below minSeq
  // from both lists and remove their references.
  FMT_DEV void obSetMinSeq() {
    int k = 0;
    for (; k < obSeqN && uni(s->ob[uni(static_cast<int>(s->obSeq[k]))].seq) <= minSeq; k++) {
      const int slot = uni(static_cast<int>(s->obSeq[k]));
      bool exists;
      const int at = findStart(slot, &exists);
      if (exists) {
        for (int i = at; i + 1 < obStartN; i++) {
          const uint8_t v = s->obStart[i + 1];
          waveSync();
          s->obStart[i] = v;
        }
        waveSync();
        obStartN--;
      }
      s->ob[slot].startId = 0;  // removeLocalReferencePosition
      s->ob[slot].endId = 0;
      waveSync();
      if (!exists) continue;  // still listed in startOrdered: its slot stays taken
      obUsed &= ~(1ull << slot);
    }
    if (k > 0) {
      for (int i = 0; i + k < obSeqN; i++) {
        const uint8_t v = s->obSeq[i + k];
        waveSync();
        s->obSeq[i] = v;
      }
      waveSync();
      obSeqN -= k;
    }
  }

  // blockInsert's obliterate branch (mergeTree.ts:1642-1746) for the new leaf k: every overlapping
  // obliterate the inserter had not seen (seq > refSeq); when one is from another client and the
  // newest is not the inserter's own, the leaf starts out removed by those other clients' ones.
  FMT_DEV void obliterateOnInsert(int k, int refSeq, int client, bool record) {
    int minSeqOther = kNotRemoved, newestSeq = -1, newestClient = -1;
    uint64_t mask = 0;
    bool any = false;
    for (int i = 0; i < obStartN; i++) {  // Obliterates.findOverlapping (:566-582)
      const int slot = uni(static_cast<int>(s->obStart[i]));
      const int si = leafOf(uni(s->ob[slot].startId));
      if (!(si >= 0 && si <= k)) break;
      const int ei = leafOf(uni(s->ob[slot].endId));
      if (!(ei >= 0 && ei >= k)) continue;
      const int oseq = uni(s->ob[slot].seq), ocl = uni(s->ob[slot].client);
      if (oseq <= refSeq) continue;
      if (ocl != client) {
        any = true;
        mask |= 1ull << ocl;
        if (oseq < minSeqOther) minSeqOther = oseq;
      }
      if (oseq > newestSeq) {
        newestSeq = oseq;
        newestClient = ocl;
      }
    }
    if (any && newestClient != client) {
      writeField(k, 2, static_cast<uint32_t>(minSeqOther));
      writeField(k, 3, static_cast<uint32_t>(mask));
      if constexpr (C::kWords > 5) writeField(k, 5, static_cast<uint32_t>(mask >> 32));
      // SnapshotV1: the leaf's stamps are overlappingAcked sorted by seq (:1715-1725); the first is
      // rm_seq, every other one is a remove-order entry (the host sorts a leaf's entries by seq)
      if constexpr (Rm) {
        if (record) {
          const uint32_t id = fId(readField(k, 4));
          bool firstSkipped = false;
          for (int i = 0; i < obStartN && status == FMT_OK; i++) {
            const int slot = uni(static_cast<int>(s->obStart[i]));
            const int si = leafOf(uni(s->ob[slot].startId));
            if (!(si >= 0 && si <= k)) break;
            const int ei = leafOf(uni(s->ob[slot].endId));
            if (!(ei >= 0 && ei >= k)) continue;
            const int oseq = uni(s->ob[slot].seq), ocl = uni(s->ob[slot].client);
            if (oseq <= refSeq || ocl == client) continue;
            if (!firstSkipped && oseq == minSeqOther) {
              firstSkipped = true;
              continue;
            }
            rmAppend(id, ocl, oseq, FMT_MT_RM_SLICE);
          }
        }
      }
    }
  }

  // ------------------------------------------------------------------ relative positions
  // posFromRelativePos (mergeTree.ts:1462-1483): the marker whose "markerId" property holds the id
  // (idToMarker: markers stay findable until zamboni unlinks them; with ids unique per document that
  // is every marker leaf still in the tree), its start in the op's perspective, then the side and
  // offset. Returns -1 when no marker holds the id, or when it is removed (getMarkerFromId,
  // mergeTree.ts:1450-1453, returns undefined for a marker with a remove stamp).
  FMT_DEV int posFromRelativePos(uint32_t idx, int refSeq, int client) {
    const uint32_t mid = uni(loadCoherent(&in.relpos[idx].marker_id));
    const int offset = static_cast<int>(uni(loadCoherent(reinterpret_cast<const uint32_t*>(&in.relpos[idx].offset))));
    const bool before = (uni(loadCoherent(&in.relpos[idx].flags)) & FMT_MT_REL_BEFORE) != 0;
    if (mid == FMT_MT_NO_MARKER || in.markerKey == FMT_MT_NO_MARKER) return -1;
    const uint32_t want = (in.markerKey << 16) | (mid & 0xFFFFu);
    const int nr = rows();
    Lane<uint32_t> hits;
    FOR_LANES(l) {
      uint32_t m = 0;
      FOR_ROWS(r, 0, nr) {
        const uint32_t pid = propsL(l, r);
        if (r * 64 + l < n && fMarker(LANE(W[4])[r]) && pid != kPropsUndef && mid <= 0xFFFFu) {
          const uint32_t cnt = s->props[pid].n;
          bool f = false;
          for (uint32_t k = 0; k < cnt && k < static_cast<uint32_t>(kKeysMax); k++) f = f || setKv(static_cast<int>(pid), k) == want;
          if (f) m |= 1u << r;
        }
      }
      LANE(hits) = m;
    }
    // several markers with one id (ids are meant to be unique): the last inserted one, as
    // idToMarker.set on insert leaves it
    int j = -1, best = -1;
    for (Lane<uint32_t> todo = hits;;) {
      const int k = firstSet(todo, nr);
      if (k < 0) break;
      FOR_LANES(l) {
        if (l == (k & 63)) LANE(todo) &= ~(1u << (k >> 6));
      }
      const int ins = static_cast<int>(readField(k, 1));
      if (ins >= best) {
        best = ins;
        j = k;
      }
    }
    if (j < 0 || static_cast<int32_t>(readField(j, 2)) != kNotRemoved) return -1;
    Lane<VR> vis, st;
    visLengths(refSeq, client, vis, nr);
    scanRows(vis, st, nr);
    int pos = static_cast<int>(readlane(selectRow(st, j >> 6), j & 63));
    if (before) pos -= offset;
    else pos += static_cast<int>(fLen(readField(j, 0))) + offset;
    return pos;
  }

  // getValidOpRange (client.ts:758-767): an undefined pos1 / pos2 comes from relativePos1 / 2.
  FMT_DEV bool resolveRelative(fmt_mt_op& op) {
    for (int k = 0; k < 2; k++) {
      if ((op.flags & (k == 0 ? FMT_MT_F_REL1 : FMT_MT_F_REL2)) == 0) continue;
      const int32_t idx = k == 0 ? op.pos1 : op.pos2;
      const int pos = idx >= 0 && static_cast<uint32_t>(idx) < in.nRelpos
                          ? posFromRelativePos(static_cast<uint32_t>(idx), op.ref_seq, op.client)
                          : -1;
      if (pos < 0) {
        fail(FMT_E_DATA);
        return false;
      }
      if (k == 0) op.pos1 = pos;
      else op.pos2 = pos;
    }
    return true;
  }

  // One member op of a remote message (client.ts:1291-1327).
  // SnapshotLoader.loadBody's append of one body-chunk segment (FMT_MT_F_LOADSEG,
  // snapshotLoader.ts:287-309): insertSegments at the local length (every acked, not removed leaf)
  // from PriorPerspective(UniversalSequenceNumber, client) with stamp {seq, client}; the segment keeps
  // specToSegment's remove stamps (snapshot_info row op.pos1).
  FMT_DEV void loadBodySegment(const fmt_mt_op& op, const Lane<uint32_t>& text0) {
    if (in.infoAll == nullptr || op.pos1 < 0 || static_cast<uint64_t>(op.pos1) >= in.nInfoAll) {
      fail(FMT_E_DATA);
      return;
    }
    const int client = op.client == FMT_MT_CLIENT_NONCOLLAB ? FMT_NON_COLLAB_CLIENT : static_cast<int>(op.client);
    const int nr = rows();
    Lane<uint32_t> acc;
    FOR_LANES(l) { LANE(acc) = 0u; }
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        if (static_cast<int32_t>(LANE(W[2])[r]) == kNotRemoved) LANE(acc) += fLen(LANE(W[0])[r]);
      }
    }
    uint32_t local;
    waveExclusiveSum(acc, &local);
    fmt_mt_op o = op;
    o.pos1 = static_cast<int32_t>(local);
    o.ref_seq = 0;
    const int k = insertText(o, text0, client, (op.flags & FMT_MT_F_GROUP_CONT) == 0);
    if (k < 0 || status != FMT_OK) return;
    const fmt_mt_snapshot_info inf = in.infoAll[op.pos1];
    int32_t rm = kNotRemoved;
    uint64_t mask = 0;
    for (uint32_t t = 0; t < inf.rm_count; t++) {
      const fmt_mt_stamp st = in.stampsAll[inf.rm_first + t];
      rm = uni(st.seq) < rm ? uni(st.seq) : rm;
      const int c = uni(st.client);
      if (c < 0 || c > kMaxClient) {  // (ids past this tier's sets: a bigger tier, up to the huge tier's 253)
        fail(c >= 0 && c <= kTopClient ? FMT_E_CAPACITY : FMT_E_UNSUPPORTED);
        return;
      }
      mask |= 1ull << c;
    }
    if (inf.rm_count) {
      writeField(k, 2, static_cast<uint32_t>(rm));
      writeField(k, 3, static_cast<uint32_t>(mask));
      if constexpr (C::kWords > 5) writeField(k, 5, static_cast<uint32_t>(mask >> 32));
    }
  }

  FMT_DEV void applyOp(const fmt_mt_op& op, const Lane<uint32_t>& text0) {
    const bool catchup = (op.flags & FMT_MT_F_CATCHUP) != 0;
    Lane<uint32_t> delta;  // catch-up: the segments of the op's delta event (row bitmask per lane)
    if (op.type == FMT_MT_INSERT) {
      const int k = insertText(op, text0);
      if (!catchup || k < 0) return;
      if constexpr (Ob) {  // an insert obliterated on arrival raises no delta (:1497-1508)
        if (static_cast<int32_t>(readField(k, 2)) != kNotRemoved) return;
      }
      FOR_LANES(l) { LANE(delta) = l == (k & 63) ? 1u << (k >> 6) : 0u; }  // the new segment (:1497-1508)
    } else {
      if (!applyRange(op, delta)) return;
    }
    // one call site: the recording is inlined once; a sided obliterate raises OBLITERATE (:2249-2253)
    recordCatchup(delta, op.type == FMT_MT_OBLITERATE_SIDED ? FMT_MT_OBLITERATE : op.type);
  }

  // Remove / annotate (after their boundary splits); fills `delta` for catch-up ops. Returns true
  // when a catch-up recording should follow.
  // (localOp, Loc: the local client's submission, its segments joining pending group `group`)
  FMT_DEV bool applyRange(const fmt_mt_op& op, Lane<uint32_t>& delta, bool localOp = false, uint32_t group = 0) {
    const int refSeq = op.ref_seq, client = op.client, seq = op.seq;
    const bool catchup = (op.flags & FMT_MT_F_CATCHUP) != 0;
    bool obliterate = false;
    if constexpr (Ob) obliterate = op.type == FMT_MT_OBLITERATE || op.type == FMT_MT_OBLITERATE_SIDED;
    const int start = op.pos1, end = op.pos2;
    Lane<uint32_t> hits;
    FOR_LANES(l) { LANE(hits) = 0u; }
    int nr;
    if (!obliterate) {
      // One view scan serves both boundary splits (ensureIntervalBoundary, mergeTree.ts:1798-1808)
      // and nodeMap's hit set (:2961-3020, leaves of positive view length inside [start, end)):
      // a split moves no view start, it only adds a leaf whose view start is the boundary.
      nr = rows();
      Lane<VR> vis, st;
      visLengths(refSeq, client, vis, nr);
      scanRows(vis, st, nr);
      stamp(kPfScan);
      FOR_ROWS(r, 0, nr) {
        FOR_LANES(l) {
          const int sp = static_cast<int>(LANE(st)[r]);
          if (LANE(vis)[r] > 0 && sp >= start && sp < end) LANE(hits) |= 1u << r;
        }
      }
      int s1 = 0, s2 = 0;
      const int j1 = containing(vis, st, start, nr, &s1);
      const int j2 = containing(vis, st, end, nr, &s2);
      if (j1 >= 0) {  // the right part of j1 starts at `start`: a hit
        if (!splitLeafAt(j1, start - s1)) return false;
        hits = maskInsert(hits, j1 + 1, true);
      }
      if (j2 >= 0) {  // the right part of j2 starts at `end`: not a hit
        const int jj = j1 < 0 || j1 > j2 ? j2 : (j1 < j2 ? j2 + 1 : j1 + 1);
        const int off = j1 == j2 ? end - start : end - s2;
        if (!splitLeafAt(jj, off)) return false;
        hits = maskInsert(hits, jj + 1, false);
      }
      nr = rows();
    } else {
      // obliterateRangeSided (mergeTree.ts:2083-2260). Places {pos, before?}: a non-sided op is
      // {pos1, Before} .. {pos2 - 1, After} (:2282-2286); a sided one carries its sides in flags
      // (client.ts:680-700). The boundaries are the places' Before edges (:2090-2091).
      const bool sided = op.type == FMT_MT_OBLITERATE_SIDED;
      const bool sB = !sided || (op.flags & FMT_MT_F_START_BEFORE) != 0;
      const bool eB = sided && (op.flags & FMT_MT_F_END_BEFORE) != 0;
      const int sPl = op.pos1, ePl = sided ? op.pos2 : op.pos2 - 1;
      const int startPos = sB ? sPl : sPl + 1, endPos = eB ? ePl : ePl + 1, endW = ePl + 1;
      if (!splitAt(startPos, refSeq, client)) return false;
      if (!splitAt(endPos, refSeq, client)) return false;
      nr = rows();
      Lane<VR> vis, st;
      visLengths(refSeq, client, vis, nr);
      scanRows(vis, st, nr);
      stamp(kPfScan);
      // nodeMap(start.pos, end.pos + 1) under RemoteObliteratePerspective visits a leaf when it has
      // length in the op's view or is not removed at all (so concurrent inserts strictly inside are
      // caught), positions from the op's view: st < end.pos + 1, start.pos < st + vis. markRemoved
      // skips the exclusive endpoints (:2145-2152): a start After leaf whose full length ends at
      // the start boundary, an end Before leaf present in the op's view that starts at the end
      // boundary. Endpoint references go to the leaves holding start.pos and end.pos in the op's
      // view (getContainingSegment, :858-886).
      int sLeaf = -1, eLeaf = -1, sOff = 0, eOff = 0;
      FOR_ROWS(r, 0, nr) {
        Lane<bool> ps, pe;
        FOR_LANES(l) {
          const int sp = static_cast<int>(LANE(st)[r]), v = static_cast<int>(LANE(vis)[r]);
          const bool removed = static_cast<int32_t>(LANE(W[2])[r]) != kNotRemoved;
          const bool excl = (!sB && startPos == sp + static_cast<int>(fLen(LANE(W[0])[r]))) ||
                            (eB && endPos == sp && v > 0);
          if (!(v == 0 && removed) && !excl && r * 64 + l < n && sp < endW && sPl < sp + v) LANE(hits) |= 1u << r;
          LANE(ps) = v > 0 && sp <= sPl && sPl < sp + v;
          LANE(pe) = v > 0 && sp <= ePl && ePl < sp + v;
        }
        const uint64_t ms = ballot(ps), me = ballot(pe);
        if (sLeaf < 0 && ms != 0) {
          sLeaf = r * 64 + ctz64(ms);
          sOff = sPl - static_cast<int>(readlane(row(st, r), ctz64(ms)));
        }
        if (eLeaf < 0 && me != 0) {
          eLeaf = r * 64 + ctz64(me);
          eOff = ePl - static_cast<int>(readlane(row(st, r), ctz64(me)));
        }
      }
      if (sLeaf < 0 || eLeaf < 0) {  // "segments cannot be undefined" (0xa3f)
        fail(FMT_E_DATA);
        return false;
      }
      if (!obAdd(fId(readField(sLeaf, 4)), sOff, fId(readField(eLeaf, 4)), eOff, seq, client)) return false;
    }
    FOR_LANES(l) { LANE(delta) = 0u; }
    if (Rm && (op.type == FMT_MT_REMOVE || obliterate) && (op.flags & FMT_MT_F_RMORDER) != 0) {  // recorded in rmFlush
      FOR_LANES(l) {
        uint32_t m = 0;
        FOR_ROWS(r, 0, nr) {
          if (((LANE(hits) >> r) & 1u) && static_cast<int32_t>(LANE(W[2])[r]) != kNotRemoved) m |= 1u << r;
        }
        LANE(rmHits) = m;
      }
      rmHitsSet = true;
    }
    if (op.type == FMT_MT_REMOVE || obliterate) {
      // markRangeRemoved (mergeTree.ts:2292-2383): first remove stays the lowest seq; the delta
      // (removedSegments) is the hit leaves not removed before this op (:2314-2321)
      FOR_ROWS(r, 0, nr) {
        FOR_LANES(l) {
          if ((LANE(hits) >> r) & 1u) {
            const int32_t rm = static_cast<int32_t>(LANE(W[2])[r]);
            if (rm == kNotRemoved) LANE(delta) |= 1u << r;
            LANE(W[2])[r] = static_cast<uint32_t>(rm < seq ? rm : seq);
            if (C::kWords > 5 && client >= 32) LANE(W[C::kWords > 5 ? 5 : 3])[r] |= 1u << (client - 32);
            else LANE(W[3])[r] |= 1u << client;
          }
        }
      }
    } else {
      // annotateRange (mergeTree.ts:2009-2081): one prop-set transition per distinct old set
      if constexpr (Adj && !Loc) {  // each hit leaf's PropertiesManager, in nodeMap order
        for (Lane<uint32_t> t = hits;;) {
          const int j = firstSet(t, nr);
          if (j < 0 || status != FMT_OK) break;
          FOR_LANES(l) {
            if (l == (j & 63)) LANE(t) &= ~(1u << (j >> 6));
          }
          pmAnnotate(j, op.payload, seq);
        }
        if (status != FMT_OK) return false;
      }
      Lane<uint32_t> todo = hits;
      if constexpr (Loc) {
        if (localOp) {  // each hit leaf's manager records the local change (segmentPropertiesManager.ts:209-211)
          for (Lane<uint32_t> t = hits;;) {
            const int j = firstSet(t, nr);
            if (j < 0 || status != FMT_OK) break;
            FOR_LANES(l) {
              if (l == (j & 63)) LANE(t) &= ~(1u << (j >> 6));
            }
            locPmLocal(j, op.payload, group);
          }
          if (status != FMT_OK) return false;
        } else if (pmN > 0 || (Adj && opHasAdjust(op.payload))) {
          // leaves whose managers hold local changes keep those keys' local values; annotate-adjust
          // batches: every leaf an adjust reaches, or whose manager has records, runs handleProperties
          // in full (remote changes join the remote list)
          const bool adj = Adj && opHasAdjust(op.payload);
          for (Lane<uint32_t> t = hits;;) {
            const int j = firstSet(t, nr);
            if (j < 0 || status != FMT_OK) break;
            FOR_LANES(l) {
              if (l == (j & 63)) LANE(t) &= ~(1u << (j >> 6));
            }
            const uint32_t leaf = fId(readField(j, 4));
            if (!adj && pmFind(leaf, 0u, Adj ? 0u : 0x30000u) < 0) continue;  // (no manager: the shared path)
            uint32_t nw;
            if constexpr (Adj) nw = locAdjRemote(j, op.payload, seq);
            else nw = locRemoteAnnotate(j, op.payload);
            if (status != FMT_OK) return false;
            const int rj = j >> 6, lane = j & 63;
            FOR_ROWS(r, rj, rj + 1) {
              FOR_LANES(l) {
                if (l == lane) {
                  setPropsL(l, r, nw);
                  LANE(todo) &= ~(1u << r);
                }
              }
            }
          }
          if (status != FMT_OK) return false;
        }
      }
      for (;;) {
        const int j = firstSet(todo, nr);
        if (j < 0) break;
        const uint32_t old = propsAt(j);
        const uint32_t nw = applyProps<true>(old, op.payload);
        if (status != FMT_OK) return false;
        FOR_ROWS(r, 0, nr) {
          FOR_LANES(l) {
            if (((LANE(todo) >> r) & 1u) && propsL(l, r) == old) {
              setPropsL(l, r, nw);
              LANE(todo) &= ~(1u << r);
            }
          }
        }
      }
      if (catchup) {  // deltaSegments: annotated and not removed (mergeTree.ts:2045-2047)
        FOR_ROWS(r, 0, nr) {
          FOR_LANES(l) {
            if (((LANE(hits) >> r) & 1u) && static_cast<int32_t>(LANE(W[2])[r]) == kNotRemoved) LANE(delta) |= 1u << r;
          }
        }
      }
    }
    stamp(kPfRange);
    if constexpr (Loc) {
      if (localOp) {  // addToPendingList for every hit leaf, in nodeMap order (mergeTree.ts:2048-2055, 2336-2341)
        for (Lane<uint32_t> t = hits; status == FMT_OK;) {
          const int j = firstSet(t, nr);
          if (j < 0) break;
          FOR_LANES(l) {
            if (l == (j & 63)) LANE(t) &= ~(1u << (j >> 6));
          }
          pendAdd(j, 1);
          recAppend(fId(readField(j, 4)), group);
        }
        return false;
      }
    }
    lruForHits(hits, seq, nr);
    stamp(kPfLru);
    return catchup && status == FMT_OK;
  }


  // ------------------------------------------------------------------ f4: the local client (Loc)
  // The document is replayed from the perspective of its own client, short id 0. Its submissions are
  // stamped {UnassignedSequenceNumber, 0, localSeq}: W1 / W2 hold FMT_MT_LOCAL_SEQ_BASE | localSeq,
  // above every sequence number, so PriorPerspective(refSeq, c) of any remote client sees neither
  // a pending insert nor a pending remove (perspective.ts:80-93), LocalReconnectingPerspective(seq,
  // 0, k) is visLengths(LOCAL_SEQ_BASE | k, none) (perspective.ts:103-118), and the local view is
  // visLengths(kLocalView, 0). A pending op's segments are a SegmentGroup (mergeTree.ts:1410-1447):
  // a queue entry in the group slab plus one record per segment in the record slab, in the order the
  // segments joined (splits append the right part, segmentGroupCollection.ts:25-59); W[kPendW]
  // counts the groups holding a leaf, which zamboni must not touch (zamboni.ts:148).
  static constexpr int32_t kLocalView = 0x7FFFFFFE;  // every stamp has occurred
  static constexpr int kGW = 8;                        // words per pending group (LocalTables::groups)
  uint32_t locSeq = 0;        // collabWindow.localSeq
  int gHead = 0, gTail = 0;   // the pending queue: group serials [gHead, gTail) of the group slab
  int recN = 0;               // group records in use (deleted ones included)
  bool recFrozen = false;     // (regeneration iterates records by index: no compaction meanwhile)
  uint32_t regenN = 0, regenTextN = 0;
  bool normSet = false;       // client.ts:1414 lastNormalization
  int normRef = 0;
  uint32_t normLocal = 0;

  FMT_DEV static bool isLocalSeq(uint32_t w) { return static_cast<int32_t>(w) >= FMT_MT_LOCAL_SEQ_BASE && static_cast<int32_t>(w) != kNotRemoved; }
  FMT_DEV uint32_t* gBase() const { return in.loc->groups + kGW * in.loc->groupOffs[in.doc]; }
  FMT_DEV int gCap() const { return static_cast<int>(in.loc->groupOffs[in.doc + 1] - in.loc->groupOffs[in.doc]); }
  FMT_DEV uint32_t gWord(int g, int w) const { return uni(loadCoherent(gBase() + kGW * g + w)); }
  FMT_DEV uint32_t* rBase() const { return in.loc->recs + 2 * in.loc->recOffs[in.doc]; }
  FMT_DEV int rCap() const { return static_cast<int>(in.loc->recOffs[in.doc + 1] - in.loc->recOffs[in.doc]); }
  FMT_DEV uint32_t rWord(int i, int w) const { return uni(loadCoherent(rBase() + 2 * i + w)); }
  FMT_DEV void rSet(int i, int w, uint32_t v) {
    uint32_t* R = rBase() + 2 * i + w;
    FOR_LANES(l) {
      if (l == 0) storeGlobal(R, v);
    }
  }

  // Drops deleted group records (leaf id 0), keeping the order.
  FMT_DEV void recCompact() {
    uint32_t* R = rBase();
    int out = 0;
    for (int base = 0; base < recN; base += 64) {
      Lane<uint32_t> w0, w1;
      Lane<bool> live;
      FOR_LANES(l) {
        const int i = base + l;
        LANE(w0) = i < recN ? loadCoherent(R + 2 * i) : 0u;
        LANE(w1) = i < recN ? loadCoherent(R + 2 * i + 1) : 0u;
        LANE(live) = LANE(w0) != 0u;
      }
      const uint64_t m = ballot(live);
      waveSync();
      FOR_LANES(l) {
        if (LANE(live)) {
          const int at = out + __builtin_popcountll(m & ((1ull << l) - 1ull));
          storeGlobal(R + 2 * at, LANE(w0));
          storeGlobal(R + 2 * at + 1, LANE(w1));
        }
      }
      waveSync();
      out += __builtin_popcountll(m);
    }
    recN = out;
  }

  FMT_DEV bool recAppend(uint32_t leaf, uint32_t g) {
    if (recN >= rCap() && !recFrozen) recCompact();
    if (recN >= rCap()) return fail(FMT_E_CAPACITY);
    uint32_t* R = rBase() + 2 * recN;
    FOR_LANES(l) {
      if (l < 2) storeGlobal(R + l, l == 0 ? leaf : g);
    }
    waveSync();
    recN++;
    return true;
  }

  // First live record at or after `from` of group g (leaf == 0: any leaf), or -1.
  FMT_DEV int recFind(uint32_t g, int from, uint32_t leaf = 0u) const {
    const uint32_t* R = rBase();
    for (int base = from; base < recN; base += 64) {
      Lane<bool> p;
      FOR_LANES(l) {
        const int i = base + l;
        const uint32_t lf = i < recN ? loadCoherent(R + 2 * i) : 0u;
        LANE(p) = i < recN && lf != 0u && loadCoherent(R + 2 * i + 1) == g && (leaf == 0u || lf == leaf);
      }
      const uint64_t m = ballot(p);
      if (m != 0) return base + ctz64(m);
    }
    return -1;
  }

  // SegmentGroupCollection.copyTo: the split's right part joins every group of the left, in order.
  FMT_DEV void recCopy(uint32_t from, uint32_t to) {
    if (!recFrozen) recCompact();  // (records keep their indices while appending)
    const int end = recN;
    for (int base = 0; base < end && status == FMT_OK; base += 64) {
      Lane<bool> p;
      Lane<uint32_t> g;
      FOR_LANES(l) {
        const int i = base + l;
        LANE(p) = i < end && loadCoherent(rBase() + 2 * i) == from;
        LANE(g) = i < end ? loadCoherent(rBase() + 2 * i + 1) : 0u;
      }
      for (uint64_t m = ballot(p); m != 0 && status == FMT_OK; m &= m - 1) recAppend(to, readlane(g, ctz64(m)));
    }
  }

  // A new pending group at the queue's tail; its serial, or -1. Group words: localSeq, type | marker
  // << 8, payload, pos2, the refSeq its op was submitted at (in flight: sequence.ts:468-499).
  FMT_DEV int groupPush(uint32_t localSeq, uint32_t typeFlags, uint32_t payload, int32_t pos2, int32_t inflightRef) {
    if (gTail >= gCap() && gHead > 0 && !recFrozen) groupCompact();
    if (gTail >= gCap()) {
      fail(FMT_E_CAPACITY);
      return -1;
    }
    uint32_t* G = gBase() + kGW * gTail;
    FOR_LANES(l) {
      if (l < kGW)
        storeGlobal(G + l, l == 0 ? localSeq : l == 1 ? typeFlags : l == 2 ? payload : l == 3 ? static_cast<uint32_t>(pos2)
                                                                         : l == 4 ? static_cast<uint32_t>(inflightRef) : 0u);
    }
    waveSync();
    return gTail++;
  }

  // The queue back to serial 0 (records renumbered).
  FMT_DEV void groupCompact() {
    const int cnt = gTail - gHead;
    uint32_t* G = gBase();
    for (int base = 0; base < kGW * cnt; base += 64) {
      Lane<uint32_t> v;
      FOR_LANES(l) { LANE(v) = base + l < kGW * cnt ? loadCoherent(G + kGW * gHead + base + l) : 0u; }
      waveSync();
      FOR_LANES(l) {
        if (base + l < kGW * cnt) storeGlobal(G + base + l, LANE(v));
      }
      waveSync();
    }
    uint32_t* R = rBase();
    for (int base = 0; base < recN; base += 64) {
      FOR_LANES(l) {
        const int i = base + l;
        if (i < recN && loadCoherent(R + 2 * i) != 0u) storeGlobal(R + 2 * i + 1, loadCoherent(R + 2 * i + 1) - static_cast<uint32_t>(gHead));
      }
    }
    waveSync();
    gTail = cnt;
    gHead = 0;
  }

  FMT_DEV void pendAdd(int j, int d) {
    if constexpr (!Loc) return;
    const int rj = j >> 6, lane = j & 63;
    FOR_ROWS(r, rj, rj + 1) {
      FOR_LANES(l) {
        if (l == lane) LANE(W[kPendW])[r] = static_cast<uint32_t>(static_cast<int>(LANE(W[kPendW])[r]) + d);
      }
    }
  }

  // getLength() from the local perspective: every leaf not removed.
  FMT_DEV int localLength() const {
    const int nr = rows();
    Lane<uint32_t> acc;
    FOR_LANES(l) { LANE(acc) = 0u; }
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        if (static_cast<int32_t>(LANE(W[2])[r]) == kNotRemoved) LANE(acc) += fLen(LANE(W[0])[r]);
      }
    }
    uint32_t total;
    waveExclusiveSum(acc, &total);
    return static_cast<int>(total);
  }

  // --- the local client's PropertiesManager records: heads {leaf, key, 0, msnConsensus}, local
  // changes {leaf, key | 0x20000, group serial, change}; with annotate-adjust (Adj) also the remote
  // changes {leaf, key | 0x10000, seq, value after it} of the shared Adj model above. A change word is
  // a raw value id, or kLocAdjust | the adjust row (segmentPropertiesManager.ts:45-52 PropertyChange).
  static constexpr uint32_t kLocAdjust = 0x80000000u;
  FMT_DEV int locHead(uint32_t leaf, uint32_t key) const { return pmFind(leaf, key, 0x3FFFFu); }
  FMT_DEV int locLocalFirst(uint32_t leaf, uint32_t key) const { return pmFind(leaf, key | 0x20000u, 0x3FFFFu); }
  FMT_DEV int locLocalLast(uint32_t leaf, uint32_t key) const {
    int last = -1;
    for (int i = locLocalFirst(leaf, key); i >= 0; i = pmFind(leaf, key | 0x20000u, 0x3FFFFu, i + 1)) last = i;
    return last;
  }
  // The leaf's current value of `key` (0: absent) from its prop set.
  FMT_DEV uint32_t keyValue(uint32_t props, uint32_t key) const {
    if (props == kPropsUndef) return 0u;
    const uint32_t cnt = uni(s->props[props].n);
    uint32_t v = 0u;
    for (uint32_t k = 0; k < cnt && k < static_cast<uint32_t>(kKeysMax); k++) {
      const uint32_t e = uni(setKv(static_cast<int>(props), k));
      if ((e >> 16) == key) v = e & 0xFFFFu;
    }
    return v;
  }
  // The working set with `key` set to v (0: deleted; a new key goes last); returns the count.
  FMT_DEV uint32_t workSetKey(uint32_t cnt, uint32_t key, uint32_t v) {
    uint32_t pos = cnt;
    for (uint32_t k = 0; k < cnt; k++)
      if ((uni(s->kvWork[k]) >> 16) == key) pos = k;
    if (v == 0u) {
      if (pos < cnt) {
        for (uint32_t k = pos; k + 1 < cnt; k++) {
          const uint32_t x = uni(s->kvWork[k + 1]);
          waveSync();
          FOR_LANES(l) {
            if (l == 0) s->kvWork[k] = x;
          }
        }
        cnt--;
      }
    } else if (pos < cnt) {
      FOR_LANES(l) {
        if (l == 0) s->kvWork[pos] = (key << 16) | v;
      }
    } else if (cnt < static_cast<uint32_t>(kKeysMax)) {
      FOR_LANES(l) {
        if (l == 0) s->kvWork[cnt] = (key << 16) | v;
      }
      cnt++;
    } else {
      fail(kCapFinal);
    }
    waveSync();
    return cnt;
  }

  // The op's change at payload word t (an adjust takes the next word, its row): the change word, and
  // the index of the op's next change.
  FMT_DEV uint32_t locChange(uint32_t t, uint32_t b, uint32_t* next) {
    const uint32_t e = uni(in.propsKv[t]);
    *next = t + 1;
    if ((e & 0xFFFFu) != FMT_MT_VALUE_ADJUST) return e & 0xFFFFu;
    if (!Adj || t + 1 >= b) {  // (adjusts: the Adj variants; a row must follow)
      fail(Adj ? FMT_E_DATA : FMT_E_UNSUPPORTED);
      return 0u;
    }
    *next = t + 2;
    return kLocAdjust | uni(in.propsKv[t + 1]);
  }
  // computePropertyValue of one change onto v (segmentPropertiesManager.ts:54-78).
  FMT_DEV uint32_t locApply(uint32_t v, uint32_t change) {
    if ((change & kLocAdjust) == 0u) return change;
    if constexpr (Adj) {
      const uint32_t r = adjustFold(in.adj, in.doc, v, change & ~kLocAdjust);
      if (r == kAdjFailData || r == kAdjFailCap) {
        fail(r == kAdjFailData ? FMT_E_DATA : kCapFinal);
        return 0u;
      }
      return r;
    }
    fail(FMT_E_UNSUPPORTED);
    return 0u;
  }
  // msnConsensus folded with the remote changes: the last remote change's value, else msnConsensus.
  FMT_DEV uint32_t locRemoteTop(uint32_t leaf, uint32_t key) {
    const int h = locHead(leaf, key);
    uint32_t v = pmWord(h, 3);
    for (int i = pmFind(leaf, key | 0x10000u, 0x3FFFFu, h + 1); i >= 0; i = pmFind(leaf, key | 0x10000u, 0x3FFFFu, i + 1))
      v = pmWord(i, 3);
    return v;
  }
  // ... then with the local changes, oldest first: properties[key] (:221-225).
  FMT_DEV uint32_t locFoldLocal(uint32_t leaf, uint32_t key, uint32_t v) {
    for (int i = locLocalFirst(leaf, key); i >= 0 && status == FMT_OK; i = pmFind(leaf, key | 0x20000u, 0x3FFFFu, i + 1))
      v = locApply(v, pmWord(i, 3));
    return v;
  }
  FMT_DEV bool locHasRemote(uint32_t leaf, uint32_t key) { return pmFind(leaf, key | 0x10000u, 0x3FFFFu) >= 0; }

  // handleProperties for a local change (segmentPropertiesManager.ts:199-211): a key's entry starts at
  // its current value, the change joins its local list. (The visible set follows the op's values,
  // applied by the caller: a local adjust folds onto the current value, which is the fold of
  // everything before it.)
  FMT_DEV void locPmLocal(int j, uint32_t opId, uint32_t g) {
    const uint32_t leaf = fId(readField(j, 4));
    const uint32_t props = propsAt(j);
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a, nx; t < b && status == FMT_OK; t = nx) {
      const uint32_t key = uni(in.propsKv[t]) >> 16;
      const uint32_t ch = locChange(t, b, &nx);
      if (status != FMT_OK) return;
      if (locHead(leaf, key) < 0 && !pmAppend(leaf, key, 0, keyValue(props, key))) return;
      if (!pmAppend(leaf, key | 0x20000u, static_cast<int>(g), ch)) return;
    }
    if constexpr (Adj) pmUpdateMsn(leaf, minSeq);
  }

  // handleProperties for a remote change in an annotate-adjust batch (segmentPropertiesManager.ts:
  // 199-238): the key's entry starts at its current value; a raw change folds into msnConsensus while
  // no remote change is pending, else it (and any adjust) joins the remote list with the value it
  // leaves; properties[key] = that fold, then the key's local changes; updateMsn(minSeq). Returns the
  // leaf's new prop set.
  FMT_DEV uint32_t locAdjRemote(int j, uint32_t opId, int seq) {
    const uint32_t leaf = fId(readField(j, 4));
    uint32_t cnt = loadWork(propsAt(j));
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a, nx; t < b && status == FMT_OK; t = nx) {
      const uint32_t key = uni(in.propsKv[t]) >> 16;
      const uint32_t ch = locChange(t, b, &nx);
      if (status != FMT_OK) return 0u;
      uint32_t prev = 0u;
      for (uint32_t k = 0; k < cnt; k++)
        if ((uni(s->kvWork[k]) >> 16) == key) prev = uni(s->kvWork[k]) & 0xFFFFu;
      int h = locHead(leaf, key);
      if (h < 0) {
        if (!pmAppend(leaf, key, 0, prev)) return 0u;
        h = pmN - 1;
      }
      if ((ch & kLocAdjust) == 0u && !locHasRemote(leaf, key)) {
        pmSet(h, 3, ch);
      } else {
        const uint32_t v = locApply(locRemoteTop(leaf, key), ch);
        if (status != FMT_OK || !pmAppend(leaf, key | 0x10000u, seq, v)) return 0u;
      }
      waveSync();
      const uint32_t v = locFoldLocal(leaf, key, locRemoteTop(leaf, key));
      if (status != FMT_OK) return 0u;
      cnt = workSetKey(cnt, key, v);
    }
    pmUpdateMsn(leaf, minSeq);
    return status == FMT_OK ? internWork(cnt) : 0u;
  }

  FMT_DEV bool opHasAdjust(uint32_t opId) const {
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a; t < b; t++)
      if ((uni(in.propsKv[t]) & 0xFFFFu) == FMT_MT_VALUE_ADJUST) return true;
    return false;
  }

  // A remote annotate on a leaf whose manager has local changes (segmentPropertiesManager.ts:213-227):
  // a key with local changes keeps its local value and folds the remote one into msnConsensus;
  // the others change as for any leaf. Returns the leaf's new prop set.
  FMT_DEV uint32_t locRemoteAnnotate(int j, uint32_t opId) {
    const uint32_t leaf = fId(readField(j, 4));
    uint32_t cnt = loadWork(propsAt(j));
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a; t < b && status == FMT_OK; t++) {
      const uint32_t e = uni(in.propsKv[t]);
      const uint32_t key = e >> 16;
      if ((e & 0xFFFFu) == FMT_MT_VALUE_ADJUST) {
        fail(FMT_E_UNSUPPORTED);
        return 0;
      }
      const int h = locHead(leaf, key);
      if (h >= 0) pmSet(h, 3, e & 0xFFFFu);
      else cnt = workSetKey(cnt, key, e & 0xFFFFu);
    }
    return status == FMT_OK ? internWork(cnt) : 0u;
  }

  // PropertiesManager.ack (segmentPropertiesManager.ts:248-267) + updateMsn: each key's oldest local
  // change leaves, msnConsensus takes the acknowledged value; a key left without changes loses its entry.
  // (Adj: a raw change folds into msnConsensus while no remote change is pending, else the change
  // joins the remote list at the ack's seq; then updateMsn with the message's minSeq, :248-267)
  FMT_DEV void locPmAck(uint32_t leaf, uint32_t opId, int seq, int msn) {
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a, nx; t < b && status == FMT_OK; t = nx) {
      const uint32_t key = uni(in.propsKv[t]) >> 16;
      const uint32_t ch = locChange(t, b, &nx);
      if (status != FMT_OK) return;
      const int c = locLocalFirst(leaf, key), h = locHead(leaf, key);
      if (c < 0 || h < 0) {  // "must have local change to ack" (0xa71)
        fail(FMT_E_DATA);
        return;
      }
      pmSet(c, 0, 0u);
      if constexpr (Adj) {
        waveSync();
        if ((ch & kLocAdjust) == 0u && !locHasRemote(leaf, key)) {
          pmSet(h, 3, ch);
        } else {
          const uint32_t v = locApply(locRemoteTop(leaf, key), ch);
          if (status != FMT_OK || !pmAppend(leaf, key | 0x10000u, seq, v)) return;
        }
        waveSync();
      } else {
        pmSet(h, 3, ch);
        waveSync();
        if (locLocalFirst(leaf, key) < 0) pmSet(h, 0, 0u);
        waveSync();
      }
    }
    if constexpr (Adj) pmUpdateMsn(leaf, msn);
  }

  // rollbackProperties (segmentPropertiesManager.ts:140-173, collaborating): each key of the op drops
  // its newest local change and takes the newest one left, else msnConsensus; a key left without
  // changes loses its entry. Sets the leaf's prop set.
  FMT_DEV void locPmRollback(int j, uint32_t opId) {
    const uint32_t leaf = fId(readField(j, 4));
    uint32_t cnt = loadWork(propsAt(j));  // (`seg.properties ??= {}`: a set even if empty)
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a, nx; t < b && status == FMT_OK; t = nx) {
      const uint32_t key = uni(in.propsKv[t]) >> 16;
      locChange(t, b, &nx);
      if (status != FMT_OK) return;
      const int h = locHead(leaf, key);
      if (h < 0) {  // "Pending changes must exist for rollback when collaborating" (0xa6f)
        fail(FMT_E_DATA);
        return;
      }
      const int c = locLocalLast(leaf, key);
      if (c >= 0) pmSet(c, 0, 0u);
      waveSync();
      uint32_t v;
      if constexpr (Adj) {  // computePropertyValue(msnConsensus, remote, local) (:157-162)
        v = locFoldLocal(leaf, key, locRemoteTop(leaf, key));
        if (locLocalFirst(leaf, key) < 0 && !locHasRemote(leaf, key)) pmSet(h, 0, 0u);
      } else {
        const int c2 = locLocalLast(leaf, key);
        v = c2 >= 0 ? pmWord(c2, 3) : pmWord(h, 3);
        if (c2 < 0) pmSet(h, 0, 0u);
      }
      waveSync();
      cnt = workSetKey(cnt, key, v);
    }
    if (status != FMT_OK) return;
    const uint32_t id = internWork(cnt);
    if (status != FMT_OK) return;
    const int rj = j >> 6, lane = j & 63;
    FOR_ROWS(r, rj, rj + 1) {
      FOR_LANES(l) {
        if (l == lane) setPropsL(l, r, id);
      }
    }
  }

  // insertSegmentLocal / removeRangeLocal / annotateRangeLocal (client.ts:273-355) after
  // getValidOpRange's local checks (client.ts:769-811: FMT_E_USAGE).
  FMT_DEV void applyLocal(const fmt_mt_op& op0, const Lane<uint32_t>& text0) {
    fmt_mt_op op = op0;
    const int length = localLength();
    if (op.type == FMT_MT_INSERT) {
      if (op.pos1 < 0 || op.pos1 > length) {
        fail(FMT_E_USAGE);
        return;
      }
      if (opLen(op) == 0) return;  // insertSegmentLocal: no segment, no op (client.ts:348-351)
    } else if (op.type == FMT_MT_REMOVE || op.type == FMT_MT_ANNOTATE) {
      if (op.pos1 < 0 || op.pos1 >= length || op.pos2 <= op.pos1) {
        fail(FMT_E_USAGE);
        return;
      }
    } else {
      fail(FMT_E_UNSUPPORTED);
      return;
    }
    if constexpr (Adj) {
      // annotateAdjustRangeLocal (client.ts:286-301): min greater than max is a UsageError (a JSON null
      // bound compares as 0)
      if (op.type == FMT_MT_ANNOTATE) {
        const uint32_t a = uni(in.propsOff[op.payload]), b = uni(in.propsOff[op.payload + 1]);
        for (uint32_t t = a; t + 1 < b; t++) {
          if ((uni(in.propsKv[t]) & 0xFFFFu) != FMT_MT_VALUE_ADJUST) continue;
          const uint32_t row = uni(in.propsKv[++t]);
          if (in.adj == nullptr || row >= in.adj->nAdjusts) {
            fail(FMT_E_DATA);
            return;
          }
          const fmt_mt_adjust* R = in.adj->adjusts + row;
          const uint32_t fl = uni(R->flags);
          const double mn = (fl & FMT_MT_ADJ_MIN_NULL) ? 0.0 : uniD(R->min), mx = (fl & FMT_MT_ADJ_MAX_NULL) ? 0.0 : uniD(R->max);
          if ((fl & FMT_MT_ADJ_MIN) && (fl & FMT_MT_ADJ_MAX) && mn > mx) {
            fail(FMT_E_USAGE);
            return;
          }
        }
      }
    }
    const uint32_t ls = ++locSeq;  // mintNextLocalOperationStamp (mergeTreeNodes.ts:685-695)
    const uint32_t marker = (op.flags & FMT_MT_F_MARKER) != 0 ? 1u : 0u;
    const int g = groupPush(ls, static_cast<uint32_t>(op.type) | (marker << 8), op.payload,
                            op.type == FMT_MT_INSERT ? op.pos2 : 0, op0.ref_seq);
    if (g < 0) return;
    op.ref_seq = kLocalView;
    op.client = 0;
    op.seq = static_cast<int32_t>(FMT_MT_LOCAL_SEQ_BASE | ls);
    if (op.type == FMT_MT_INSERT) {
      const int k = insertText(op, text0, 0, true, true);
      if (k < 0 || status != FMT_OK) return;
      pendAdd(k, 1);
      recAppend(fId(readField(k, 4)), static_cast<uint32_t>(g));
    } else {
      Lane<uint32_t> delta;
      applyRange(op, delta, true, static_cast<uint32_t>(g));
    }
  }

  // ackOp (mergeTree.ts:1325-1408 + ackSegment :149-215): the oldest pending group takes {seq, 0};
  // each of its segments enters the LRU set in the group's order. (Zamboni follows in replay.)
  FMT_DEV void ackOp(const fmt_mt_op& op) {
    if (gHead == gTail || static_cast<int>(gWord(gHead, 1) & 0xFFu) != op.type) {
      fail(FMT_E_DATA);
      return;
    }
    const uint32_t g = static_cast<uint32_t>(gHead++);
    for (int i = recFind(g, 0); i >= 0 && status == FMT_OK; i = recFind(g, i + 1)) {
      const uint32_t leaf = rWord(i, 0);
      const int j = findLeafById(leaf);
      if (j < 0) {
        fail(FMT_E_DATA);
        return;
      }
      rSet(i, 0, 0u);
      waveSync();
      if (op.type == FMT_MT_INSERT) {
        if (!isLocalSeq(readField(j, 1))) {  // "On insert, seq number already assigned!" (0x045)
          fail(FMT_E_DATA);
          return;
        }
        writeField(j, 1, static_cast<uint32_t>(op.seq));
      } else if (op.type == FMT_MT_REMOVE) {
        const uint32_t rm = readField(j, 2);
        if (isLocalSeq(rm)) writeField(j, 2, static_cast<uint32_t>(op.seq));  // (an earlier acked remove stays first)
        else if (rm == static_cast<uint32_t>(kNotRemoved)) {
          fail(FMT_E_DATA);
          return;
        }
      } else {
        locPmAck(leaf, op.payload, op.seq, op.min_seq);
      }
      pendAdd(j, -1);
      lruForLeaf(j, static_cast<int>(fBlk(readField(j, 0))), op.seq);
    }
  }

  // rollback (mergeTree.ts:2388-2514) of the newest pending group.
  FMT_DEV void rollbackOp(const fmt_mt_op& op) {
    if (gHead == gTail || static_cast<int>(gWord(gTail - 1, 1) & 0xFFu) != op.type) {  // "Rollback op doesn't match last edit"
      fail(FMT_E_DATA);
      return;
    }
    const uint32_t g = static_cast<uint32_t>(--gTail);
    const uint32_t payload = gWord(static_cast<int>(g), 2);
    for (int i = recFind(g, 0); i >= 0 && status == FMT_OK; i = recFind(g, i + 1)) {
      const uint32_t leaf = rWord(i, 0);
      const int j = findLeafById(leaf);
      if (j < 0) {
        fail(FMT_E_DATA);
        return;
      }
      rSet(i, 0, 0u);
      waveSync();
      pendAdd(j, -1);
      if (op.type == FMT_MT_REMOVE) {
        // a peer's concurrent remove keeps the segment removed; otherwise removeRemovalInfo
        if (isLocalSeq(readField(j, 2))) {
          writeField(j, 2, static_cast<uint32_t>(kNotRemoved));
          writeField(j, 3, 0u);
          if constexpr (C::kWords > 5) writeField(j, 5, 0u);
        }
      } else if (op.type == FMT_MT_INSERT) {
        // insert = {TreeMaintenanceSequenceNumber, NonCollabClient}, then markRangeRemoved over exactly
        // the segment's span in the local view with that stamp (rollback's position,
        // findRollbackPosition :2519-2536), then zamboni
        if (readField(j, 2) != static_cast<uint32_t>(kNotRemoved)) {
          fail(FMT_E_DATA);
          return;
        }
        writeField(j, 1, static_cast<uint32_t>(-2));
        writeField(j, 2, static_cast<uint32_t>(-2));
        const uint32_t w4 = readField(j, 4);
        writeField(j, 4, mkW4(fId(w4), FMT_NON_COLLAB_CLIENT) | (w4 & kW4Marker));
        zamboni();
      } else {
        // removed: rollbackProperties directly; else annotateRange(rollback) over its span, then zamboni
        const bool removed = readField(j, 2) != static_cast<uint32_t>(kNotRemoved);
        locPmRollback(j, payload);
        if (!removed && status == FMT_OK) zamboni();
      }
    }
  }

  // normalizeSegmentsOnRebase (mergeTree.ts:2734-2766) + normalizeAdjacentSegments (:2613-2712): runs of
  // adjacent segments that are removed or locally inserted, holding both a local insert and a
  // segment removed by an acked op, are reordered — acked-removed segments after the last segment the
  // local client affected, locally removed ones past the local inserts made after their removal —
  // and the new order takes the run's slots (leaf blocks stay; the text moves with its segments).
  // Serial over the document's leaves (reconnects are rare), state in the document's scratch slab.
  FMT_DEV void normalizeOnRebase() {
    uint32_t* S = in.loc->scratch + in.loc->scratchOffs[in.doc];
    const uint64_t cap = in.loc->scratchOffs[in.doc + 1] - in.loc->scratchOffs[in.doc];
    if (cap < 5ull * static_cast<uint64_t>(n) + 16ull) {
      fail(FMT_E_CAPACITY);
      return;
    }
    // scratch: A[j] = W1, B[j] = W2 of every leaf, a run's list links (nxt, prv) and new order (perm),
    // then permuteRun's copies
    // A[j] = W1, B[j] = W2 of every leaf
    const int nr = rows();
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        const int j = r * 64 + l;
        if (j < n) {
          storeGlobal(S + j, LANE(W[1])[r]);
          storeGlobal(S + n + j, LANE(W[2])[r]);
        }
      }
    }
    waveSync();
    uint32_t* nxt = S + 2 * n;  // list links of one run (members 0..m-1)
    uint32_t* prv = S + 3 * n;
    const uint32_t kNil = 0xFFFFFFFFu;
    auto ins = [&](int j) { return uni(loadCoherent(S + j)); };
    auto rm = [&](int j) { return uni(loadCoherent(S + n + j)); };
    auto inRun = [&](int j) { return rm(j) != static_cast<uint32_t>(kNotRemoved) || isLocalSeq(ins(j)); };
    auto ackedRm = [&](int j) { return rm(j) != static_cast<uint32_t>(kNotRemoved) && !isLocalSeq(rm(j)); };
    auto put = [&](uint32_t* p, uint32_t v) {
      FOR_LANES(l) {
        if (l == 0) storeGlobal(p, v);
      }
      waveSync();
    };
    auto get = [&](const uint32_t* p) { return uni(loadCoherent(p)); };
    for (int a = 0; a < n && status == FMT_OK;) {
      if (!inRun(a)) {
        a++;
        continue;
      }
      int b = a;
      bool hasLocal = false, hasRemote = false;
      while (b < n && inRun(b)) {
        hasLocal = hasLocal || isLocalSeq(ins(b));
        hasRemote = hasRemote || ackedRm(b);
        b++;
      }
      const int m = b - a;
      if (hasLocal && hasRemote && m > 1) {
        for (int k = 0; k < m; k++) {
          put(nxt + k, k + 1 < m ? static_cast<uint32_t>(k + 1) : kNil);
          put(prv + k, k > 0 ? static_cast<uint32_t>(k - 1) : kNil);
        }
        uint32_t head = 0, tail = static_cast<uint32_t>(m - 1);
        auto unlink = [&](uint32_t x) {
          const uint32_t p = get(prv + x), q = get(nxt + x);
          if (p != kNil) put(nxt + p, q);
          else head = q;
          if (q != kNil) put(prv + q, p);
          else tail = p;
        };
        auto insertAfter = [&](uint32_t at, uint32_t x) {
          const uint32_t q = get(nxt + at);
          put(nxt + x, q);
          put(prv + x, at);
          put(nxt + at, x);
          if (q != kNil) put(prv + q, x);
          else tail = x;
        };
        uint32_t lastLocal = kNil;
        for (uint32_t x = tail; x != kNil; x = get(prv + x))
          if (!ackedRm(a + static_cast<int>(x))) {
            lastLocal = x;
            break;
          }
        if (lastLocal != kNil) {
          for (uint32_t slide = lastLocal;;) {
            const uint32_t nearer = get(prv + slide);
            const int sj = a + static_cast<int>(slide);
            if (ackedRm(sj)) {
              unlink(slide);
              insertAfter(lastLocal, slide);
            } else if (rm(sj) != static_cast<uint32_t>(kNotRemoved)) {
              uint32_t cur = slide;
              for (uint32_t scan = get(nxt + cur); scan != kNil; scan = get(nxt + scan)) {
                const int qj = a + static_cast<int>(scan);
                if (ackedRm(qj) || !isLocalSeq(ins(qj)) || ins(qj) <= rm(sj)) break;
                cur = scan;
              }
              if (cur != slide) {
                unlink(slide);
                insertAfter(cur, slide);
              }
            }
            if (nearer == kNil) break;
            slide = nearer;
          }
          // the new order: perm[k] = the member that takes slot a + k
          uint32_t* perm = S + 4 * n;
          bool identity = true;
          int k = 0;
          for (uint32_t x = head; x != kNil; x = get(nxt + x), k++) {
            identity = identity && x == static_cast<uint32_t>(k);
            put(perm + k, x);
          }
          if (!identity) permuteRun(a, m, perm, S + 5 * n, cap - 5ull * static_cast<uint64_t>(n));
        }
      }
      a = b;
    }
  }

  // The run of leaves [a, a + m) takes the order perm (perm[k]: the member now in slot a + k): leaf
  // words and text move with their segment, each slot keeps its leaf block (assignChild(parent, seg,
  // index), mergeTree.ts:2680-2685).
  FMT_DEV void permuteRun(int a, int m, const uint32_t* perm, uint32_t* area, uint64_t areaCap) {
    const int b = a + m;
    const uint32_t ca = charOffsetOf(a), cb = charOffsetOf(b);
    const uint64_t need = static_cast<uint64_t>(kWords) * m + static_cast<uint64_t>(m) + (cb - ca + 1) / 2 + 1;
    if (need > areaCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    uint32_t* R = area;                                  // kWords words per member
    uint32_t* co = area + static_cast<size_t>(kWords) * m;  // members' char offsets in the run (original order)
    uint16_t* T = reinterpret_cast<uint16_t*>(co + m);   // the run's text
    const int r0 = a >> 6, r1 = ((b - 1) >> 6) + 1;
    FOR_ROWS(r, r0, r1) {
      FOR_LANES(l) {
        const int j = r * 64 + l;
        if (j >= a && j < b)
          for (int f = 0; f < kWords; f++) storeGlobal(R + static_cast<size_t>(j - a) * kWords + f, LANE(W[f])[r]);
      }
    }
    FOR_LANES(l) {
      for (uint32_t t = l; t < cb - ca; t += 64) storeGlobal(T + t, static_cast<uint16_t>(chRead(static_cast<int>(ca + t))));
    }
    waveSync();
    uint32_t off = 0;
    for (int k = 0; k < m; k++) {  // (serial: runs are short, reconnects rare)
      const uint32_t len = fLen(uni(loadCoherent(R + static_cast<size_t>(k) * kWords)));
      FOR_LANES(l) {
        if (l == 0) storeGlobal(co + k, off);
      }
      off += len;
    }
    waveSync();
    FOR_ROWS(r, r0, r1) {
      FOR_LANES(l) {
        const int j = r * 64 + l;
        if (j >= a && j < b) {
          const uint32_t src = loadCoherent(perm + (j - a));
          const uint32_t blk = fBlk(LANE(W[0])[r]);
          for (int f = 0; f < kWords; f++) {
            uint32_t v = loadCoherent(R + static_cast<size_t>(src) * kWords + f);
            if (f == 0) v = mkW0(fLen(v), blk, fProps(v));
            LANE(W[f])[r] = v;
          }
        }
      }
    }
    uint32_t dst = ca;
    for (int k = 0; k < m; k++) {
      const uint32_t src = uni(loadCoherent(perm + k));
      const uint32_t so = uni(loadCoherent(co + src));
      const uint32_t len = fLen(uni(loadCoherent(R + static_cast<size_t>(src) * kWords)));
      FOR_LANES(l) {
        for (uint32_t t = l; t < len; t += 64) chWrite(static_cast<int>(dst + t), loadCoherent(T + so + t));
      }
      dst += len;
    }
    waveSync();
  }

  // regeneratePendingOp for every pending op in order (client.ts:1452-1542, squash false): segments
  // normalized once per (currentSeq, localSeq) (:1480-1507); each pending group, its segments in
  // document order, becomes one op per segment at its position in LocalReconnectingPerspective(
  // currentSeq, 0, localSeq) (resetPendingDeltaToOps :1160-1289) — an annotate unless the segment was
  // removed by an acked op, an insert of its current text with the original op's props, a remove
  // while its first remove is still the local one — and a new pending group. The ops go to the
  // document's regen slab.
  FMT_DEV void regenerate() {
    if (gHead == gTail) return;
    if (!normSet || curSeq != normRef || locSeq != normLocal) {
      normalizeOnRebase();
      if (status != FMT_OK) return;
      normSet = true;
      normRef = curSeq;
      normLocal = locSeq;
    }
    if (gHead > 0) groupCompact();
    recCompact();
    recFrozen = true;
    const int g1 = gTail;
    fmt_mt_op* outOps = in.loc->regen + in.loc->regenOffs[in.doc];
    const uint32_t opCap = static_cast<uint32_t>(in.loc->regenOffs[in.doc + 1] - in.loc->regenOffs[in.doc]);
    uint16_t* outText = in.loc->regenText + in.loc->regenTextOffs[in.doc];
    const uint64_t textCap = in.loc->regenTextOffs[in.doc + 1] - in.loc->regenTextOffs[in.doc];
    for (int g = gHead; g < g1 && status == FMT_OK; g++) {
      const uint32_t ls = gWord(g, 0), tf = gWord(g, 1), payload = gWord(g, 2);
      const int32_t pos2 = static_cast<int32_t>(gWord(g, 3)), inflightRef = static_cast<int32_t>(gWord(g, 4));
      const int type = static_cast<int>(tf & 0xFFu);
      // the group's segments as a row bitmask (document order), its records released
      const int nr = rows();
      Lane<uint32_t> segs;
      FOR_LANES(l) { LANE(segs) = 0u; }
      for (int i = recFind(static_cast<uint32_t>(g), 0); i >= 0 && status == FMT_OK; i = recFind(static_cast<uint32_t>(g), i + 1)) {
        const int j = findLeafById(rWord(i, 0));
        if (j < 0) {
          fail(FMT_E_DATA);
          break;
        }
        rSet(i, 0, 0u);
        FOR_LANES(l) {
          if (l == (j & 63)) LANE(segs) |= 1u << (j >> 6);
        }
      }
      waveSync();
      if (status != FMT_OK) break;
      Lane<VR> vis, st;
      visLengths(static_cast<int>(FMT_MT_LOCAL_SEQ_BASE | ls), -5, vis, nr);  // findReconnectionPosition
      scanRows(vis, st, nr);
      for (Lane<uint32_t> todo = segs; status == FMT_OK;) {
        const int j = firstSet(todo, nr);
        if (j < 0) break;
        FOR_LANES(l) {
          if (l == (j & 63)) LANE(todo) &= ~(1u << (j >> 6));
        }
        const uint32_t w1 = readField(j, 1), w2 = readField(j, 2), w4 = readField(j, 4);
        const uint32_t len = fLen(readField(j, 0));
        const int pos = static_cast<int>(readlane(selectRow(st, j >> 6), j & 63));
        const bool removed = w2 != static_cast<uint32_t>(kNotRemoved);
        bool emit = false;
        fmt_mt_op o;
        o.seq = static_cast<int32_t>(ls);
        o.ref_seq = curSeq;
        o.min_seq = 0;
        o.pos1 = pos;
        o.pos2 = pos + static_cast<int32_t>(len);
        o.payload = payload;
        o.len = 0;
        o.client = 0;
        o.type = static_cast<uint8_t>(type);
        o.flags = 0;
        if (type == FMT_MT_ANNOTATE) {
          emit = !(removed && !isLocalSeq(w2));  // not isRemovedAndAcked
        } else if (type == FMT_MT_INSERT) {
          if (!isLocalSeq(w1)) {  // "Segment already has assigned sequence number" (0x037)
            fail(FMT_E_DATA);
            break;
          }
          if (removed && !isLocalSeq(w2)) {  // obliterated on arrival: obliterate reconnect is not in this build
            fail(FMT_E_UNSUPPORTED);
            break;
          }
          if (regenTextN + len > textCap) {
            fail(FMT_E_CAPACITY);
            break;
          }
          const uint32_t c0 = charOffsetOf(j);
          FOR_LANES(l) {
            for (uint32_t t = l; t < len; t += 64) storeGlobal(outText + regenTextN + t, static_cast<uint16_t>(chRead(static_cast<int>(c0 + t))));
          }
          o.pos2 = pos2;
          o.payload = regenTextN;
          o.len = static_cast<uint16_t>(len & 0xFFFFu);
          o.flags = (len & FMT_MT_F_LEN_HI_MASK) | (fMarker(w4) ? FMT_MT_F_MARKER : 0u);
          regenTextN += len;
          emit = true;
        } else {
          emit = removed && isLocalSeq(w2);  // nobody else removed it meanwhile
        }
        if (emit) {
          if (regenN >= opCap) {
            fail(FMT_E_CAPACITY);
            break;
          }
          FOR_LANES(l) {
            if (l == 0) outOps[regenN] = o;
          }
          regenN++;
          const int ng = groupPush(ls, tf, payload, pos2, inflightRef);
          if (ng < 0) break;
          recAppend(fId(w4), static_cast<uint32_t>(ng));
        } else {
          pendAdd(j, -1);
        }
      }
    }
    waveSync();
    gHead = g1;  // (the old groups are replaced by the new ones, [g1, gTail))
    recFrozen = false;
  }

  // ------------------------------------------------------------------ zamboni (zamboni.ts)
  // scourNode over leaf block b: drops tombstones removed at/below minSeq and appends acked,
  // same-props, appendable leaves onto the previous kept leaf. Returns the new child count.
  FMT_DEV int scourLeafBlock(int b) {
    const int cnt = uni(static_cast<int>(s->blk[b].count));
    if (cnt == 0) return 0;
    const int first = firstLeafOf(static_cast<uint32_t>(b));
    // One pass packs what the decisions need for every leaf of the block (at most 2 rows):
    // len | props << kLenBits | removed << 24 | removed at/below minSeq << 25 | insert at/below minSeq << 26
    // | last UTF-16 unit is '\n' << 27 (TextSegment.canAppend, textSegment.ts:76-93: one LDS read for
    // all leaves, at their char offsets from a scan of the block's lengths)
    const int r0 = first >> 6, r1 = (first + cnt - 1) >> 6;
    Lane<uint32_t> pk0, pk1;
    Lane<uint32_t> pp0, pp1;  // (large tier: prop-set ids of up to 1024 sets beside the packed words)
    FOR_LANES(l) {
      LANE(pk0) = 0u;
      LANE(pk1) = 0u;
      LANE(pp0) = 0u;
      LANE(pp1) = 0u;
    }
    uint32_t cs = charOffsetOf(first);  // running char offset of leaf first + k
    uint32_t rowBase = cs;
    FOR_ROWS(r, r0, r1 + 1) {
      Lane<uint32_t> blen;
      FOR_LANES(l) {
        const int idx = r * 64 + l;
        LANE(blen) = idx >= first && idx < first + cnt ? fLen(LANE(W[0])[r]) : 0u;
      }
      uint32_t tot;
      const Lane<uint32_t> ex = waveExclusiveSum(blen, &tot);
      FOR_LANES(l) {
        const uint32_t w0 = LANE(W[0])[r];
        const int32_t ins = static_cast<int32_t>(LANE(W[1])[r]), rm = static_cast<int32_t>(LANE(W[2])[r]);
        const uint32_t bl = LANE(blen);
        const bool nl = bl > 0 && chRead(static_cast<int>(rowBase + LANE(ex) + bl - 1)) == 10u;
        const uint32_t pr = propsL(l, r);
        bool held = false;  // (Loc) a leaf with pending local ops (zamboni.ts:148)
        if constexpr (Loc) held = LANE(W[kPendW])[r] != 0u;
        const uint32_t p = fLen(w0) | ((kPW ? 0u : pr) << C::kLenBits) | (rm != kNotRemoved ? 1u << 24 : 0u) |
                           (rm <= minSeq ? 1u << 25 : 0u) | (ins <= minSeq ? 1u << 26 : 0u) | (nl ? 1u << 27 : 0u) |
                           (fMarker(LANE(W[4])[r]) ? 1u << 28 : 0u) | (held ? 1u << 29 : 0u);
        if (r == r0) LANE(pk0) = p;
        else LANE(pk1) = p;
        if constexpr (kPW) {
          if (r == r0) LANE(pp0) = pr;
          else LANE(pp1) = pr;
        }
      }
      rowBase += tot;
    }
    stamp(kPfZChars);
    // serial decisions over <= 7 leaves: keep, merge into the previous kept leaf, or drop
    uint32_t mergeMask = 0, dropMask = 0;
    int prev = -1;
    uint32_t prevLen = 0, prevProps = 0, prevBlk = 0;
    bool prevNl = false;
    int kept = 0;
    for (int k = 0; k < cnt; k++) {
      const int j = first + k;
      const uint32_t p = (j >> 6) == r0 ? readlane(pk0, j & 63) : readlane(pk1, j & 63);
      const uint32_t len = p & kLenMask;
      uint32_t props = (p >> C::kLenBits) & kPropsUndef;
      if constexpr (kPW) props = (j >> 6) == r0 ? readlane(pp0, j & 63) : readlane(pp1, j & 63);
      s->tmp[k] = cs;  // char offset and length, for the deletions below
      s->tmp[kMaxNodes + k] = len;
      if ((p >> 29) & 1u) {  // held: kept as it is, and nothing appends onto it
        prev = -1;
        kept++;
      } else if (((p >> 24) & 1u) == 0) {
        if ((p >> 26) & 1u) {
          const bool lastNl = ((p >> 27) & 1u) != 0;
          const bool marker = ((p >> 28) & 1u) != 0;  // Marker: never appends, nothing appends onto it
          const bool canAppend = prev >= 0 && !prevNl && !marker &&
                                 (prevLen <= static_cast<uint32_t>(kGranularity) ||
                                  len <= static_cast<uint32_t>(kGranularity)) &&
                                 propsMatch(prevProps, props) && len > 0;
          if (canAppend) {
            mergeMask |= 1u << k;
            if constexpr (Ob) {  // LocalReferenceCollection.append (localReference.ts:233-251)
              if (obUsed != 0) obRefsMove(fId(readField(j, 4)), fId(readField(prev, 4)), 0, static_cast<int>(prevLen));
            }
            prevLen += len;
            prevNl = lastNl;
            // the head keeps its index until the deletions below, so its length can be set now
            writeField(prev, 0, mkW0(prevLen, prevBlk, prevProps));
          } else {
            prev = len > 0 && !marker ? j : -1;
            prevLen = len;
            prevProps = props;
            prevBlk = static_cast<uint32_t>(b);
            prevNl = lastNl;
            kept++;
          }
        } else {
          prev = -1;
          kept++;
        }
      } else {
        if ((p >> 25) & 1u) {
          dropMask |= 1u << k;
        } else {
          kept++;
        }
        prev = -1;
      }
      cs += len;
    }
    waveSync();
    stamp(kPfZSerial);
    // Dropped leaves take their text with them: one pass moves every later char down by the dropped
    // lengths before it (chars of merged leaves stay, they already follow their head's).
    if (dropMask != 0) {
      uint32_t c0 = 0, dropped = 0;
      for (int k = cnt - 1; k >= 0; k--)
        if ((dropMask >> k) & 1u) c0 = uni(s->tmp[k]);
      for (int k = 0; k < cnt; k++)
        if ((dropMask >> k) & 1u) dropped += uni(s->tmp[kMaxNodes + k]);
      const int newChars = nChars - static_cast<int>(dropped);
      for (int base = static_cast<int>(c0); base < newChars; base += 64) {
        Lane<uint32_t> v;
        FOR_LANES(l) {
          const int c = base + l;
          uint32_t shift = 0, before = 0;
          for (int k = 0; k < cnt; k++) {
            if ((dropMask >> k) & 1u) {
              const uint32_t ks = uni(s->tmp[k]), kl = uni(s->tmp[kMaxNodes + k]);
              if (static_cast<uint32_t>(c) >= ks - before) shift += kl;
              before += kl;
            }
          }
          LANE(v) = c < newChars ? chRead(c + static_cast<int>(shift)) : 0u;
        }
        waveSync();
        FOR_LANES(l) {
          if (base + l < newChars) chWrite(base + l, LANE(v));
        }
        waveSync();
      }
      nChars = newChars;
    }
    if constexpr (Adj || Loc) {  // appended and unlinked leaves take their managers with them
      for (uint32_t m = pmN > 0 ? (mergeMask | dropMask) : 0u; m != 0; m &= m - 1) pmDropLeaf(fId(readField(first + ctz32(m), 4)));
    }
    deleteLeaves(first, cnt, mergeMask | dropMask);
    stamp(kPfZDelete);
    return kept;
  }

  // packParent redistribution (zamboni.ts:83-139) of `total` held children into
  // min(7, total/4) (>= 1) new blocks; leaf level re-tags the contiguous leaves, interior level
  // re-parents the grandchildren listed in s->tmp.
  FMT_DEV void redistribute(int p, int total, bool leafLevel, int firstLeaf) {
    const int pc = uni(static_cast<int>(s->blk[p].count));
    for (int i = 0; i < pc; i++) freeBlk(uni(static_cast<int>(s->blk[p].child[i])));
    if (total > 0) {
      int nb = total / (kMaxNodes / 2);
      if (nb > kMaxNodes - 1) nb = kMaxNodes - 1;
      if (nb < 1) nb = 1;
      const int base = total / nb;
      int rem = total % nb;
      int consumed = 0;
      for (int q = 0; q < nb; q++) {
        int cnt = base;
        if (rem > 0) {
          cnt++;
          rem--;
        }
        const int id = allocBlk(leafLevel ? 1 : 0);
        if (id < 0) return;
        s->blk[id].count = static_cast<uint8_t>(cnt);
        s->blk[id].parent = static_cast<BId>(p);
        if (leafLevel) {
          tagLeaves(firstLeaf + consumed, cnt, static_cast<uint32_t>(id));
        } else {
          for (int k = 0; k < cnt; k++) {
            const int g = uni(static_cast<int>(s->tmp[consumed + k]));
            s->blk[id].child[k] = static_cast<BId>(g);
            s->blk[g].parent = static_cast<BId>(id);
          }
        }
        s->blk[p].child[q] = static_cast<BId>(id);
        waveSync();
        consumed += cnt;
      }
      s->blk[p].count = static_cast<uint8_t>(nb);
    } else {
      s->blk[p].count = 0;
      if (p == root) s->blk[p].leaf = 1;
    }
    waveSync();
    stamp(kPfZPack);
  }

  // zamboni.ts:33-80, with packParent (zamboni.ts:83-139) folded in so that every block scour —
  // the popped block's own and each sibling's during packParent — goes through one call site.
  FMT_DEV void zamboni() {
    for (int i = 0; i < 2; i++) {
      if (heapN == 0) break;
      if constexpr (Adj) {  // segmentToScour?.segment?.propertyManager?.updateMsn(minSeq) (zamboni.ts:44)
        if (pmN > 0) pmUpdateMsn(uni(s->heap[1].leafId), minSeq);
      }
      if (heapSeq(1) > minSeq) break;
      const HeapEnt ent = heapGet();
      const int j = findLeafById(ent.leafId);
      stamp(kPfZFind);
      if (j < 0) continue;  // unlinked or appended: segment.parent is undefined
      const int b = static_cast<int>(fBlk(readField(j, 0)));
      if (uni(static_cast<int>(s->blk[b].needsScour)) == 0) continue;
      const int oldCount = uni(static_cast<int>(s->blk[b].count));
      int target = b, p = -1, ci = 0, total = 0, firstLeaf = -1;
      for (;;) {
        const int kept = scourLeafBlock(target);
        if (status != FMT_OK) return;
        if (p < 0) {  // the popped block itself
          s->blk[b].needsScour = 0;
          waveSync();
          if (kept >= oldCount) break;
          s->blk[b].count = static_cast<uint8_t>(kept);
          waveSync();
          const int parent = uni(static_cast<int>(s->blk[b].parent));
          if (kept >= kMaxNodes / 2 || parent == static_cast<int>(kNoBlk)) break;
          p = parent;  // packParent(parent): scour every child block of p, in order
          ci = 0;
          target = uni(static_cast<int>(s->blk[p].child[0]));
          continue;
        }
        s->blk[target].count = static_cast<uint8_t>(kept);
        waveSync();
        if (kept > 0 && firstLeaf < 0) firstLeaf = firstLeafOf(static_cast<uint32_t>(target));
        total += kept;
        if (++ci < uni(static_cast<int>(s->blk[p].count))) {
          target = uni(static_cast<int>(s->blk[p].child[ci]));
          continue;
        }
        redistribute(p, total, true, firstLeaf);
        if (status != FMT_OK) return;
        // interior levels: scourNode holds block children as they are
        for (;;) {
          const int pp = uni(static_cast<int>(s->blk[p].parent));
          if (uni(static_cast<int>(s->blk[p].count)) >= kMaxNodes / 2 || pp == static_cast<int>(kNoBlk)) break;
          p = pp;
          const int pc = uni(static_cast<int>(s->blk[p].count));
          int held = 0;
          for (int q = 0; q < pc; q++) {
            const int c = uni(static_cast<int>(s->blk[p].child[q]));
            const int cc = uni(static_cast<int>(s->blk[c].count));
            for (int k = 0; k < cc; k++) s->tmp[held++] = uni(static_cast<int>(s->blk[c].child[k]));
          }
          waveSync();
          redistribute(p, held, false, -1);
          if (status != FMT_OK) return;
        }
        break;
      }
    }
  }

  // ------------------------------------------------------------------ driver
  FMT_DEV void init() {
    n = 0;
    nChars = 0;
    heapN = 0;
    nProps = 0;
    curSeq = 0;
    minSeq = 0;
    status = FMT_OK;
    failSeq = 0;
    nextId = 1;
    obSeqN = 0;
    obStartN = 0;
    obUsed = 0;
    FOR_LANES(l) {
      VR z;
#pragma unroll
      for (int r = 0; r < kRows; r++) z[r] = 0u;
      LANE(W[0]) = z;
      LANE(W[1]) = z;
      LANE(W[2]) = z;
      LANE(W[3]) = z;
      if constexpr (C::kWords > 5) {
        LANE(W[5]) = z;
        LANE(W[kPropW]) = z;
      }
      LANE(W[4]) = z;
      if constexpr (Loc) LANE(W[kPendW]) = z;
    }
    FOR_LANES(l) {
      for (int i = l; i < kMaxBlocks; i += 64) s->freeList[i] = static_cast<BId>(kMaxBlocks - 1 - i);
    }
    waveSync();
    nFree = kMaxBlocks;
    root = allocBlk(1);
  }

  // Initial text inserted locally before collaboration (client.replay.spec.ts:30-33):
  // one leaf, insert stamp {seq 0, LocalClientId}.
  FMT_DEV void loadInitial() {
    const int len = static_cast<int>(in.initLen);
    if (len == 0) return;
    if (len > kCapChars || static_cast<uint32_t>(len) > kLenMask) {
      fail(FMT_E_CAPACITY);
      return;
    }
    const uint16_t* src = in.text + in.initOff;
    FOR_LANES(l) {
      for (int t = l; t < len; t += 64) chWrite(t, src[t]);
    }
    waveSync();
    nChars = len;
    const uint32_t w0 = mkW0(static_cast<uint32_t>(len), static_cast<uint32_t>(root), kPropsUndef);
    const uint32_t w4 = mkW4(nextId++, FMT_LOCAL_CLIENT);
    FOR_LANES(l) {
      if (l == 0) {
        LANE(W[0])[0] = w0;
        LANE(W[1])[0] = 0u;
        LANE(W[2])[0] = static_cast<uint32_t>(kNotRemoved);
        LANE(W[3])[0] = 0u;
        LANE(W[4])[0] = w4;
        if constexpr (kPW) LANE(W[kPropW])[0] = kPropsUndef;
      }
    }
    n = 1;
    s->blk[root].count = 1;
    waveSync();
  }

  // ------------------------------------------------------------------ snapshot load (f3)
  // SnapshotLoader (snapshotLoader.ts:59-348) for a legacy summary: the header chunk's segments
  // rebuild the tree bottom-up, MaxNodesInBlock - 1 = 7 children per block (reloadFromSegments,
  // mergeTree.ts:751-800); collaboration starts at (minSeq, seq) (loadHeader :189-219); each body
  // segment is appended through insertSegments at the end (loadBody :221-311), which lands it in the
  // last leaf's block and splits on overflow. Every loaded segment is stamped
  // {UniversalSequenceNumber, NonCollabClient} (specToSegment :180-186). Runs right after init(),
  // so block ids are handed out in order: level by level, leaf blocks first.
  FMT_DEV void appendLoadedChars(uint32_t off, uint32_t len) {
    FOR_LANES(l) {
      for (uint32_t t = l; t < len; t += 64) chWrite(nChars + static_cast<int>(t), in.text[off + t]);
    }
    waveSync();
    nChars += static_cast<int>(len);
  }

  // Properties of the loaded leaves [first, last) whose row bits are set in `pending`: one interned
  // prop set per distinct props op (a spec's props applied onto undefined properties).
  FMT_DEV void loadProps(int first, int last) {
    FOR_ROWS(r, first >> 6, (last + 63) >> 6) {
      Lane<uint32_t> op;
      FOR_LANES(l) {
        const int j = r * 64 + l;
        LANE(op) = j >= first && j < last ? in.snapSegs[j].props : FMT_MT_NO_PROPS;
      }
      for (;;) {
        Lane<bool> p;
        FOR_LANES(l) { LANE(p) = LANE(op) != FMT_MT_NO_PROPS; }
        const uint64_t m = ballot(p);
        if (m == 0) break;
        const uint32_t id = readlane(op, ctz64(m));
        if (id >= in.nPropsOps) {
          fail(FMT_E_DATA);
          return;
        }
        const uint32_t pid = applyProps(kPropsUndef, id);
        if (status != FMT_OK) return;
        FOR_LANES(l) {
          if (LANE(op) == id) {
            setPropsL(l, r, pid);
            LANE(op) = FMT_MT_NO_PROPS;
          }
        }
      }
    }
  }

  // SnapshotV1 merge info (specToSegment, snapshotLoader.ts:105-175) of header segments: the insert
  // stamp, and the remove stamps folded into the leaf's first remove seq and remove-client set.
  FMT_DEV bool loadMergeInfo(int H, int N) {
    const int nr = (N + 63) >> 6;
    Lane<bool> bad, wide;  // body-chunk merge info (host-rejected); more writers than this tier holds
    FOR_LANES(l) {
      LANE(bad) = false;
      LANE(wide) = false;
    }
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        const int j = r * 64 + l;
        if (j < N) {
          const fmt_mt_snapshot_info inf = in.snapInfo[j];
          if (j >= H && (inf.ins_seq != 0 || inf.rm_count != 0)) LANE(bad) = true;
          int32_t rm = kNotRemoved;
          uint64_t mask = 0;
          for (uint32_t t = 0; t < inf.rm_count; t++) {
            const fmt_mt_stamp st = in.snapStamps[inf.rm_first + t];
            rm = st.seq < rm ? st.seq : rm;
            if (st.client < 0 || st.client > kMaxClient) LANE(wide) = true;
            else mask |= 1ull << st.client;
          }
          if (inf.ins_client > kMaxClient) LANE(wide) = true;
          LANE(W[1])[r] = static_cast<uint32_t>(inf.ins_seq);
          LANE(W[2])[r] = static_cast<uint32_t>(rm);
          LANE(W[3])[r] = static_cast<uint32_t>(mask);
          if constexpr (C::kWords > 5) LANE(W[5])[r] = static_cast<uint32_t>(mask >> 32);
          const uint32_t w4 = LANE(W[4])[r];
          LANE(W[4])[r] = mkW4(fId(w4), inf.ins_client) | (w4 & kW4Marker);
        }
      }
    }
    if (ballot(bad) != 0) {
      fail(FMT_E_UNSUPPORTED);
      return false;
    }
    if (ballot(wide) != 0) {
      fail(FMT_E_CAPACITY);
      return false;
    }
    return true;
  }

  FMT_DEV void loadSnapshot() {
    const int H = static_cast<int>(in.nHeader), N = static_cast<int>(in.nHeader + in.nBody);
    if (N > kCapLeaves) {
      fail(FMT_E_CAPACITY);
      return;
    }
    uint32_t chars = 0;
    for (int k = 0; k < N; k++) {
      const uint32_t len = uni(in.snapSegs[k].len) & ~FMT_MT_SEG_MARKER;
      if (len == 0) {
        fail(FMT_E_DATA);
        return;
      }
      chars += len;
    }
    if (chars > static_cast<uint32_t>(kCapChars)) {
      fail(FMT_E_CAPACITY);
      return;
    }
    // Every loaded leaf in one row pass (lengths staged through the still-unused char area); slots
    // past N stay all-zero. Header leaf j belongs to leaf block j / 7, body leaves get theirs below.
    // (the large tier reads the lengths straight from the segment records)
    uint32_t* stage = reinterpret_cast<FMT_LDS uint32_t*>(s->chars);
    if constexpr (!C::kHbmChars) {
      FOR_LANES(l) {
        for (int j = l; j < N; j += 64) stage[j] = in.snapSegs[j].len;  // (with FMT_MT_SEG_MARKER)
      }
      waveSync();
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) {
      FOR_LANES(l) {
        const int j = r * 64 + l;
        const bool live = j < N;
        const uint32_t lenF = live ? (C::kHbmChars ? in.snapSegs[j].len : stage[j]) : 0u;
        const uint32_t len = lenF & ~FMT_MT_SEG_MARKER;
        LANE(W[0])[r] = live ? mkW0(len, static_cast<uint32_t>(j < H ? j / 7 : 0), kPropsUndef) : 0u;
        LANE(W[2])[r] = live ? static_cast<uint32_t>(kNotRemoved) : 0u;
        LANE(W[4])[r] = live ? mkW4(static_cast<uint32_t>(j + 1), FMT_NON_COLLAB_CLIENT) | ((lenF & FMT_MT_SEG_MARKER) != 0 ? kW4Marker : 0u) : 0u;
        if constexpr (kPW) LANE(W[kPropW])[r] = live ? kPropsUndef : 0u;
      }
    }
    waveSync();
    if (in.snapInfo != nullptr && !loadMergeInfo(H, N)) return;
    nextId = static_cast<uint32_t>(N + 1);
    if (H > 0) {  // reloadFromSegments: leaf blocks [0, cnt), then each level above
      int lo = 0, cnt = (H + 6) / 7;
      for (int b = 0; b < cnt; b++) {
        s->blk[b].count = static_cast<uint8_t>(H - 7 * b < 7 ? H - 7 * b : 7);
        s->blk[b].parent = static_cast<BId>(kNoBlk);
        s->blk[b].leaf = 1;
        s->blk[b].needsScour = -1;
      }
      waveSync();
      while (cnt > 1) {
        const int nb = (cnt + 6) / 7, nlo = lo + cnt;
        for (int q = 0; q < nb; q++) {
          const int id = nlo + q;
          const int c = cnt - 7 * q < 7 ? cnt - 7 * q : 7;
          s->blk[id].count = static_cast<uint8_t>(c);
          s->blk[id].parent = static_cast<BId>(kNoBlk);
          s->blk[id].leaf = 0;
          s->blk[id].needsScour = -1;
          for (int k = 0; k < c; k++) {
            s->blk[id].child[k] = static_cast<BId>(lo + 7 * q + k);
            s->blk[lo + 7 * q + k].parent = static_cast<BId>(id);
          }
        }
        waveSync();
        lo = nlo;
        cnt = nb;
      }
      root = lo;
      nFree = kMaxBlocks - (lo + 1);  // the free list hands out ids in increasing order
    }
    n = H;
    minSeq = in.snapMinSeq;  // loadHeader: startOrUpdateCollaboration(minSeq, seq)
    curSeq = in.snapSeq;
    // loadBody: each body segment goes through the inserting walk at the end, which puts it in the
    // last leaf's block (the empty root when there is no header) and splits on overflow
    for (int k = H; k < N; k++) {
      const int blk = n > 0 ? static_cast<int>(fBlk(readField(n - 1, 0))) : root;
      if (uni(static_cast<int>(s->blk[blk].count)) == 0) {
        s->blk[blk].leaf = 1;
        waveSync();
      }
      tagLeaves(k, 1, static_cast<uint32_t>(blk));
      n++;
      childAdded(blk);
      if (status != FMT_OK) return;
    }
    loadProps(0, N);
    for (int k = 0; k < N && status == FMT_OK; k++)
      appendLoadedChars(uni(in.snapSegs[k].text), uni(in.snapSegs[k].len) & ~FMT_MT_SEG_MARKER);
  }

  // Op records are prefetched two ahead and an insert's first 64 text units one op ahead, so the
  // global-load latency of the dependent op stream overlaps the previous op's work. A record is
  // either eight lanes of one vector load (lanes 0..7 hold its dwords, read back with v_readlane) or,
  // with FMT_SCALAR_OPS, eight SGPRs of one scalar load (the address is wave-uniform).
#if FMT_SCALAR_OPS && FMT_GPU
  struct OpRec {
    uint32_t w[8];
  };
  FMT_DEV OpRec fetchOp(uint64_t i) const {
    OpRec r;
    typedef const __attribute__((address_space(4))) uint32_t* ConstPtr;
    if (i < in.end) {
      const uint64_t a = reinterpret_cast<uintptr_t>(in.ops + i);
      const uint64_t au = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a))) |
                          (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a >> 32)))) << 32);
      const ConstPtr p = (ConstPtr)(au);  // NOLINT: address-space cast (a wave-uniform address in SGPRs)
#pragma unroll
      for (int k = 0; k < 8; k++) r.w[k] = p[k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) r.w[k] = 0u;
    }
    return r;
  }
  FMT_DEV static uint32_t recWord(const OpRec& r, int k) { return r.w[k]; }
#else
  using OpRec = Lane<uint32_t>;
  FMT_DEV OpRec fetchOp(uint64_t i) const {
    Lane<uint32_t> x;
    if (i < in.end) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(in.ops + i);
      FOR_LANES(l) { LANE(x) = l < 8 ? p[l] : 0u; }
    } else {
      FOR_LANES(l) { LANE(x) = 0u; }
    }
    return x;
  }
  FMT_DEV static uint32_t recWord(const OpRec& r, int k) { return readlane(r, k); }
#endif

  FMT_DEV static uint32_t opLen(const fmt_mt_op& op) { return op.len | (op.flags & FMT_MT_F_LEN_HI_MASK); }
  FMT_DEV static fmt_mt_op decodeOp(const OpRec& rec) {
    fmt_mt_op op;
    op.seq = static_cast<int32_t>(recWord(rec, 0));
    op.ref_seq = static_cast<int32_t>(recWord(rec, 1));
    op.min_seq = static_cast<int32_t>(recWord(rec, 2));
    op.pos1 = static_cast<int32_t>(recWord(rec, 3));
    op.pos2 = static_cast<int32_t>(recWord(rec, 4));
    op.payload = recWord(rec, 5);
    const uint32_t lct = recWord(rec, 6);
    op.len = static_cast<uint16_t>(lct & 0xFFFF);
    op.client = static_cast<uint8_t>((lct >> 16) & 0xFF);
    op.type = static_cast<uint8_t>(lct >> 24);
    op.flags = recWord(rec, 7);
    return op;
  }

  FMT_DEV Lane<uint32_t> fetchText(const OpRec& rec) const {
    const uint32_t lct = recWord(rec, 6);
    const int len = (lct >> 24) == FMT_MT_INSERT ? static_cast<int>((lct & 0xFFFF) | (recWord(rec, 7) & FMT_MT_F_LEN_HI_MASK)) : 0;
    const uint32_t payload = recWord(rec, 5);
    Lane<uint32_t> x;
    FOR_LANES(l) { LANE(x) = l < len ? static_cast<uint32_t>(in.text[payload + l]) : 0u; }
    return x;
  }

  FMT_DEV void replay(uint64_t first) {
    stamp(kPfOutput);
    OpRec rec0 = fetchOp(first);
    OpRec rec1 = fetchOp(first + 1);
    Lane<uint32_t> txt0 = fetchText(rec0);
    const bool canSave = kSavesCkpt ? ckpt != nullptr : bigCkpt != nullptr && (!Ob || ckpt != nullptr);
    for (uint64_t i = first; i < in.end; i++) {
      fmt_mt_op op = decodeOp(rec0);
      if constexpr (kSavesHuge) {
        // large tier: the same limits — rows, text, blocks, prop sets, writers past 63 — stop the
        // document for the huge tier (a document still empty restarts there instead)
        const bool loaderNonCollab = (op.flags & FMT_MT_F_LOADSEG) != 0 && op.client == FMT_MT_CLIENT_NONCOLLAB;
        if (hugeCkpt != nullptr && n > 0 &&
            (n + 2 > kCapLeaves || (op.type == FMT_MT_INSERT && nChars + static_cast<int>(opLen(op)) > kCapChars) ||
             (op.client > kMaxClient && !loaderNonCollab) || nFree < 16 ||
             ((op.type == FMT_MT_ANNOTATE || op.type == FMT_MT_INSERT) && nProps > kPropCap - 4))) {
          ckptNext = i;
          status = kCkptEscalate;
          return;
        }
      }
      if constexpr (kSavesCkpt || kSavesBig) {
        // the op could outgrow the rows (at most two new leaves), the text, or (small tier) the
        // writer set of this tier
        // (the small tier also stops near its block and prop-set limits, which the large tier's
        // 1023 / 1024 lift: an op's splits allocate a few blocks, an annotate a few sets)
        const bool loaderNonCollab = (op.flags & FMT_MT_F_LOADSEG) != 0 && op.client == FMT_MT_CLIENT_NONCOLLAB;
        if (canSave &&
            (n + 2 > kCapLeaves || (op.type == FMT_MT_INSERT && nChars + static_cast<int>(opLen(op)) > kCapChars) ||
             (kSavesBig && ((op.client > kMaxClient && !loaderNonCollab) ||
                            // (margins: plain batches only — obliterate documents near them mostly
                            // finish in this tier, measured on the obliterate farms)
                            (!Ob && (nFree < 16 || ((op.type == FMT_MT_ANNOTATE || op.type == FMT_MT_INSERT) &&
                                                    nProps > kPropCap - 4))))))) {
          // plain batches: saved by run(), outside the op loop (T1: 455 -> 450 ms, 159 -> 152 VGPRs
          // in the compact tier); the obliterate variants' code schedules better with it here
          // (compact tier 427 vs 464 ms on the obliterate farms)
          if constexpr (Ob) {
            if constexpr (kSavesCkpt) saveCkpt(i);
            else saveBig(i);
          } else {
            ckptNext = i;
          }
          status = kCkptEscalate;
          return;
        }
      }
      const Lane<uint32_t> text = txt0;
      rec0 = rec1;
      txt0 = fetchText(rec0);
      rec1 = fetchOp(i + 2);
      stamp(kPfOpLoad);
      opIdx = static_cast<uint32_t>(i - in.begin);
      const bool loader = (op.flags & FMT_MT_F_LOADSEG) != 0;
      if constexpr (Loc) {
        // the local client's own events: a submission, a rollback or a reconnect changes no collab
        // window and runs no window zamboni (an ACK is a sequenced message: below)
        if (op.flags & (FMT_MT_F_LOCAL | FMT_MT_F_ROLLBACK | FMT_MT_F_REGEN)) {
          if (op.flags & FMT_MT_F_LOCAL) applyLocal(op, text);
          else if (op.flags & FMT_MT_F_ROLLBACK) rollbackOp(op);
          else regenerate();
          if (status != FMT_OK) {
            failSeq = op.seq;
            break;
          }
          continue;
        }
      }
      // The op's checks first: a failing one leaves the loop at once, so its path (leaf rows unchanged)
      // does not join the ones that change the rows, where the compiler would keep both copies of them
      // live (the obliterate small tier spilled 16 VGPRs per op at that join).
      int bad = FMT_OK;
      if (loader) {
        if (!(op.client == FMT_MT_CLIENT_NONCOLLAB || op.client <= kMaxClient))
          bad = op.client <= kTopClient ? FMT_E_CAPACITY : FMT_E_UNSUPPORTED;
      } else if (op.client > kMaxClient) {  // the small tier's 31 writers: the large tier takes 63, the huge 253
        bad = op.client <= kTopClient ? FMT_E_CAPACITY : FMT_E_UNSUPPORTED;
      } else if (op.type > FMT_MT_ANNOTATE && !(Ob && (op.type == FMT_MT_OBLITERATE || op.type == FMT_MT_OBLITERATE_SIDED))) {
        bad = FMT_E_UNSUPPORTED;
      } else if (op.type == FMT_MT_ANNOTATE && op.payload >= in.nPropsOps) {
        bad = FMT_E_DATA;
      }
      // (Rm variants keep the checks' failures on the joined path: the early exit costs them spills)
      if constexpr (!Rm) {
        if (bad != FMT_OK) {
          fail(bad);
          failSeq = op.seq;
          break;
        }
      }
      if (bad != FMT_OK) fail(bad);
      else if (loader) loadBodySegment(op, text);
      else if (Loc && (op.flags & FMT_MT_F_ACK)) ackOp(op);
      else if ((op.flags & (FMT_MT_F_REL1 | FMT_MT_F_REL2)) == 0 || resolveRelative(op)) applyOp(op, text);
      if constexpr (Rm) {
        if (rmPendN > 0 || rmHitsSet)
          rmFlush(op.client, op.seq, op.type == FMT_MT_REMOVE ? FMT_MT_RM_SET : FMT_MT_RM_SLICE);
      }
      // (a loader segment updates no collab window; a batch of them is no GROUP message)
      const bool lastMember = !loader && (i + 1 == in.end || (recWord(rec0, 7) & (FMT_MT_F_GROUP_CONT | FMT_MT_F_LOADSEG)) !=
                                                                 FMT_MT_F_GROUP_CONT);
      // zamboni once inside the op (mergeTree.ts:1510-1516, 2074-2080, 2376-2382), then, after the
      // message's last member, updateSeqNumbers (client.ts:1381-1391) → setMinSeq
      // (mergeTree.ts:1147-1166), which runs zamboni again only if minSeq advanced.
      for (int z = 0; z < 2 && status == FMT_OK; z++) {
        if (z == 1) {
          if (!lastMember) break;
          if (curSeq > op.seq || op.min_seq > op.seq || minSeq > op.min_seq) {
            fail(FMT_E_DATA);
            break;
          }
          curSeq = op.seq;
          int eff = op.min_seq;
          if constexpr (Loc) {  // bounded by the oldest in-flight op's refSeq (client.ts:1374-1378, sequence.ts:499)
            if (gHead < gTail && static_cast<int32_t>(gWord(gHead, 4)) < eff) eff = static_cast<int32_t>(gWord(gHead, 4));
          }
          if (eff <= minSeq) break;
          minSeq = eff;
          if constexpr (Ob) obSetMinSeq();
        }
        zamboni();
        stamp(z == 0 ? kPfZamboniOp : kPfWindow);
      }
      if (status != FMT_OK) {
        failSeq = op.seq;
        break;
      }
    }
  }

  FMT_DEV void writeOutputs(const DocOutputs& out) {
    if constexpr (Loc) {
      FOR_LANES(l) {
        if (l < 2) storeGlobal(in.loc->regenCount + 2 * in.doc + l, l == 0 ? regenN : regenTextN);
      }
    }
    if constexpr (Adj) {
      if (out.legacyProps != nullptr && status == FMT_OK && !savingHuge) {
        pmLegacyProps(out.legacyProps);
        if (status != FMT_OK) {
          // the legacy getAtSeq view did not fit the prop-set table. Small tier: escalate (the large
          // tier holds 1024 sets). Large tier: the replay state stands and only the legacy summary is
          // unavailable (kLegacyUnavailable: summaryRunsKernel and fmt_mt_fetch_legacy_props report
          // FMT_E_CAPACITY for this document).
          if constexpr (C::kHbmChars) {
            status = FMT_OK;
            FOR_LANES(l) {
              for (int t = l; t < n; t += 64) out.legacyProps[t] = kLegacyUnavailable;
            }
            waveSync();
          } else {
            status = FMT_E_CAPACITY;
          }
        }
      }
    }
    const int nr = rows();
    // char offsets and leaf-block ordinals
    Lane<VR> cst;
    charStarts(cst, nr);
    Lane<VR> startFlag, ord;
    FOR_ROWS(r, 0, nr) {
      const Lane<uint32_t> cur = row(W[0], r);
      const Lane<uint32_t> up = shflUp1(cur);
      const uint32_t carry = r > 0 ? readlane(row(W[0], r > 0 ? r - 1 : 0), 63) : 0u;
      FOR_LANES(l) {
        const int idx = r * 64 + l;
        const uint32_t pb = fBlk(l == 0 ? carry : LANE(up));
        LANE(startFlag)[r] = idx < n && (idx == 0 || fBlk(LANE(cur)) != pb) ? 1u : 0u;
      }
    }
    const uint32_t nLeafBlocks = scanRows(startFlag, ord, nr);
    uint32_t visible = 0;
    {
      Lane<VR> vlen, tmp;
      FOR_ROWS(r, 0, nr) {
        FOR_LANES(l) {
          const bool live = static_cast<int32_t>(LANE(W[2])[r]) == kNotRemoved;
          LANE(vlen)[r] = live ? fLen(LANE(W[0])[r]) : 0u;
        }
      }
      visible = scanRows(vlen, tmp, nr);
    }
    FOR_ROWS(r, 0, nr) {
      FOR_LANES(l) {
        const int idx = r * 64 + l;
        if (idx < n) {
          fmt_mt_leaf L;
          const uint32_t w0 = LANE(W[0])[r];
          L.ins_seq = static_cast<int32_t>(LANE(W[1])[r]);
          L.rm_seq = static_cast<int32_t>(LANE(W[2])[r]);
          L.rm_clients = LANE(W[3])[r];
          if constexpr (C::kWords > 5) L.rm_clients |= static_cast<uint64_t>(LANE(W[5])[r]) << 32;
          L.char_off = LANE(cst)[r];
          L.len = fLen(w0);
          L.ins_client = static_cast<int16_t>(fClient(LANE(W[4])[r]));
          const uint32_t pid = propsL(l, r);
          L.props = pid == kPropsUndef ? 0xFFFFu : static_cast<uint16_t>(pid);
          L.block = static_cast<uint16_t>(LANE(ord)[r] + LANE(startFlag)[r] - 1u);
          L.pad = fMarker(LANE(W[4])[r]) ? FMT_MT_LEAF_MARKER : 0u;
          out.leaves[idx] = L;
        }
      }
    }
    FOR_LANES(l) {
      if constexpr (!C::kHbmChars)
        for (int t = l; t < nChars; t += 64) out.chars[t] = s->chars[t];
    }
    {  // prop sets word by word (lane = one word of the flat table): no per-lane struct copies
      constexpr int kPW = 1 + FMT_MT_PROPS_MAX;
      uint32_t* dst = reinterpret_cast<uint32_t*>(out.props);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(s->props);
      FOR_LANES(l) {
        for (int t = l; t < nProps * kPW; t += 64) dst[t] = src[t];
      }
    }
    // remove-order entries: leaf id -> final leaf index (FMT_MT_LEAF_GONE once zamboni dropped it;
    // at a stop for the huge tier they keep their ids, which it goes on with)
    for (uint32_t k = 0; Rm && !savingHuge && k < rmN; k++) {
      const uint32_t id = uni(loadCoherent(&rmOut[k].leaf));
      const int j = findLeafById(id);
      FOR_LANES(l) {
        if (l == 0) rmOut[k].leaf = j >= 0 ? static_cast<uint32_t>(j) : FMT_MT_LEAF_GONE;
      }
    }
    int depth = 1;
    for (int b = root; uni(static_cast<int>(s->blk[b].leaf)) == 0 && uni(static_cast<int>(s->blk[b].count)) > 0;
         b = uni(static_cast<int>(s->blk[b].child[0])))
      depth++;
    FOR_LANES(l) {
      if (l == 0) {
        fmt_mt_doc_result h;
        h.status = status;
        h.fail_seq = failSeq;
        h.cur_seq = curSeq;
        h.min_seq = minSeq;
        h.n_leaves = static_cast<uint32_t>(n);
        h.n_chars = static_cast<uint32_t>(nChars);
        h.n_props = static_cast<uint32_t>(nProps);
        h.n_blocks = nLeafBlocks;
        h.depth = static_cast<uint32_t>(depth);
        h.visible_len = visible;
        h.n_catchup = cuN;
        h.n_rm_order = rmN;
        *out.header = h;
      }
    }
  }

  FMT_DEV void run(const DocInputs& inputs, const DocOutputs& out) {
#if FMT_PROFILE && FMT_GPU
    profT = __builtin_amdgcn_s_memtime();
#endif
    in = inputs;
    savingHuge = false;
    cuOut = out.catchup;
    cuCap = out.catchup ? out.catchupCap : 0u;
    cuN = 0;

    rmOut = out.rmOrder;
    rmCap = out.rmOrder ? out.rmOrderCap : 0u;
    rmN = 0;
    if constexpr (C::kHbmChars) gch = out.chars;
    ckpt = out.ckpt;
    init();
    uint64_t first = in.begin;
    bigCkpt = out.bigCkpt;
    bigCkptChars = out.bigCkptChars;
    if (kResumesCkpt && ckpt != nullptr && out.ckptResume) {
      first = restoreCkpt();  // (computed numbers: the slab and its count stay in memory)
    } else if (kResumesBig && bigCkpt != nullptr && out.ckptResume) {
      first = restoreBig();
    } else {
      if (in.adj != nullptr) {  // a fresh replay (also a restart in the next tier) starts an empty table
        FOR_LANES(l) {
          if (l == 0) storeGlobal(in.adj->numCount + in.doc, 0u);
        }
      }
      pmN = 0;
      if constexpr (Loc) {
        locSeq = 0;
        gHead = gTail = 0;
        recN = 0;
        recFrozen = false;
        regenN = regenTextN = 0;
        normSet = false;
      }
      if (in.loaded) loadSnapshot();
      else loadInitial();
    }
    hugeCkpt = out.hugeCkpt;
    if (status == FMT_OK) replay(first);
    if constexpr (kSavesHuge) {
      if (status == kCkptEscalate) {  // the huge tier resumes: the result slabs, then the record
        status = FMT_OK;
        savingHuge = true;
        writeOutputs(out);
        saveHuge(ckptNext);
        FOR_LANES(l) {
          if (l == 0) out.header->status = fmt_ckpt::kStatusHuge;
        }
        return;
      }
    }
    if ((kSavesCkpt || kSavesBig) && status == kCkptEscalate) {  // the next tier writes everything else
      if constexpr (!Ob && kSavesCkpt) saveCkpt(ckptNext);
      else if constexpr (!Ob && kSavesBig) saveBig(ckptNext);
      FOR_LANES(l) {
        if (l == 0) out.header->status = status;
      }
      return;
    }
    writeOutputs(out);
    stamp(kPfOutput);
  }
};

}  // namespace fmt_mt
