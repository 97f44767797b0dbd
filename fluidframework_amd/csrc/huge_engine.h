// huge_engine.h — merge-tree observer replay of ONE very large document (BASELINE config 5, T3:
// 10M segments, 64 clients, refSeq windows thousands of ops deep) on ONE wavefront, state in HBM.
//
// Same reference semantics as mt_engine.h (Client.applyMsg → insertSegments / markRangeRemoved /
// annotateRange, mergeTree.ts:1484-1517, 2009-2081, 2292-2383; zamboni.ts:33-213 with its LRU heap
// core-utils/src/heap.ts:54-182; setMinSeq mergeTree.ts:1147-1166), but the document no longer fits
// one wave's registers, so the leaf list is paged:
//
//   * Leaf blocks of the exact B+tree (≤ 8 leaves, mergeTreeNodes.ts:248) ARE the pages: each leaf
//     block stores its leaves inline (SoA fields, 8 slots). Interior blocks hold child block ids. The
//     tree decides zamboni scope and the segmentation summaries expose, so it is kept exactly.
//   * The leaf blocks in document order are listed by groups: gOrder (LDS) lists the groups in
//     document order; each group lists up to kSlotCap leaf blocks (HBM) with each block's stable
//     length. A block split inserts a slot; packParent removes slots; a full group splits.
//   * Length index (what PartialSequenceLengths is to the reference, partialLengths.ts:973-1005; only
//     an index, :1189-1240): a leaf's length from PriorPerspective(refSeq, client) differs from its
//     length at minSeq only if it was inserted or removed in the collaboration window. Such "window
//     leaves" are kept in a window table (HBM, a few thousand entries: one per leaf inserted or removed
//     above minSeq) tagged with their group and leaf block; every other leaf contributes its fixed
//     length to its block's and group's stable sums. Resolving a view position is then: one pass of
//     the wave over the window table (per-group corrections, LDS atomics) + a scan over the groups
//     (LDS), a scan over one group's slots (two coalesced loads per 64 slots + that group's window
//     corrections), and the ≤ 8 leaves of one block evaluated directly.
//   * When minSeq advances, window entries whose insert and remove are both at or below it graduate
//     into the stable sums (their length no longer depends on the perspective).
//   * The LRU heap (verbatim heap.ts sift order) lives in LDS. Text: each leaf names a run of one
//     UTF-16 arena (the batch's text, then a merge area where zamboni appends build their text).
//
// Every decision that mt_engine.h makes with a view scan over all leaves is made here on the first
// qualifying leaf of the hierarchical search (the same flat rules, proven there against the oracle):
//   ensureIntervalBoundary: split the leaf that strictly contains pos in the op's view;
//   insert: before the first leaf whose view start is pos, skipping leaves removed at/below minSeq
//           except the very last leaf (mergeTree.ts:1862-1875), into that leaf's block; past the
//           end into the last leaf's block;
//   nodeMap: the leaves of positive view length inside [start, end).
#pragma once

#include "../../include/fmt.h"
#include "wave.h"
#include "adjust.h"
#include "huge_ckpt.h"

#include <algorithm>
#include <vector>

namespace fmt_huge {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kMaxNodes = 8;          // MaxNodesInBlock (mergeTreeNodes.ts:248)
constexpr int kGranularity = 256;     // TextSegmentGranularity (textSegment.ts:21)
constexpr int32_t kNotRemoved = 0x7fffffff;
#ifndef FMT_HUGE_SLOTCAP  // (the emulation tests also build tiny groups to exercise group splits)
#define FMT_HUGE_SLOTCAP 2048
#define FMT_HUGE_FILL 1024
#endif
constexpr int kSlotCap = FMT_HUGE_SLOTCAP;  // leaf blocks listed per group
constexpr int kGroupCap = 2048;       // groups
constexpr int kHeapCap = 10240;       // LRU heap entries (≈ blocks registered in one window)
constexpr int kPropCap = 65534;       // interned prop sets per document (ids fit the meta word's 16 bits)
constexpr int kPropLds = 2048;        // match classes of the first sets cached in LDS
constexpr uint32_t kPropHash = 1u << 17;  // buckets per prop-set hash table (exact content, match class)
constexpr int kPropWords = 1 + FMT_MT_PROPS_MAX;  // a prop set in HBM: n, kv[]
constexpr int kKeyChunks = FMT_MT_PROPS_KEYS_MAX / 64;  // working-set slot k = chunk k / 64, lane k % 64
static_assert(FMT_MT_PROPS_KEYS_MAX % 64 == 0, "prop-set slots come in whole waves");
constexpr int kFill = FMT_HUGE_FILL;  // leaf blocks per group at load
// short client ids 0..253 (0xFE: FMT_MT_CLIENT_NONCOLLAB); remove-client sets: two mask words for ids
// 0..63 + HugeState::hiMask, kHiWords per leaf id for ids 64..253 (round 6: was 127, two words)
constexpr int kMaxClient = 253;
constexpr int kHiWords = (kMaxClient + 1 - 64 + 31) / 32;
constexpr int kHiOutWords = kHiWords / 2;  // (writeOutputs: 64-bit words per leaf, ids 64..127, 128..191, 192..255)

// Leaf meta word: insert client (int8) | prop set id << 8 (0xFFFF = properties undefined)
// (0..253 a short id; 0xFE NonCollab = -2, 0xFF = -1: the reference's special client ids)
FMT_DEV int32_t mClient(uint32_t m) {
  const int32_t v = static_cast<int32_t>(m & 0xFFu);
  return v >= 0xFE ? v - 256 : v;
}
FMT_DEV uint32_t mProps(uint32_t m) { return (m >> 8) & 0xFFFFu; }
FMT_DEV uint32_t mkMeta(int32_t client, uint32_t props) { return (static_cast<uint32_t>(client) & 0xFFu) | (props << 8); }
constexpr uint32_t kMetaMarker = 1u << 24;  // the leaf is a Marker (mergeTreeNodes.ts:495-564)
FMT_DEV bool mMarker(uint32_t m) { return (m & kMetaMarker) != 0; }
constexpr uint32_t kNoProps = 0xFFFFu;
FMT_DEV uint32_t mix32(uint32_t x) {  // (a 32-bit finalizer: prop-set hashes)
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  return x ^ (x >> 16);
}

// Window meta word: insert client (int8) | first remover (u8) << 8 | "more removers" << 16; the
// record's word 3 adds the entry's group << 17
// NOT reliable after a large → huge checkpoint (loadFromLarge): the large tier keeps the remove-client
// set, not which remover came first, so the lowest id stands in there. Nothing reads it today (the
// passes use the set; SnapshotV1's removedClientIds come from the op at the leaf's rm_seq and the
// remove-order entries, which the checkpoint carries); a future reader must carry the first remover
// through huge_ckpt.h first.
FMT_DEV uint32_t wFirstRm(uint32_t m) { return (m >> 8) & 0xFFu; }
constexpr uint32_t kWMetaMask = 0x1FFFFu;
constexpr int kWGroupShift = 17;
// The first kWinLds window entries are mirrored in LDS (HugeLds::wRecL / wMaskL; HBM stays the
// authoritative copy and every write updates both): the per-op window passes read them there instead
// of issuing L2 round trips (round 6). T3 keeps about 1.2k entries in its window.
constexpr uint32_t kWinLds = 1280;

// One live obliterate (mergeTree.ts ObliterateInfo) is a 6-word record of HugeState::obRec: its
// endpoint references as (leaf id, offset) — id 0 once the reference is removed — and its stamp.

typedef uint32_t u32x4 __attribute__((vector_size(16)));
typedef uint32_t u32x2 __attribute__((vector_size(8)));
FMT_DEV u32x2 ld2(const uint32_t* p) {  // one 8-byte vector load (p 8-byte aligned)
#if FMT_GPU
  return *reinterpret_cast<const u32x2*>(p);
#else
  u32x2 v;
  __builtin_memcpy(&v, p, sizeof v);
  return v;
#endif
}
FMT_DEV u32x4 ld4(const uint32_t* p) {  // one 16-byte vector load (p 16-byte aligned)
#if FMT_GPU
  return *reinterpret_cast<const u32x4*>(p);
#else
  u32x4 v;
  __builtin_memcpy(&v, p, sizeof v);
  return v;
#endif
}

// HugeState's / HugeInputs' buffers are global memory: typed so in the kernel (hugedoc.hip), every
// access to them is a global load/store (SGPR base + lane offset) instead of a flat one, which would
// also count against the LDS counter and make each LDS wait wait for the outstanding HBM loads (T3
// slice 9.84 -> 9.72 s, profiles/r5/ab/ab_t3_chunks_global.json). Host code that fills the structs
// sees plain pointers (same layout).
#if FMT_GPU && defined(FMT_HUGE_KERNEL)
#define FMT_HBM __attribute__((address_space(1)))
#else
#define FMT_HBM
#endif

struct HeapEnt {
  int32_t maxSeq;
  uint32_t leafId;
};

// Device buffers of one huge document (all sized by the runtime from host-side bounds).
struct HugeState {
  // leaf fields, [blockCap * 8]: slot k of leaf block b at b * 8 + k
  FMT_HBM uint32_t* lLen;
  FMT_HBM int32_t* lIns;
  FMT_HBM int32_t* lRm;
  FMT_HBM uint32_t* lMlo;
  FMT_HBM uint32_t* lMhi;
  FMT_HBM uint32_t* lId;
  FMT_HBM uint32_t* lText;
  FMT_HBM uint32_t* lMeta;
  // blocks [blockCap]
  FMT_HBM uint32_t* bCount;
  FMT_HBM uint32_t* bParent;
  FMT_HBM uint32_t* bLeaf;
  FMT_HBM int32_t* bScour;
  FMT_HBM uint32_t* bChild;   // [blockCap * 8] (interior blocks)
  FMT_HBM uint32_t* bGroup;   // leaf blocks: group id
  FMT_HBM uint32_t* bSlot;    // leaf blocks: slot in the group
  FMT_HBM uint32_t* freeBlk;  // [blockCap] stack of freed block ids
  uint32_t blockCap;
  // groups [kGroupCap * kSlotCap]
  FMT_HBM uint32_t* gSlotBlk;
  FMT_HBM int32_t* gSlotStable;
  // leaf id → leaf block / window entry, [idCap]
  FMT_HBM uint32_t* leafBlk;
  FMT_HBM uint32_t* winIdx;
  uint32_t idCap;
  // window table [winCap]: one 16-byte record per entry {ins, rm, len, meta | group << 17} (one
  // vector load per entry in the window passes), plus the entry's leaf block and leaf id
  FMT_HBM uint32_t* wRec;
  FMT_HBM uint32_t* wMask;  // [winCap * 2]: the leaf's remove-client set (lo, hi), loaded with the record
  FMT_HBM uint32_t* wBlk;
  FMT_HBM uint32_t* wLeaf;
  uint32_t winCap;
  // text arena, one offset space: [0, textLen) is the batch's shared text (read in place through
  // base, never copied per document); [textLen, textCap) is this document's merge area, addressed
  // through text (its allocation minus textLen units, so text + off is valid for off >= textLen)
  const FMT_HBM uint16_t* base;
  FMT_HBM uint16_t* text;
  uint64_t textLen;   // batch text (read-only part)
  uint64_t textCap;   // end of the merge area: two halves of (textCap - textLen) / 2 units, one in use
  FMT_HBM uint32_t* props;    // [kPropCap * kPropWords]: n, kv[FMT_MT_PROPS_MAX]
  FMT_HBM uint32_t* pClass;   // [kPropCap]: prop set id -> its match class (the first set with the same content)
  FMT_HBM uint32_t* pHead;    // [2 * kPropHash]: bucket heads (set id + 1, 0 = empty), exact content then class
  FMT_HBM uint32_t* pNext;    // [2 * kPropCap]: per set, the next set of its exact-content / class bucket
  FMT_HBM uint32_t* cuIds;    // [idCap]: the current catch-up op's delta leaves in document order (or nullptr)
  FMT_HBM uint32_t* rmIds;    // [idCap]: the current remove-order op's already-removed hits; at output, leaf id ->
                      // output index (or nullptr: no remove-order recording)
  FMT_HBM uint32_t* mkIds;    // [mkCap]: every marker leaf ever in the document, in insertion order (relative
  uint32_t mkCap;     //   positions; nullptr: the batch has none)
  FMT_HBM uint32_t* outIdx;   // [idCap]: at output, leaf id -> output index (annotate-adjust batches; else nullptr)
  // [idCap * kHiWords]: per leaf id, the remove clients with short ids 64..253 (bit c - 64), beyond the
  // two mask words every leaf and window entry carry (nullptr: the batch has no such client; zeroed)
  FMT_HBM uint32_t* hiMask;
  // live obliterates (Obliterates, mergeTree.ts:515-635), [obCap] each: per slot its record
  // {startId, startOff, endId, endOff, seq, client} (obRec, 6 words) and whether it is in use, and the
  // two ordered slot lists seqOrdered / startOrdered (nullptr / 0: the document has no obliterate;
  // obCap = its obliterate ops, the most that can be live at once)
  FMT_HBM uint32_t* obRec;
  FMT_HBM uint32_t* obUsed;
  FMT_HBM uint32_t* obSeq;
  FMT_HBM uint32_t* obStart;
  uint32_t obCap;
};

// LDS state of the wave.
struct HugeLds {
  // window entries [0, kWinLds): their 16-byte records and remove-client masks (HugeState::wRec / wMask)
  alignas(16) uint32_t wRecL[kWinLds * 4];
  alignas(16) uint32_t wMaskL[kWinLds * 2];
  uint16_t gOrder[kGroupCap];    // group ids in document order
  int32_t gStable[kGroupCap];    // by group id: Σ stable lengths of its slots
  uint16_t gCount[kGroupCap];    // by group id: slots (<= kSlotCap)
  int32_t gCorr[kGroupCap];      // by group id: window correction of the current perspective
  // chunks of 32 group positions (document order): the group scan's first level
  uint16_t gPos[kGroupCap];      // by group id: its position in gOrder
  int32_t cStable[kGroupCap / 32];  // by chunk: Σ gStable of its groups
  int32_t cCorr[kGroupCap / 32];    // by chunk: Σ gCorr of its groups (the current perspective)
  int32_t sLen[kSlotCap];        // the group being searched: view length per slot
  uint32_t sBlk[kSlotCap];
  HeapEnt heap[kHeapCap + 1];    // 1-based (heap.ts)
  uint32_t tmp[128];             // (indices < 128: a split's counts [0, 64) and sources [64, 128))
  uint16_t pClass[kPropLds];     // S.pClass of the first kPropLds sets
  uint32_t kvWork[FMT_MT_PROPS_KEYS_MAX];  // applyProps' working set (slot k = entry k)
  int32_t cmd[8];                // pass command from wave 0 to the helper waves (HugeDoc::PassCmd)
};

struct HugeInputs {
  const FMT_HBM fmt_mt_op* ops;
  uint64_t begin, end;
  const FMT_HBM uint32_t* propsOff;
  const FMT_HBM uint32_t* propsKv;
  uint32_t nPropsOps;
  const FMT_HBM fmt_mt_snapshot_seg* segs;  // loaded segments: the header chunk, then the body chunk(s)
  uint32_t nSegs;
  // Tree shape of the loaded segments when a body follows the header (nullptr: the header alone,
  // reloaded 7 wide): [L, n_0 .. n_{L-1}, then per level its n_l nodes as (start, count)] —
  // level 0 the leaf blocks (start: first segment), level l > 0 interior blocks (start: first
  // child on level l - 1), level L - 1 the root. Built on the host by loadShape below.
  const FMT_HBM uint32_t* shape;
  int32_t snapMinSeq, snapSeq;
  // client of the loaded segments' insert stamp: FMT_NON_COLLAB_CLIENT for a summary's segments
  // (specToSegment, snapshotLoader.ts:180-186), FMT_LOCAL_CLIENT for a document's initial text (the
  // replay harness inserts it locally before collaborating, client.replay.spec.ts:30-33)
  int32_t initClient;
  uint32_t segProps;  // some loaded segment has properties
  // SnapshotV1 merge info of the loaded segments (aligned with segs; nullptr: none) and the batch's
  // remove stamps its rows index (specToSegment, snapshotLoader.ts:105-175)
  const FMT_HBM fmt_mt_snapshot_info* info;
  const FMT_HBM fmt_mt_stamp* stamps;
  // the batch's whole merge-info table: V1 body-chunk segments with merge info arrive as
  // FMT_MT_F_LOADSEG insert ops naming a row of it (nullptr: none in the batch)
  const FMT_HBM fmt_mt_snapshot_info* infoAll;
  uint64_t nInfoAll;
  // catch-up ranges of FMT_MT_F_CATCHUP ops (the document's slab; nullptr: the batch records none)
  FMT_HBM fmt_mt_catchup_range* catchup;
  uint32_t catchupCap;
  // remove-order entries of FMT_MT_F_RMORDER ops (the document's slab; nullptr: none recorded)
  FMT_HBM fmt_mt_remove_order* rmOrder;
  uint32_t rmOrderCap;
  // legacy relative positions (FMT_MT_F_REL1/REL2 ops index the table; nullptr: none in the batch)
  const FMT_HBM fmt_mt_relpos* relpos;
  uint32_t nRelpos;
  uint32_t markerKey;  // key id of "markerId"
  // annotate-adjust (nullptr: none in the batch): the batch's tables (adjust.h), this document's
  // index into their per-document slabs (computed numbers, PropertiesManager records)
  const FMT_HBM fmt_mt::AdjustTables* adj;
  uint32_t doc;
  // large → huge checkpoint (huge_ckpt.h; nullptr: load from the segments above): the large tier's
  // record and its result slabs for this document at the op it stopped before
  const FMT_HBM uint32_t* ck = nullptr;
  const FMT_HBM fmt_mt_leaf* ckLeaves = nullptr;
  const FMT_HBM uint16_t* ckChars = nullptr;
  const FMT_HBM fmt_mt_propset* ckProps = nullptr;
};

// The tree a legacy summary loads into (huge_engine.h HugeInputs::shape): reloadFromSegments of the
// header — 7 leaves per block, 7 blocks per interior block up to one root (mergeTree.ts:751-800) —
// then loadBody's appends (snapshotLoader.ts:277-309), each into the last leaf block, a full block
// (MaxNodesInBlock) splitting 4 / 4 and the split climbing the right edge, a new root above a split
// root (mergeTree.ts:1946-1987; an empty root first becomes the leaf block). Only the right edge
// changes, so this tracks node counts per level. (Host code: the runtime and the emulation tests.)
inline void loadShape(uint64_t nHeader, uint64_t nBody, std::vector<uint32_t>& out) {
  std::vector<std::vector<uint32_t>> lv;
  if (nHeader > 0) {
    uint64_t below = nHeader;
    do {
      std::vector<uint32_t> level;
      for (uint64_t q = 0; q * 7 < below; q++) level.push_back(static_cast<uint32_t>(std::min<uint64_t>(7, below - 7 * q)));
      below = level.size();
      lv.push_back(std::move(level));
    } while (below > 1);
  }
  for (uint64_t i = 0; i < nBody; i++) {
    if (lv.empty()) lv.push_back({0});
    lv[0].back()++;
    for (size_t l = 0; lv[l].back() == kMaxNodes; l++) {
      lv[l].back() = kMaxNodes / 2;
      lv[l].push_back(kMaxNodes / 2);
      if (l + 1 == lv.size()) {
        lv.push_back({2});
        break;
      }
      lv[l + 1].back()++;
    }
  }
  out.assign(1, static_cast<uint32_t>(lv.size()));
  for (const auto& level : lv) out.push_back(static_cast<uint32_t>(level.size()));
  for (const auto& level : lv) {
    uint32_t st = 0;
    for (uint32_t cnt : level) {
      out.push_back(st);
      out.push_back(cnt);
      st += cnt;
    }
  }
}

// A leaf found by the hierarchical search.
struct Hit {
  bool found;
  int gpos;        // position of its group in gOrder
  int slot;        // slot of its block in the group
  uint32_t blk;
  int k;           // slot in the block
  int st;          // view start of the leaf
  int vis;         // view length of the leaf
};

// Adj: the variant for batches with annotate-adjust (the fold and the PropertiesManager records);
// Rm: the variant for batches that record the SnapshotV1 remove order (FMT_MT_F_RMORDER ops).
// Batches without them run code that has none of it in its op loop (the remove-order hooks alone
// cost a T3 slice 39%: 6.55 s -> 9.12 s, profiles/r4/ab_t3_bisect.json).
template <bool Adj = false, bool Rm = false>
class HugeDocT {
 public:
  HugeState S;
  HugeLds* L;
  HugeInputs in;
  int root = 0;
  int nGroups = 0;
  uint32_t nextBlock = 0, nFree = 0;
  int nProps = 0;
  uint32_t nextId = 1;
  uint32_t nWin = 0;
  uint64_t textTop = 0;
  int heapN = 0;
  int curSeq = 0, minSeq = 0;
  int status = FMT_OK, failSeq = 0;
  uint32_t lastBlk = kNone;  // the last leaf block in document order (kNone: document empty)
  int obLive = 0, obSeqN = 0, obStartN = 0, obSlotsHi = 0;
  uint64_t mergeLo = 0, mergeHi = 0;  // the merge-area half in use
  bool textFull = false;              // a scour plan's runs did not fit the merge area's half
  // catch-up recording (FMT_MT_F_CATCHUP ops): ranges written, the op's delta leaves, its index
  uint32_t cuN = 0, cuIdN = 0, opIdx = 0;
  bool cuRec = false;
  // remove-order recording (FMT_MT_F_RMORDER ops, SnapshotV1): entries written, the op's hits on
  // leaves already removed, split copies pending (at most two splits per op), the op's stamp kind
  uint32_t rmN = 0, rmHitN = 0;
  bool rmRec = false;
  int rmPendN = 0;
  // (named scalars, not arrays: an array member indexed by a counter sends the whole engine object to
  // scratch memory)
  uint32_t rmPendFrom0 = 0, rmPendTo0 = 0, rmPendFrom1 = 0, rmPendTo1 = 0;
  uint32_t rmKind = FMT_MT_RM_SET;
  uint32_t mkN = 0;  // markers listed in S.mkIds
  int pmN = 0;       // PropertiesManager records in use (deleted ones included), annotate-adjust batches
  // shader-clock totals per phase (diagnostics, written to HugeOut::prof; inclusive, so nested phases
  // overlap): 0 replay, 1 window pass (groups), 2 window pass (slots), 3 zamboni, 4 graduation,
  // 5 load, 6 output, 7 finds, 8 scour, 9 leaf-parent pack, 10 slot insert/remove, 11 heap,
  // 12 insert, 13 range ops, 14 leaf split, 15 interior pack; counts: 16 group passes, 17 slot
  // passes, 18 Σ window entries at group passes, 19 Σ groups at group passes; 20 wave 0's window
  // share time, 21 group scan time, 22 merge-area compactions, 23 merge-area units in use
  static constexpr int kProf = 25;  // [24]: the op a large → huge checkpoint resumed at
  uint64_t prof[kProf] = {};
  struct ProfScope {
    uint64_t& a;
    uint64_t t;
    FMT_DEV explicit ProfScope(uint64_t& acc) : a(acc), t(clk()) {}
    FMT_DEV ~ProfScope() { a += clk() - t; }
  };
  FMT_DEV static uint64_t clk() {
#if FMT_GPU
    return __builtin_amdgcn_s_memtime();
#else
    return 0;
#endif
  }
  bool corrValid = false;    // gCorr holds the current op's perspective
  uint32_t epoch = 0;        // bumped by every change of the index (window table, slots, stable sums)
  uint32_t slotCacheG = kNone, slotCacheEpoch = 0;  // sLen / sBlk hold group slotCacheG at that epoch
  FMT_DEV void invalidate() {
    corrValid = false;
    epoch++;
  }

  FMT_DEV bool fail(int code, int line = __builtin_LINE()) {
#ifdef FMT_HUGE_CHECK
    if (status == FMT_OK && std::getenv("FMT_HUGE_TRACE")) std::fprintf(stderr, "huge_engine.h:%d fails %d\n", line, code);
#else
    (void)line;
#endif
    if (status == FMT_OK) status = code;
    return false;
  }

  // ------------------------------------------------------------------ small helpers
  // Reads of HBM state: plain vector loads served by this CU's L1 (which the wave's own stores keep
  // current; no other CU writes this document's state; the helper waves read after a workgroup
  // barrier). They were workgroup-scope atomic loads until round 5: an atomic load is an ordered
  // memory reference to the scheduler, so independent loads issued one round trip at a time (T3
  // slice 9.69 -> 9.16 s as plain loads, profiles/r5/ab/ab_t3_plainrd.json; the kernel's scalar
  // loads stay the 142 of its arguments: the compiler picks a scalar load only where no store of
  // this kernel can reach it). rd() inside FOR_LANES bodies, ldu()/ldi() for wave-uniform values.
  FMT_DEV static uint32_t rd(const uint32_t* p) { return *p; }
  FMT_DEV static int32_t rd(const int32_t* p) { return *p; }
  FMT_DEV static uint32_t ldu(const uint32_t* p) { return uni(*p); }
  FMT_DEV static int32_t ldi(const int32_t* p) { return uni(*p); }
  // one text unit at arena offset off (batch text below textLen, the merge area above)
  FMT_DEV uint32_t textAt(uint64_t off) const {
    return loadWg((off < S.textLen ? S.base : static_cast<const FMT_HBM uint16_t*>(S.text)) + off);
  }
  // one lane stores a wave-uniform value
  template <class P, class T>
  FMT_DEV static void st1(P* p, T v) {
    FOR_LANES(l) {
      if (l == 0) *p = v;
    }
  }
  FMT_DEV static bool removedBy(uint32_t mlo, uint32_t mhi, int c) {
    return c < 32 ? ((mlo >> c) & 1u) != 0 : ((mhi >> (c - 32)) & 1u) != 0;
  }
  // leaf length from PriorPerspective(r, c) (perspective.ts:80-93), c < 64
  FMT_DEV static int visOf(uint32_t len, int32_t ins, int32_t rm, uint32_t mlo, uint32_t mhi, int32_t ic, int r, int c) {
    const bool present = (ins <= r || ic == c) && !(rm <= r || removedBy(mlo, mhi, c));
    return present ? static_cast<int>(len) : 0;
  }
  // ---- remove clients 64..253 (getOrAddShortClientId interns without bound, client.ts:831-855): a
  // per-leaf-id side table; a perspective of such a client (wave-uniform c) reads it, others never do
  // (a set of them in registers: bit c - 64 of w)
  struct HiSet {
    uint32_t w[kHiWords];
    FMT_DEV void clear() {
      for (int k = 0; k < kHiWords; k++) w[k] = 0u;
    }
    FMT_DEV void add(int c) { w[(c - 64) >> 5] |= 1u << ((c - 64) & 31); }
    FMT_DEV int count() const {
      int n = 0;
      for (int k = 0; k < kHiWords; k++) n += __builtin_popcount(w[k]);
      return n;
    }
  };
  FMT_DEV bool hiRemovedBy(uint32_t id, int c) const {
    const uint32_t b = static_cast<uint32_t>(c - 64);
    return ((rd(S.hiMask + kHiWords * static_cast<size_t>(id) + (b >> 5)) >> (b & 31u)) & 1u) != 0;
  }
  // PriorPerspective(r, c) of leaf `id` for any c (the mask words for c < 64, the side table above)
  FMT_DEV int visAny(uint32_t len, int32_t ins, int32_t rm, uint32_t mlo, uint32_t mhi, int32_t ic, int r, int c,
                     uint32_t id) const {
    if (c < 64) return visOf(len, ins, rm, mlo, mhi, ic, r, c);
    const bool present = (ins <= r || ic == c) && !(rm <= r || (S.hiMask != nullptr && hiRemovedBy(id, c)));
    return present ? static_cast<int>(len) : 0;
  }
  FMT_DEV void hiSet(uint32_t id, int c) {  // (c in 64..253, S.hiMask present)
    const uint32_t b = static_cast<uint32_t>(c - 64);
    uint32_t* p = S.hiMask + kHiWords * static_cast<size_t>(id) + (b >> 5);
    const uint32_t v = ldu(p) | (1u << (b & 31u));
    st1(p, v);
  }
  FMT_DEV void hiPut(uint32_t id, const HiSet& h) {
    FOR_LANES(l) {
      if (l == 0)
        for (int k = 0; k < kHiWords; k++) S.hiMask[kHiWords * static_cast<size_t>(id) + k] = h.w[k];
    }
  }
  FMT_DEV HiSet hiGet(uint32_t id) const {
    HiSet h;
    for (int k = 0; k < kHiWords; k++) h.w[k] = ldu(S.hiMask + kHiWords * static_cast<size_t>(id) + k);
    return h;
  }
  FMT_DEV int hiCount(uint32_t id) const { return S.hiMask == nullptr ? 0 : hiGet(id).count(); }

  FMT_DEV uint32_t allocBlk(uint32_t leaf) {
    uint32_t b;
    if (nFree > 0) {
      b = ldu(S.freeBlk + --nFree);
    } else {
      if (nextBlock >= S.blockCap) {
        fail(FMT_E_CAPACITY);
        return kNone;
      }
      b = nextBlock++;
    }
    st1(S.bCount + b, 0u);
    st1(S.bParent + b, kNone);
    st1(S.bLeaf + b, leaf);
    st1(S.bScour + b, -1);
    return b;
  }
  FMT_DEV void freeBlock(uint32_t b) {
    st1(S.freeBlk + nFree, b);
    nFree++;
  }

  // ------------------------------------------------------------------ window table
  FMT_DEV uint32_t winAdd(uint32_t id, int32_t ins, int32_t rm, uint32_t len, uint32_t meta, uint32_t grp, uint32_t blk,
                         uint32_t mlo = 0, uint32_t mhi = 0) {
    invalidate();
    if (nWin >= S.winCap) {
      fail(FMT_E_CAPACITY);
      return kNone;
    }
    const uint32_t w = nWin++;
    FOR_LANES(l) {
      if (l == 0) {
        uint32_t* rec = S.wRec + static_cast<size_t>(w) * 4;
        rec[0] = static_cast<uint32_t>(ins);
        rec[1] = static_cast<uint32_t>(rm);
        rec[2] = len;
        rec[3] = (meta & kWMetaMask) | (grp << kWGroupShift);
        S.wMask[2 * w] = mlo;
        S.wMask[2 * w + 1] = mhi;
        S.wBlk[w] = blk;
        S.wLeaf[w] = id;
        S.winIdx[id] = w;
      }
    }
    if (w < kWinLds) {  // (uniform LDS stores)
      L->wRecL[4 * w] = static_cast<uint32_t>(ins);
      L->wRecL[4 * w + 1] = static_cast<uint32_t>(rm);
      L->wRecL[4 * w + 2] = len;
      L->wRecL[4 * w + 3] = (meta & kWMetaMask) | (grp << kWGroupShift);
      L->wMaskL[2 * w] = mlo;
      L->wMaskL[2 * w + 1] = mhi;
    }
    return w;
  }
  FMT_DEV void winRemove(uint32_t w) {  // swap-remove
    invalidate();
    const uint32_t last = nWin - 1;
    const uint32_t id = ldu(S.wLeaf + w);
    if (w != last) {
      const uint32_t* src = S.wRec + static_cast<size_t>(last) * 4;
      const uint32_t a = ldu(src), b = ldu(src + 1), c = ldu(src + 2), d = ldu(src + 3);
      const uint32_t ml = ldu(S.wMask + 2 * last), mh = ldu(S.wMask + 2 * last + 1);
      const uint32_t f = ldu(S.wBlk + last), g = ldu(S.wLeaf + last);
      FOR_LANES(l) {
        if (l == 0) {
          uint32_t* rec = S.wRec + static_cast<size_t>(w) * 4;
          rec[0] = a;
          rec[1] = b;
          rec[2] = c;
          rec[3] = d;
          S.wMask[2 * w] = ml;
          S.wMask[2 * w + 1] = mh;
          S.wBlk[w] = f;
          S.wLeaf[w] = g;
          S.winIdx[g] = w;
        }
      }
      if (w < kWinLds) {
        L->wRecL[4 * w] = a;
        L->wRecL[4 * w + 1] = b;
        L->wRecL[4 * w + 2] = c;
        L->wRecL[4 * w + 3] = d;
        L->wMaskL[2 * w] = ml;
        L->wMaskL[2 * w + 1] = mh;
      }
    }
    st1(S.winIdx + id, kNone);
    nWin = last;
  }

  FMT_DEV uint32_t* wWord(uint32_t w, int f) const { return S.wRec + static_cast<size_t>(w) * 4 + f; }
  FMT_DEV uint32_t* wWord3(uint32_t w) const { return wWord(w, 3); }
  // (uniform w) record word f of entry w, in HBM and in the LDS mirror
  FMT_DEV void wSet(uint32_t w, int f, uint32_t v) {
    st1(wWord(w, f), v);
    if (w < kWinLds) L->wRecL[4 * w + f] = v;
  }
  FMT_DEV void wSetMask(uint32_t w, uint32_t lo, uint32_t hi) {
    st1(S.wMask + 2 * w, lo);
    st1(S.wMask + 2 * w + 1, hi);
    if (w < kWinLds) {
      L->wMaskL[2 * w] = lo;
      L->wMaskL[2 * w + 1] = hi;
    }
  }
  // (lane-level) an entry's leaf moved to block b (of group g)
  FMT_DEV void wRetag(uint32_t w, uint32_t b, uint32_t g) {
    S.wBlk[w] = b;
    const uint32_t v = (rd(wWord3(w)) & kWMetaMask) | (g << kWGroupShift);
    *wWord3(w) = v;
    if (w < kWinLds) L->wRecL[4 * w + 3] = v;
  }
  // (lane-level) the record and mask of entry w for a pass: from the LDS mirror when it holds it
  FMT_DEV u32x4 wRecOf(uint32_t w) const {
    return w < kWinLds ? *reinterpret_cast<const u32x4*>(&L->wRecL[4 * w]) : ld4(S.wRec + static_cast<size_t>(w) * 4);
  }
  FMT_DEV u32x2 wMaskOf(uint32_t w) const {
    return w < kWinLds ? *reinterpret_cast<const u32x2*>(&L->wMaskL[2 * w]) : ld2(S.wMask + static_cast<size_t>(w) * 2);
  }

  // ------------------------------------------------------------------ stable sums
  // gStable[g] += delta, and its chunk's sum (wave-uniform: every lane stores the same value)
  FMT_DEV void stableAdd(uint32_t g, int delta) {
    L->gStable[g] += delta;
    L->cStable[L->gPos[g] >> 5] += delta;
  }
  // Group positions and chunk sums from gOrder / gStable (at load, and after a group split moved
  // the positions of the groups after it).
  FMT_DEV void chunksRebuild() {
    FOR_LANES(l) {
      for (int k = l; k < nGroups; k += 64) L->gPos[L->gOrder[k]] = static_cast<uint16_t>(k);
    }
    waveSync();
    FOR_LANES(l) {
      if (l < kGroupCap / 32) {
        int32_t sum = 0;
        for (int k = l * 32; k < l * 32 + 32 && k < nGroups; k++) sum += L->gStable[L->gOrder[k]];
        L->cStable[l] = sum;
      }
    }
    waveSync();
  }

  // Stable length of a leaf: its length for every perspective at/above minSeq (non-window leaves).
  FMT_DEV void addStable(uint32_t blk, int delta) {
    invalidate();
    if (delta == 0) return;
    const uint32_t g = ldu(S.bGroup + blk), s = ldu(S.bSlot + blk);
    int32_t* p = S.gSlotStable + static_cast<size_t>(g) * kSlotCap + s;
    const int32_t v = ldi(p);
    st1(p, v + delta);
    stableAdd(g, delta);  // (uniform LDS stores)
    waveSync();
  }

  FMT_DEV void addStableAt(uint32_t g, uint32_t s, int delta) {  // block in slot s of group g
    invalidate();
    int32_t* p = S.gSlotStable + static_cast<size_t>(g) * kSlotCap + s;
    const int32_t v = ldi(p);
    st1(p, v + delta);
    stableAdd(g, delta);
    waveSync();
  }

  // ------------------------------------------------------------------ group lists
  FMT_DEV uint32_t* slotBlkPtr(uint32_t g) const { return S.gSlotBlk + static_cast<size_t>(g) * kSlotCap; }
  FMT_DEV int32_t* slotStPtr(uint32_t g) const { return S.gSlotStable + static_cast<size_t>(g) * kSlotCap; }

  FMT_DEV int groupPos(uint32_t g) const {  // position of group g in gOrder
    for (int base = 0; base < nGroups; base += 64) {
      Lane<bool> p;
      FOR_LANES(l) { LANE(p) = base + l < nGroups && L->gOrder[base + l] == g; }
      const uint64_t m = ballot(p);
      if (m) return base + ctz64(m);
    }
    return -1;
  }

  static constexpr int kShiftU = 4;  // slot-list passes: 4 x 64 slots per step

  // Insert leaf block nb into group g at slot `at` with stable length st (slots at/after shift up).
  // Splits the group first when it is full; returns false on failure.
  FMT_DEV bool slotInsert(uint32_t g, int at, uint32_t nb, int st) {
    ProfScope ps_(prof[10]);
    invalidate();
    int cnt = static_cast<int>(L->gCount[g]);
    if (cnt >= kSlotCap) {
      if (!groupSplit(g)) return false;
      cnt = static_cast<int>(L->gCount[g]);
      if (at > cnt) {  // the slot moved to the new group (half full: no second split)
        const int gp = groupPos(g);
        g = L->gOrder[gp + 1];
        at -= cnt;
        cnt = static_cast<int>(L->gCount[g]);
      }
    }
    uint32_t* sb = slotBlkPtr(g);
    int32_t* ss = slotStPtr(g);
    // shift [at, cnt) up by one, top-down in chunks of kShiftU x 64 slots: a chunk's loads are all in
    // flight before its stores (it writes only into slots the chunk above has already read)
    for (int top = cnt - 1; top >= at; top -= 64 * kShiftU) {
      Lane<uint32_t> b[kShiftU];
      Lane<int32_t> st[kShiftU];
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < kShiftU; u++) {
          const int i = top - 64 * u - l;
          if (i >= at) {
            LANE(b[u]) = rd(sb + i);
            LANE(st[u]) = rd(ss + i);
          }
        }
      }
      waveSync();
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < kShiftU; u++) {
          const int i = top - 64 * u - l;
          if (i >= at) {
            sb[i + 1] = LANE(b[u]);
            ss[i + 1] = LANE(st[u]);
            S.bSlot[LANE(b[u])] = static_cast<uint32_t>(i + 1);
          }
        }
      }
      waveSync();
    }
    FOR_LANES(l) {
      if (l == 0) {
        sb[at] = nb;
        ss[at] = st;
        S.bSlot[nb] = static_cast<uint32_t>(at);
        S.bGroup[nb] = g;
      }
    }
    L->gCount[g] = static_cast<uint16_t>(cnt + 1);
    stableAdd(g, st);
    waveSync();
    return true;
  }

  // Remove slots [at, at + n) of group g (their blocks are being freed or moved); returns the
  // stable length they held.
  FMT_DEV void slotRemove(uint32_t g, int at, int n) {
    ProfScope ps_(prof[10]);
    invalidate();
    const int cnt = static_cast<int>(L->gCount[g]);
    uint32_t* sb = slotBlkPtr(g);
    int32_t* ss = slotStPtr(g);
    Lane<uint32_t> rv;  // (n <= 64)
    FOR_LANES(l) { LANE(rv) = l < n ? static_cast<uint32_t>(rd(ss + at + l)) : 0u; }
    uint32_t removedU;
    waveExclusiveSum(rv, &removedU);
    const int removed = static_cast<int>(removedU);
    for (int base = at + n; base < cnt; base += 64 * kShiftU) {  // shift down by n, bottom-up
      Lane<uint32_t> b[kShiftU];
      Lane<int32_t> st[kShiftU];
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < kShiftU; u++) {
          const int i = base + 64 * u + l;
          if (i < cnt) {
            LANE(b[u]) = rd(sb + i);
            LANE(st[u]) = rd(ss + i);
          }
        }
      }
      waveSync();
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < kShiftU; u++) {
          const int i = base + 64 * u + l;
          if (i < cnt) {
            sb[i - n] = LANE(b[u]);
            ss[i - n] = LANE(st[u]);
            S.bSlot[LANE(b[u])] = static_cast<uint32_t>(i - n);
          }
        }
      }
      waveSync();
    }
    L->gCount[g] = static_cast<uint16_t>(cnt - n);
    stableAdd(g, -removed);
    waveSync();
  }

  // A full group splits in two halves; the new group follows it in gOrder. Window entries of
  // blocks that moved are re-tagged.
  FMT_DEV bool groupSplit(uint32_t g) {
    if (nGroups >= kGroupCap) return fail(FMT_E_CAPACITY);
    const uint32_t g2 = static_cast<uint32_t>(nGroups);  // group ids are never freed
    const int cnt = static_cast<int>(L->gCount[g]), half = cnt / 2, moved = cnt - half;
    uint32_t* sb = slotBlkPtr(g);
    int32_t* ss = slotStPtr(g);
    uint32_t* db = slotBlkPtr(g2);
    int32_t* ds = slotStPtr(g2);
    Lane<int32_t> acc;
    FOR_LANES(l) { LANE(acc) = 0; }
    for (int base = 0; base < moved; base += 64) {
      FOR_LANES(l) {
        const int i = base + l;
        if (i < moved) {
          const uint32_t b = rd(sb + half + i);
          const int32_t s = rd(ss + half + i);
          db[i] = b;
          ds[i] = s;
          S.bGroup[b] = g2;
          S.bSlot[b] = static_cast<uint32_t>(i);
          LANE(acc) += s;
        }
      }
    }
    uint32_t tot;
    Lane<uint32_t> au;
    FOR_LANES(l) { LANE(au) = static_cast<uint32_t>(LANE(acc)); }
    waveExclusiveSum(au, &tot);
    const int gp = groupPos(g);
    for (int k = nGroups; k > gp + 1; k--) {
      const uint16_t v = L->gOrder[k - 1];
      waveSync();
      L->gOrder[k] = v;
    }
    L->gOrder[gp + 1] = static_cast<uint16_t>(g2);
    L->gCount[g] = static_cast<uint16_t>(half);
    L->gCount[g2] = static_cast<uint16_t>(moved);
    L->gStable[g] -= static_cast<int32_t>(tot);
    L->gStable[g2] = static_cast<int32_t>(tot);
    L->gCorr[g2] = 0;
    waveSync();
    nGroups++;
    chunksRebuild();
    // window entries follow their blocks
    for (uint32_t base = 0; base < nWin; base += 64) {
      FOR_LANES(l) {
        const uint32_t w = base + l;
        if (w < nWin) {
          const uint32_t m = rd(wWord3(w));
          if ((m >> kWGroupShift) == g) {
            const uint32_t v = (m & kWMetaMask) | (rd(S.bGroup + (rd(S.wBlk + w))) << kWGroupShift);
            *wWord3(w) = v;
            if (w < kWinLds) L->wRecL[4 * w + 3] = v;
          }
        }
      }
    }
    invalidate();
    return true;
  }

  // ------------------------------------------------------------------ perspective corrections
  // View length of window entry w (fields already loaded) for PriorPerspective(r, c).
  FMT_DEV static int winVis(int32_t ins, int32_t rm, uint32_t len, uint32_t m, uint32_t mlo, uint32_t mhi, int r, int c) {
    return visOf(len, ins, rm, mlo, mhi, mClient(m), r, c);
  }

  // ---- passes shared by the workgroup's waves. Wave 0 replays; when it needs a pass it posts the
  // command in LDS and the kWaves waves (one per SIMD) each take every kWaves-th step of it, between
  // workgroup barriers. (Host emulation: wave 0 runs every share itself.)
  static constexpr int kWaves = 4;
  enum : int { kCmdExit = 0, kCmdGroups = 1, kCmdSlots = 2 };
  struct PassCmd {
    int op, r, c;
    uint32_t g, nWin;
  };
  FMT_DEV void runPass(int op, int r, int c, uint32_t g) {
    const PassCmd cmd{op, r, c, g, nWin};
    FOR_LANES(l) {
      if (l == 0) {
        L->cmd[0] = op;
        L->cmd[1] = r;
        L->cmd[2] = c;
        L->cmd[3] = static_cast<int32_t>(g);
        L->cmd[4] = static_cast<int32_t>(nWin);
      }
    }
    waveSync();
#if FMT_GPU
    groupBarrier();
    if (op == kCmdSlots) {
      slotShare(cmd, 0);
      groupBarrier();
    }
    {
      ProfScope psW_(prof[20]);
      windowShare(cmd, 0);
    }
    groupBarrier();
#else
    if (op == kCmdSlots)
      for (int w = 0; w < kWaves; w++) slotShare(cmd, w);
    for (int w = 0; w < kWaves; w++) windowShare(cmd, w);
#endif
  }
  // Helper waves 1..kWaves-1: serve pass commands until wave 0 posts kCmdExit.
  FMT_DEV void helperLoop(int wave) {
    for (;;) {
      groupBarrier();
      const PassCmd cmd{uni(L->cmd[0]), uni(L->cmd[1]), uni(L->cmd[2]), static_cast<uint32_t>(uni(L->cmd[3])),
                        static_cast<uint32_t>(uni(L->cmd[4]))};
      if (cmd.op == kCmdExit) return;
      if (cmd.op == kCmdSlots) {
        slotShare(cmd, wave);
        groupBarrier();
      }
      windowShare(cmd, wave);
      groupBarrier();
    }
  }
  FMT_DEV void postExit() {  // wave 0, after the replay: releases the helper waves
    FOR_LANES(l) {
      if (l == 0) L->cmd[0] = kCmdExit;
    }
    waveSync();
#if FMT_GPU
    groupBarrier();
#endif
  }

  // Slots of group cmd.g into sLen / sBlk (their stable lengths), this wave's steps.
  FMT_DEV void slotShare(const PassCmd& cmd, int wave) {
    const uint32_t g = cmd.g;
    const int cnt = static_cast<int>(L->gCount[g]);
    const uint32_t* sb = slotBlkPtr(g);
    const int32_t* ss = slotStPtr(g);
    // 64-slot pieces dealt round-robin to the waves: piece (u * kWaves + wave) of each step
    for (int base = 0; base < cnt; base += kWaves * 64 * kShiftU) {
      Lane<uint32_t> bb[kShiftU];
      Lane<int32_t> sv[kShiftU];
#pragma unroll
      for (int u = 0; u < kShiftU; u++) {
        const int p0 = base + (u * kWaves + wave) * 64;
        if (p0 < cnt) {
          FOR_LANES(l) {
            const int i = p0 + l;
            if (i < cnt) {
              LANE(bb[u]) = rd(sb + i);
              LANE(sv[u]) = rd(ss + i);
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kShiftU; u++) {
        const int p0 = base + (u * kWaves + wave) * 64;
        if (p0 < cnt) {
          FOR_LANES(l) {
            const int i = p0 + l;
            if (i < cnt) {
              L->sBlk[i] = LANE(bb[u]);
              L->sLen[i] = LANE(sv[u]);
            }
          }
        }
      }
    }
    waveSync();
  }

  // This wave's steps of one pass over the window table (entries below kWinLds from the LDS mirror,
  // the rest from HBM, kPassU x 64 per step with every load of a step in flight together): each entry
  // of positive view length is added to gCorr[group] and its chunk's cCorr (kCmdGroups), or, if it
  // belongs to group cmd.g, to sLen[slot of its block] (kCmdSlots: few entries per group, so their
  // block / slot lookups are per lane).
  static constexpr int kPassU = 2;
  FMT_DEV void windowShare(const PassCmd& cmd, int wave) {
    const int r = cmd.r, c = cmd.c;
    const uint32_t n = cmd.nWin;
    const bool bySlot = cmd.op == kCmdSlots;
    const uint32_t only = bySlot ? cmd.g : kNone;
    for (uint32_t base = 0; base < n; base += kWaves * 64 * kPassU) {
      Lane<u32x4> rec[kPassU];
      Lane<u32x2> msk[kPassU];
      int nu = 0;  // this wave's pieces in this step
#pragma unroll
      for (int u = 0; u < kPassU; u++) {
        const uint32_t p0 = base + static_cast<uint32_t>(u * kWaves + wave) * 64;
        if (p0 < n) {
          nu = u + 1;
          FOR_LANES(l) {
            const uint32_t w = p0 + l;
            if (w < n) {
              LANE(rec[u]) = wRecOf(w);
              LANE(msk[u]) = wMaskOf(w);
            }
          }
        }
      }
      FOR_LANES(l) {
#pragma unroll
        for (int u = 0; u < kPassU; u++) {
          const uint32_t w = base + static_cast<uint32_t>(u * kWaves + wave) * 64 + l;
          if (u < nu && w < n) {
            const u32x4 x = LANE(rec[u]);
            const uint32_t grp = x[3] >> kWGroupShift;
            if (only == kNone || grp == only) {
              const u32x2 mk = LANE(msk[u]);
              const uint32_t v =
                  c < 64 ? static_cast<uint32_t>(winVis(static_cast<int32_t>(x[0]), static_cast<int32_t>(x[1]), x[2], x[3] & kWMetaMask, mk[0], mk[1], r, c))
                         : static_cast<uint32_t>(visAny(x[2], static_cast<int32_t>(x[0]), static_cast<int32_t>(x[1]), 0u, 0u,
                                                        mClient(x[3]), r, c, rd(S.wLeaf + w)));
              if (v && !bySlot) {
                atomicAddLds(&L->gCorr[grp], static_cast<int>(v));
                atomicAddLds(&L->cCorr[L->gPos[grp] >> 5], static_cast<int>(v));
              }
              if (v && bySlot) atomicAddLds(&L->sLen[rd(S.bSlot + rd(S.wBlk + w))], static_cast<int>(v));
            }
          }
        }
      }
    }
    waveSync();
  }
  // gCorr[g] = Σ view length of the window leaves of group g (their stable contribution is 0)
  FMT_DEV void groupCorrections(int r, int c) {
    ProfScope ps_(prof[1]);
    FOR_LANES(l) {
      for (int g = l; g < nGroups; g += 64) L->gCorr[g] = 0;
      if (l < kGroupCap / 32) L->cCorr[l] = 0;
    }
    waveSync();
    prof[16]++;
    prof[18] += nWin;
    prof[19] += static_cast<uint64_t>(nGroups);
    runPass(kCmdGroups, r, c, kNone);
    corrValid = true;
  }

  // View length of the groups at positions [k0, k0 + 64) (lane l: position k0 + l; 0 past the end).
  FMT_DEV Lane<uint32_t> groupLens(int k0) const {
    Lane<uint32_t> len;
    FOR_LANES(l) {
      const int k = k0 + l;
      uint32_t x = 0;
      if (k < nGroups) {
        const uint32_t g = L->gOrder[k];
        x = static_cast<uint32_t>(L->gStable[g] + L->gCorr[g]);
      }
      LANE(len) = x;
    }
    return len;
  }

  FMT_DEV int totalView() const {
    uint32_t total = 0;
    for (int k0 = 0; k0 < nGroups; k0 += 64) {
      uint32_t tot;
      waveExclusiveSum(groupLens(k0), &tot);
      total += tot;
    }
    return static_cast<int>(total);
  }

  // Slot view lengths of group g into L->sLen / L->sBlk (stable + that group's window corrections).
  FMT_DEV void slotLengths(uint32_t g, int r, int c) {
    slotCacheG = g;
    slotCacheEpoch = epoch;
    ProfScope ps_(prof[2]);
    prof[17]++;
    runPass(kCmdSlots, r, c, g);
  }

  // ------------------------------------------------------------------ the hierarchical search
  // The first leaf (document order) with st <= p < st + vis, or st == p, vis == 0 and not skipped
  // (removed at/below minSeq, unless it is the document's very last leaf).
  FMT_DEV Hit find(int p, int r, int c) {
    ProfScope ps_(prof[7]);
    Hit h;
    h.found = false;
    if (!corrValid) groupCorrections(r, c);
    // first group whose end reaches p: running view start over 64-group chunks (one wave scan each,
    // stopping at the chunk that holds it)
    int k = -1, base = 0;
    {
      // two levels: lane l takes chunk l (group positions [32 l, 32 l + 32): its stable sum and its
      // window correction, kept as the groups' change), one wave scan finds the first chunk whose end
      // reaches p, a second scans that chunk's groups
      ProfScope psScan_(prof[21]);
      const int nc = (nGroups + 31) / 32;
      Lane<uint32_t> run;
      FOR_LANES(l) { LANE(run) = l < nc ? static_cast<uint32_t>(L->cStable[l] + L->cCorr[l]) : 0u; }
      uint32_t tot;
      const Lane<uint32_t> ex = waveExclusiveSum(run, &tot);
      Lane<bool> q;
      FOR_LANES(l) { LANE(q) = l < nc && static_cast<int>(LANE(ex) + LANE(run)) >= p; }
      const uint64_t m = ballot(q);
      if (m) {
        const int lr = ctz64(m);
        base = static_cast<int>(readlane(ex, lr));
        const int k0 = lr * 32;
        Lane<uint32_t> len;
        FOR_LANES(l) {
          const int kk = k0 + l;
          uint32_t x = 0;
          if (l < 32 && kk < nGroups) {
            const uint32_t g = L->gOrder[kk];
            x = static_cast<uint32_t>(L->gStable[g] + L->gCorr[g]);
          }
          LANE(len) = x;
        }
        uint32_t t2;
        const Lane<uint32_t> ex2 = waveExclusiveSum(len, &t2);
        Lane<bool> q2;
        FOR_LANES(l) { LANE(q2) = l < 32 && k0 + l < nGroups && base + static_cast<int>(LANE(ex2) + LANE(len)) >= p; }
        const uint64_t m2 = ballot(q2);
        if (m2) {  // (always: the chunk's end reaches p)
          k = k0 + ctz64(m2);
          base += static_cast<int>(readlane(ex2, ctz64(m2)));
        }
      }
    }
    if (k < 0) return h;
    for (; k < nGroups; k++) {  // (base: the view start of group position k)
      const uint32_t g = L->gOrder[k];
      if (slotCacheG != g || slotCacheEpoch != epoch) slotLengths(g, r, c);
      const int cnt = static_cast<int>(L->gCount[g]);
      for (int s0 = 0; s0 < cnt; s0 += 64) {
        Lane<uint32_t> len;
        FOR_LANES(l) { LANE(len) = s0 + l < cnt ? static_cast<uint32_t>(L->sLen[s0 + l]) : 0u; }
        uint32_t tot;
        const Lane<uint32_t> ex = waveExclusiveSum(len, &tot);
        // candidate slots: end >= p, in order
        Lane<bool> q;
        FOR_LANES(l) { LANE(q) = s0 + l < cnt && base + static_cast<int>(LANE(ex) + LANE(len)) >= p; }
        uint64_t m = ballot(q);
        while (m) {
          const int lane = ctz64(m);
          m &= m - 1;
          const int s = s0 + lane;
          const int bst = base + static_cast<int>(readlane(ex, lane));
          if (bst > p) return h;  // passed p: nothing qualifies (cannot happen for valid ops)
          if (leafInBlock(L->sBlk[s], bst, p, r, c, h)) {
            h.gpos = k;
            h.slot = s;
            return h;
          }
        }
        base += static_cast<int>(tot);
      }
    }
    return h;
  }

  // Search one leaf block whose view start is bst.
  FMT_DEV bool leafInBlock(uint32_t b, int bst, int p, int r, int c, Hit& h) {
    // the block's 8 leaf slots are loaded beside its count (one memory round trip, not two: slots past
    // the count hold stale fields and are masked after)
    Lane<uint32_t> fl, fi, fr, flo, fhi, fm, fid;
    FOR_LANES(l) {
      const size_t i = static_cast<size_t>(b) * 8 + (l & 7);
      LANE(fl) = rd(S.lLen + i);
      LANE(fi) = static_cast<uint32_t>(rd(S.lIns + i));
      LANE(fr) = static_cast<uint32_t>(rd(S.lRm + i));
      LANE(flo) = rd(S.lMlo + i);
      LANE(fhi) = rd(S.lMhi + i);
      LANE(fm) = rd(S.lMeta + i);
      LANE(fid) = c < 64 ? 0u : rd(S.lId + i);
    }
    const uint32_t cnt = ldu(S.bCount + b);
    Lane<uint32_t> vis;
    Lane<bool> skipped;
    FOR_LANES(l) {
      uint32_t v = 0;
      bool sk = false;
      if (l < static_cast<int>(cnt)) {
        const int32_t rm = static_cast<int32_t>(LANE(fr));
        v = static_cast<uint32_t>(visAny(LANE(fl), static_cast<int32_t>(LANE(fi)), rm, LANE(flo), LANE(fhi), mClient(LANE(fm)), r, c,
                                         LANE(fid)));
        sk = rm <= minSeq && !(b == lastBlk && l == static_cast<int>(cnt) - 1);
      }
      LANE(vis) = v;
      LANE(skipped) = sk;
    }
    uint32_t tot;
    const Lane<uint32_t> ex = waveExclusiveSum(vis, &tot);
    Lane<bool> q;
    FOR_LANES(l) {
      const int st = bst + static_cast<int>(LANE(ex));
      const int v = static_cast<int>(LANE(vis));
      LANE(q) = l < static_cast<int>(cnt) && ((st <= p && p < st + v) || (st == p && v == 0 && !LANE(skipped)));
    }
    const uint64_t m = ballot(q);
    if (!m) return false;
    const int k = ctz64(m);
    h.found = true;
    h.blk = b;
    h.k = k;
    h.st = bst + static_cast<int>(readlane(ex, k));
    h.vis = static_cast<int>(readlane(vis, k));
    return true;
  }

  // ------------------------------------------------------------------ leaves inside a block
  FMT_DEV size_t li(uint32_t b, int k) const { return static_cast<size_t>(b) * 8 + k; }

  struct Leaf {
    uint32_t len;
    int32_t ins, rm;
    uint32_t mlo, mhi, id, text, meta;
  };
  FMT_DEV Leaf getLeaf(uint32_t b, int k) const {
    const size_t i = li(b, k);
    Leaf x;
    x.len = ldu(S.lLen + i);
    x.ins = ldi(S.lIns + i);
    x.rm = ldi(S.lRm + i);
    x.mlo = ldu(S.lMlo + i);
    x.mhi = ldu(S.lMhi + i);
    x.id = ldu(S.lId + i);
    x.text = ldu(S.lText + i);
    x.meta = ldu(S.lMeta + i);
    return x;
  }
  FMT_DEV void putLeaf(uint32_t b, int k, const Leaf& x) {
    const size_t i = li(b, k);
    FOR_LANES(l) {
      if (l == 0) {
        S.lLen[i] = x.len;
        S.lIns[i] = x.ins;
        S.lRm[i] = x.rm;
        S.lMlo[i] = x.mlo;
        S.lMhi[i] = x.mhi;
        S.lId[i] = x.id;
        S.lText[i] = x.text;
        S.lMeta[i] = x.meta;
        S.leafBlk[x.id] = b;
      }
    }
  }
  // ------------------------------------------------------------------ B+tree
  FMT_DEV uint32_t childAt(uint32_t p, int i) const { return ldu(S.bChild + static_cast<size_t>(p) * 8 + i); }
  FMT_DEV void setChild(uint32_t p, int i, uint32_t c) {
    st1(S.bChild + static_cast<size_t>(p) * 8 + i, c);
    st1(S.bParent + c, p);
  }

  // A leaf block held in registers (lane l = leaf l: fields f, window entry wi), with its count,
  // group, slot and parent; edits are made in registers and written back by commitBlock.
  struct BlockRegs {
    Lane<uint32_t> f[8], wi;
    int cnt;
    uint32_t b, g, s, parent;
  };
  FMT_DEV void loadBlock(uint32_t b, BlockRegs& R) const {
    R.b = b;
    R.cnt = static_cast<int>(ldu(S.bCount + b));
    R.g = ldu(S.bGroup + b);
    R.s = ldu(S.bSlot + b);
    R.parent = ldu(S.bParent + b);
    FOR_LANES(l) {
      const size_t i = li(b, l & 7);
      LANE(R.f[0]) = rd(S.lLen + i);
      LANE(R.f[1]) = static_cast<uint32_t>(rd(S.lIns + i));
      LANE(R.f[2]) = static_cast<uint32_t>(rd(S.lRm + i));
      LANE(R.f[3]) = rd(S.lMlo + i);
      LANE(R.f[4]) = rd(S.lMhi + i);
      LANE(R.f[5]) = rd(S.lId + i);
      LANE(R.f[6]) = rd(S.lText + i);
      LANE(R.f[7]) = rd(S.lMeta + i);
    }
    FOR_LANES(l) { LANE(R.wi) = l < R.cnt ? rd(S.winIdx + LANE(R.f[5])) : kNone; }
  }
  FMT_DEV static Leaf regLeaf(const BlockRegs& R, int k) {
    Leaf x;
    x.len = readlane(R.f[0], k);
    x.ins = static_cast<int32_t>(readlane(R.f[1], k));
    x.rm = static_cast<int32_t>(readlane(R.f[2], k));
    x.mlo = readlane(R.f[3], k);
    x.mhi = readlane(R.f[4], k);
    x.id = readlane(R.f[5], k);
    x.text = readlane(R.f[6], k);
    x.meta = readlane(R.f[7], k);
    return x;
  }
  // Insert leaf x (window entry w) at position k: leaves k.. move up one lane.
  FMT_DEV static void regsInsert(BlockRegs& R, int k, const Leaf& x, uint32_t w) {
    Lane<int> src;
    FOR_LANES(l) { LANE(src) = l > k ? l - 1 : l; }
#pragma unroll
    for (int i = 0; i < 8; i++) R.f[i] = gather(R.f[i], src);
    R.wi = gather(R.wi, src);
    FOR_LANES(l) {
      if (l == k) {
        LANE(R.f[0]) = x.len;
        LANE(R.f[1]) = static_cast<uint32_t>(x.ins);
        LANE(R.f[2]) = static_cast<uint32_t>(x.rm);
        LANE(R.f[3]) = x.mlo;
        LANE(R.f[4]) = x.mhi;
        LANE(R.f[5]) = x.id;
        LANE(R.f[6]) = x.text;
        LANE(R.f[7]) = x.meta;
        LANE(R.wi) = w;
      }
    }
    R.cnt++;
  }
  FMT_DEV void storeLeafLane(uint32_t b, int k, const BlockRegs& R, int l) {
    const size_t i = li(b, k);
    S.lLen[i] = LANE(R.f[0]);
    S.lIns[i] = static_cast<int32_t>(LANE(R.f[1]));
    S.lRm[i] = static_cast<int32_t>(LANE(R.f[2]));
    S.lMlo[i] = LANE(R.f[3]);
    S.lMhi[i] = LANE(R.f[4]);
    S.lId[i] = LANE(R.f[5]);
    S.lText[i] = LANE(R.f[6]);
    S.lMeta[i] = LANE(R.f[7]);
  }

  // Write the block back. A block that reached MaxNodesInBlock leaves splits (mergeTree.ts:1946-1987):
  // leaves 4..7 go to a new leaf block listed in the next slot, both stable sums are recomputed from
  // the registers, and the new block is inserted after b in the parent chain. Returns the new block
  // (kNone when there was no split).
  FMT_DEV uint32_t commitBlock(BlockRegs& R) {
    constexpr int half = kMaxNodes / 2;
    const uint32_t b = R.b;
    if (R.cnt < kMaxNodes) {
      FOR_LANES(l) {
        if (l < R.cnt) storeLeafLane(b, l, R, l);
      }
      waveSync();
      st1(S.bCount + b, static_cast<uint32_t>(R.cnt));
      return kNone;
    }
    const uint32_t nb = allocBlk(1);
    if (nb == kNone) return kNone;
    st1(S.bGroup + nb, R.g);  // (tentative: a group split in slotInsert may move it)
    Lane<uint32_t> stv;
    FOR_LANES(l) {
      const bool stable = l < kMaxNodes && LANE(R.wi) == kNone && static_cast<int32_t>(LANE(R.f[2])) == kNotRemoved;
      LANE(stv) = stable ? LANE(R.f[0]) : 0u;
      if (l < half) storeLeafLane(b, l, R, l);
      else if (l < kMaxNodes) {
        storeLeafLane(nb, l - half, R, l);
        S.leafBlk[LANE(R.f[5])] = nb;
      }
    }
    uint32_t stTot;
    const Lane<uint32_t> stEx = waveExclusiveSum(stv, &stTot);
    const int stB = static_cast<int>(readlane(stEx, half)), stN = static_cast<int>(stTot) - stB;
    waveSync();
    st1(S.bCount + b, static_cast<uint32_t>(half));
    st1(S.bCount + nb, static_cast<uint32_t>(half));
    int32_t* sp = slotStPtr(R.g) + R.s;
    const int32_t oldSt = ldi(sp);
    st1(sp, stB);
    stableAdd(R.g, stB - oldSt);
    waveSync();
    invalidate();
    if (!slotInsert(R.g, static_cast<int>(R.s) + 1, nb, stN)) return kNone;
    const uint32_t g2 = ldu(S.bGroup + nb);
    FOR_LANES(l) {
      if (l >= half && l < kMaxNodes && LANE(R.wi) != kNone) wRetag(LANE(R.wi), nb, g2);
    }
    waveSync();
    if (lastBlk == b) lastBlk = nb;
    addChildAfter(R.parent, b, nb);
    return nb;
  }

  // Insert block nb after its sibling b into parent p, splitting full interior blocks upward and
  // growing the root (mergeTree.ts:1313-1320, 1946-1987).
  FMT_DEV void addChildAfter(uint32_t p, uint32_t b, uint32_t nb) {
    constexpr int half = kMaxNodes / 2;
    for (;;) {
      if (p == kNone) {
        const uint32_t r = allocBlk(0);
        if (r == kNone) return;
        st1(S.bCount + r, 2u);
        setChild(r, 0, b);
        setChild(r, 1, nb);
        root = static_cast<int>(r);
        return;
      }
      const int pc = static_cast<int>(ldu(S.bCount + p));
      Lane<uint32_t> ch;
      Lane<bool> isB;
      FOR_LANES(l) {
        LANE(ch) = rd(S.bChild + (static_cast<size_t>(p) * 8 + (l & 7)));
        LANE(isB) = l < pc && LANE(ch) == b;
      }
      const int idx = ctz64(ballot(isB));
      Lane<int> src;
      FOR_LANES(l) { LANE(src) = l <= idx ? l : l - 1; }
      Lane<uint32_t> ch2 = gather(ch, src);
      FOR_LANES(l) {
        if (l == idx + 1) LANE(ch2) = nb;
      }
      const int cnt = pc + 1;
      if (cnt < kMaxNodes) {
        FOR_LANES(l) {
          if (l > idx && l < cnt) S.bChild[static_cast<size_t>(p) * 8 + l] = LANE(ch2);
          if (l == 0) {
            S.bParent[nb] = p;
            S.bCount[p] = static_cast<uint32_t>(cnt);
          }
        }
        waveSync();
        return;
      }
      const uint32_t np = allocBlk(0);
      if (np == kNone) return;
      FOR_LANES(l) {
        if (l > idx && l < half) S.bChild[static_cast<size_t>(p) * 8 + l] = LANE(ch2);
        if (l >= half && l < kMaxNodes) {
          S.bChild[static_cast<size_t>(np) * 8 + (l - half)] = LANE(ch2);
          S.bParent[LANE(ch2)] = np;
        }
        if (l == 0) {
          if (idx + 1 < half) S.bParent[nb] = p;
          S.bCount[p] = static_cast<uint32_t>(half);
          S.bCount[np] = static_cast<uint32_t>(half);
        }
      }
      waveSync();
      const uint32_t pp = ldu(S.bParent + p);
      b = p;
      nb = np;
      p = pp;
    }
  }

  // ------------------------------------------------------------------ LRU heap (heap.ts)
  FMT_DEV int heapSeq(int k) const { return uni(L->heap[k].maxSeq); }
  // heap.ts sift order, moving a hole instead of swapping (the same final arrangement)
  FMT_DEV void heapAdd(int maxSeq, uint32_t leafId) {
    ProfScope ps_(prof[11]);
    if (heapN >= kHeapCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    int k = ++heapN;
    while (k > 1) {
      const HeapEnt up = L->heap[k >> 1];
      if (!(uni(up.maxSeq) - maxSeq > 0)) break;
      waveSync();
      L->heap[k] = up;
      k >>= 1;
    }
    waveSync();
    L->heap[k].maxSeq = maxSeq;
    L->heap[k].leafId = leafId;
    waveSync();
  }
  FMT_DEV HeapEnt heapGet() {
    ProfScope ps_(prof[11]);
    HeapEnt top;
    top.maxSeq = uni(L->heap[1].maxSeq);
    top.leafId = uni(L->heap[1].leafId);
    const HeapEnt x = L->heap[heapN];  // the last entry sifts down from the root
    const int xs = uni(x.maxSeq);
    waveSync();
    heapN--;
    int k = 1;
    while ((k << 1) <= heapN) {
      int j = k << 1;
      // both children in one LDS round trip (entry heapN + 1 is inside the array and never chosen)
      const HeapEnt a = L->heap[j], b = L->heap[j + 1];
      HeapEnt c = a;
      if (j < heapN && uni(a.maxSeq) - uni(b.maxSeq) > 0) {
        j++;
        c = b;
      }
      if (xs - uni(c.maxSeq) <= 0) break;
      waveSync();
      L->heap[k] = c;
      k = j;
    }
    waveSync();
    if (heapN >= 1) L->heap[k] = x;
    waveSync();
    return top;
  }

  // addToLRUSet (mergeTree.ts:812-822): the first registration of a block sets needsScour.
  FMT_DEV void lru(uint32_t b, uint32_t leafId, int seq) {
    if (ldi(S.bScour + b) != 1 && seq > curSeq) {
      st1(S.bScour + b, 1);
      heapAdd(seq, leafId);
    }
  }

  // ------------------------------------------------------------------ props
  // matchProperties (properties.ts:32-61, undefined ≡ {}) as equality of match classes: interned
  // sets with the same (key, value) content in any key order share the class of the first of them.
  FMT_DEV uint32_t propClass(uint32_t a) const {
    return a == kNoProps ? 0xFFFFu : a < static_cast<uint32_t>(kPropLds) ? L->pClass[a] : rd(S.pClass + a);
  }
  FMT_DEV bool propsMatch(uint32_t a, uint32_t b) const { return a == b || uni(propClass(a)) == uni(propClass(b)); }
  // `seg.properties ??= {}` then raw LWW per key, null deletes (segmentPropertiesManager.ts:188-238).
  // The working set lives in LDS (kvWork, slot k = lane k % 64 of chunk k / 64; slots past the set's
  // count are never read); a set wider than FMT_MT_PROPS_MAX entries takes consecutive records (fmt.h
  // fmt_mt_propset).
  FMT_DEV uint32_t setKv(uint32_t p, uint32_t k) const {
    return rd(S.props + ((static_cast<size_t>(p) + k / FMT_MT_PROPS_MAX) * kPropWords + 1 + k % FMT_MT_PROPS_MAX));
  }
  FMT_DEV uint32_t loadWork(uint32_t old) {
    const uint32_t cnt = old != kNoProps ? ldu(S.props + old * kPropWords) : 0u;
    for (int c = 0; c < kKeyChunks && c * 64 < static_cast<int>(cnt); c++) {
      FOR_LANES(l) {
        const int k = c * 64 + l;
        if (k < static_cast<int>(cnt)) L->kvWork[k] = setKv(old, static_cast<uint32_t>(k));
      }
    }
    waveSync();
    return cnt;
  }
  // adjSite: the annotate call site, the only one whose props ops may hold annotate-adjust entries
  // ((key, FMT_MT_VALUE_ADJUST) then the adjust row; computePropertyValue folds into the current value)
  FMT_DEV uint32_t applyProps(uint32_t old, uint32_t opId, bool adjSite = false) {
    constexpr int kKeysMax = FMT_MT_PROPS_KEYS_MAX;
    uint32_t cnt = loadWork(old);
    const uint32_t a = ldu(in.propsOff + opId), b = ldu(in.propsOff + opId + 1);
    for (uint32_t t = a; t < b; t++) {
      uint32_t e = ldu(in.propsKv + t);
      uint32_t pos = cnt;
      for (int c = 0; c < kKeyChunks && pos == cnt && c * 64 < static_cast<int>(cnt); c++) {
        Lane<bool> hit;
        FOR_LANES(l) {
          const int k = c * 64 + l;
          LANE(hit) = k < static_cast<int>(cnt) && (L->kvWork[k] >> 16) == (e >> 16);
        }
        const uint64_t m = ballot(hit);
        if (m) pos = static_cast<uint32_t>(c * 64 + ctz64(m));
      }
      if ((e & 0xFFFFu) == FMT_MT_VALUE_ADJUST) {
        if constexpr (Adj) {
          if (!adjSite || in.adj == nullptr || ++t >= b) {
            fail(FMT_E_DATA);
            return kNoProps;
          }
          const uint32_t cur = pos < cnt ? uni(L->kvWork[pos]) & 0xFFFFu : 0u;  // absent: null
          const uint32_t v = fmt_mt::adjustFold(in.adj, in.doc, cur, ldu(in.propsKv + t));
          if (v == fmt_mt::kAdjFailData || v == fmt_mt::kAdjFailCap) {
            fail(v == fmt_mt::kAdjFailData ? FMT_E_DATA : FMT_E_CAPACITY);
            return kNoProps;
          }
          e = (e & 0xFFFF0000u) | v;
        } else {
          fail(FMT_E_DATA);  // (the runtime launches the Adj variant for batches with adjusts)
          return kNoProps;
        }
      }
      if ((e & 0xFFFFu) == 0) {  // null: delete the key
        if (pos < cnt) {  // entries pos+1 .. cnt-1 move down one slot, a chunk at a time in slot order
          for (int c = static_cast<int>(pos) / 64; c < kKeyChunks && c * 64 < static_cast<int>(cnt); c++) {
            Lane<uint32_t> v;
            FOR_LANES(l) {
              const int k = c * 64 + l;
              LANE(v) = (k < kKeysMax - 1 && k >= static_cast<int>(pos)) ? L->kvWork[k + 1] : 0u;
            }
            waveSync();
            FOR_LANES(l) {
              const int k = c * 64 + l;
              if (k >= static_cast<int>(pos) && k + 1 < static_cast<int>(cnt)) L->kvWork[k] = LANE(v);
            }
            waveSync();
          }
          cnt--;
        }
      } else if (pos < cnt) {
        FOR_LANES(l) {
          if (l == static_cast<int>(pos % 64)) L->kvWork[pos] = e;
        }
      } else {
        if (cnt >= static_cast<uint32_t>(kKeysMax)) {
          fail(FMT_E_CAPACITY);
          return kNoProps;
        }
        FOR_LANES(l) {
          if (l == static_cast<int>(cnt % 64)) L->kvWork[cnt] = e;
        }
        cnt++;
      }
      waveSync();
    }
    return internWork(cnt);
  }
  // The interned id of the working set (kvWork[0 .. cnt)), a new set if none has its entries.
  FMT_DEV uint32_t internWork(uint32_t cnt) {
    // Interned already? Sets are found through two hash tables in HBM: one keyed by the ordered
    // entries (the same set), one by the entries in any order (its match class).
    uint32_t so = 0, su = 0;
    for (int c = 0; c < kKeyChunks && c * 64 < static_cast<int>(cnt); c++) {
      Lane<uint32_t> ho, hu;
      FOR_LANES(l) {
        const int k = c * 64 + l;
        const bool on = k < static_cast<int>(cnt);
        const uint32_t e = on ? L->kvWork[k] : 0u;
        LANE(ho) = on ? mix32(e ^ (0x9E3779B9u * static_cast<uint32_t>(k + 1))) : 0u;
        LANE(hu) = on ? mix32(e) : 0u;
      }
      uint32_t to, tu;
      waveExclusiveSum(ho, &to);
      waveExclusiveSum(hu, &tu);
      so += to;
      su += tu;
    }
    const uint32_t bo = mix32(so + cnt) & (kPropHash - 1);
    const uint32_t bu = kPropHash + (mix32(su ^ (cnt * 0x85EBCA6Bu)) & (kPropHash - 1));
    for (uint32_t p = ldu(S.pHead + bo); p != 0; p = ldu(S.pNext + 2 * (p - 1))) {
      const uint32_t q = p - 1;
      if (ldu(S.props + q * kPropWords) != cnt) continue;
      bool same = true;
      for (int c = 0; same && c * 64 < static_cast<int>(cnt); c++) {
        Lane<bool> diff;
        FOR_LANES(l) {
          const int k = c * 64 + l;
          LANE(diff) = k < static_cast<int>(cnt) && setKv(q, static_cast<uint32_t>(k)) != L->kvWork[k];
        }
        same = ballot(diff) == 0;
      }
      if (same) return q;
    }
    const int rec = cnt > FMT_MT_PROPS_MAX ? static_cast<int>((cnt + FMT_MT_PROPS_MAX - 1) / FMT_MT_PROPS_MAX) : 1;
    if (nProps + rec > kPropCap) {
      fail(FMT_E_CAPACITY);
      return kNoProps;
    }
    const uint32_t id = static_cast<uint32_t>(nProps);
    uint32_t cls = cnt == 0 ? 0xFFFFu : id;  // same content, other key order? (the class bucket lists
    for (uint32_t p = cnt > 0 ? ldu(S.pHead + bu) : 0u; p != 0 && cls == id; p = ldu(S.pNext + 2 * (p - 1) + 1)) {
      const uint32_t q = p - 1;                //  only the first set of each class)
      if (ldu(S.props + q * kPropWords) != cnt) continue;
      bool all = true;
      for (int c = 0; all && c * 64 < static_cast<int>(cnt); c++) {
        Lane<bool> miss;
        FOR_LANES(l) {
          const int k = c * 64 + l;
          bool found = k >= static_cast<int>(cnt);
          for (uint32_t j = 0; !found && j < cnt; j++) found = setKv(q, j) == L->kvWork[k];
          LANE(miss) = !found;
        }
        all = ballot(miss) == 0;
      }
      if (all) cls = q;
    }
    const uint32_t headO = ldu(S.pHead + bo), headU = ldu(S.pHead + bu);
    for (int ch = 0; ch * 64 < rec * FMT_MT_PROPS_MAX; ch++) {  // (slots past cnt: unused entries, 0)
      FOR_LANES(l) {
        const int j = ch * 64 + l, q = j / FMT_MT_PROPS_MAX, k = j % FMT_MT_PROPS_MAX;
        if (q < rec) {
          const size_t r = static_cast<size_t>(id + q) * kPropWords;
          if (k == 0) {
            const uint32_t c = q == 0 ? cls : 0xFFFEu;
            S.props[r] = q == 0 ? cnt : FMT_MT_PROPS_CONT;
            S.pClass[id + q] = c;
            if (id + q < static_cast<uint32_t>(kPropLds)) L->pClass[id + q] = static_cast<uint16_t>(c);
          }
          S.props[r + 1 + k] = j < static_cast<int>(cnt) ? L->kvWork[j] : 0u;
        }
      }
    }
    FOR_LANES(l) {
      if (l == 0) {
        S.pNext[2 * id] = headO;
        S.pHead[bo] = id + 1;
        if (cls == id) {
          S.pNext[2 * id + 1] = headU;
          S.pHead[bu] = id + 1;
        }
      }
    }
    waveSync();
    nProps += rec;
    return id;
  }

  // ------------------------------------------------------------------ PropertiesManager (annotate-adjust)
  // Per leaf, the remote changes a legacy summary's getAtSeq(properties, minSeq) needs
  // (segmentPropertiesManager.ts:140-345), as mt_engine.h keeps them: records of 4 words in the
  // document's HBM slab (AdjustTables::pm), in creation order — a head {leaf id, key, kind 0, value =
  // msnConsensus} per (leaf, key) with pending changes (the manager's Map order) and the changes
  // {leaf id, key | 1 << 16, seq, value after the change}. Leaf id 0 marks a deleted record.
  FMT_DEV uint32_t* pmBase() const { return in.adj->pm + 4 * in.adj->pmOffsets[in.doc]; }
  FMT_DEV int pmCap() const { return static_cast<int>(in.adj->pmOffsets[in.doc + 1] - in.adj->pmOffsets[in.doc]); }
  FMT_DEV uint32_t pmWord(int i, int w) const { return ldu(pmBase() + 4 * i + w); }
  FMT_DEV void pmSet(int i, int w, uint32_t v) { st1(pmBase() + 4 * i + w, v); }
  // First record at or after `from` whose (leaf id, key | kind) match under `mask`, or -1.
  FMT_DEV int pmFind(uint32_t leaf, uint32_t keyKind, uint32_t mask, int from = 0) const {
    const uint32_t* R = pmBase();
    for (int base = from; base < pmN; base += 64) {
      Lane<bool> p;
      FOR_LANES(l) {
        const int i = base + l;
        LANE(p) = i < pmN && rd(R + 4 * i) == leaf && (rd(R + 4 * i + 1) & mask) == (keyKind & mask);
      }
      const uint64_t m = ballot(p);
      if (m != 0) return base + ctz64(m);
    }
    return -1;
  }
  FMT_DEV void pmCompact() {  // drops deleted records, keeping the order
    uint32_t* R = pmBase();
    int out = 0;
    for (int base = 0; base < pmN; base += 64) {
      Lane<uint32_t> w0, w1, w2, w3;
      Lane<bool> live;
      FOR_LANES(l) {
        const int i = base + l;
        LANE(w0) = i < pmN ? rd(R + 4 * i) : 0u;
        LANE(w1) = i < pmN ? rd(R + 4 * i + 1) : 0u;
        LANE(w2) = i < pmN ? rd(R + 4 * i + 2) : 0u;
        LANE(w3) = i < pmN ? rd(R + 4 * i + 3) : 0u;
        LANE(live) = LANE(w0) != 0u;
      }
      const uint64_t m = ballot(live);
      waveSync();
      FOR_LANES(l) {
        if (LANE(live)) {
          const int at = out + __builtin_popcountll(m & ((1ull << l) - 1ull));
          R[4 * at] = LANE(w0);
          R[4 * at + 1] = LANE(w1);
          R[4 * at + 2] = LANE(w2);
          R[4 * at + 3] = LANE(w3);
        }
      }
      waveSync();
      out += __builtin_popcountll(m);
    }
    pmN = out;
  }
  FMT_DEV bool pmAppend(uint32_t leaf, uint32_t keyKind, int seq, uint32_t value) {
    if (pmN >= pmCap()) pmCompact();
    if (pmN >= pmCap()) return fail(FMT_E_CAPACITY);
    uint32_t* R = pmBase() + 4 * pmN;
    FOR_LANES(l) {
      if (l < 4) R[l] = l == 0 ? leaf : l == 1 ? keyKind : l == 2 ? static_cast<uint32_t>(seq) : value;
    }
    waveSync();
    pmN++;
    return true;
  }
  // updateMsn(msn) (:275-291) on the manager of `leaf`: changes at or below msn fold into
  // msnConsensus; a key left with none leaves the manager.
  FMT_DEV void pmUpdateMsn(uint32_t leaf, int msn) {
    for (int h = pmFind(leaf, 0u, 0x10000u); h >= 0 && status == FMT_OK; h = pmFind(leaf, 0u, 0x10000u, h + 1)) {
      const uint32_t key = pmWord(h, 1) & 0xFFFFu;
      uint32_t* R = pmBase();
      int last = -1;
      bool pending = false;
      for (int base = h + 1; base < pmN; base += 64) {  // (a head precedes its key's changes)
        Lane<bool> fold, keep;
        FOR_LANES(l) {
          const int i = base + l;
          const bool mine = i < pmN && rd(R + 4 * i) == leaf && rd(R + 4 * i + 1) == (key | 0x10000u);
          const int sq = mine ? static_cast<int>(rd(R + 4 * i + 2)) : 0;
          LANE(fold) = mine && sq <= msn;
          LANE(keep) = mine && sq > msn;
        }
        const uint64_t mf = ballot(fold), mk = ballot(keep);
        if (mf != 0) last = base + 63 - __builtin_clzll(mf);
        pending = pending || mk != 0;
        waveSync();
        FOR_LANES(l) {
          if (LANE(fold)) R[4 * (base + l)] = 0u;  // folded: deleted (its value word stays readable)
        }
        waveSync();
      }
      if (last >= 0) pmSet(h, 3, pmWord(last, 3));
      if (!pending) pmSet(h, 0, 0u);
    }
  }
  FMT_DEV void pmCopy(uint32_t from, uint32_t to) {
    if (pmFind(from, 0u, 0u) < 0) return;
    pmCompact();  // (no compaction while copying: record indices stay put)
    const int end = pmN;
    for (int i = pmFind(from, 0u, 0u); i >= 0 && i < end && status == FMT_OK; i = pmFind(from, 0u, 0u, i + 1)) {
      if (pmN >= pmCap()) {
        fail(FMT_E_CAPACITY);
        return;
      }
      pmAppend(to, pmWord(i, 1), static_cast<int>(pmWord(i, 2)), pmWord(i, 3));
    }
  }
  FMT_DEV void pmDropLeaf(uint32_t leaf) {
    uint32_t* R = pmBase();
    for (int base = 0; base < pmN; base += 64) {
      Lane<bool> mine;
      FOR_LANES(l) {
        const int i = base + l;
        LANE(mine) = i < pmN && rd(R + 4 * i) == leaf;
      }
      waveSync();
      FOR_LANES(l) {
        if (LANE(mine)) R[4 * (base + l)] = 0u;
      }
      waveSync();
    }
  }
  // Working-set edit: key set to v (v == 0: deleted), in kvWork[0 .. cnt).
  FMT_DEV uint32_t workSet(uint32_t cnt, uint32_t key, uint32_t v) {
    uint32_t pos = cnt;
    for (uint32_t k = 0; k < cnt; k++)
      if ((uni(L->kvWork[k]) >> 16) == key) pos = k;
    if (v == 0u) {
      if (pos < cnt) {
        for (uint32_t k = pos; k + 1 < cnt; k++) {
          const uint32_t x = uni(L->kvWork[k + 1]);
          waveSync();
          FOR_LANES(l) {
            if (l == 0) L->kvWork[k] = x;
          }
        }
        cnt--;
      }
    } else if (pos < cnt) {
      FOR_LANES(l) {
        if (l == 0) L->kvWork[pos] = (key << 16) | v;
      }
    } else if (cnt < static_cast<uint32_t>(FMT_MT_PROPS_KEYS_MAX)) {
      FOR_LANES(l) {
        if (l == 0) L->kvWork[cnt] = (key << 16) | v;
      }
      cnt++;
    }
    waveSync();
    return cnt;
  }
  // handleProperties (:188-238) of an annotate op on one leaf, before its prop set changes: every
  // change in opToChanges order (a raw change folds into msnConsensus while its key has nothing
  // pending), then updateMsn(minSeq).
  FMT_DEV void pmAnnotate(uint32_t leaf, uint32_t old, uint32_t opId, int seq) {
    uint32_t cnt = loadWork(old);
    const uint32_t a = ldu(in.propsOff + opId), b = ldu(in.propsOff + opId + 1);
    for (uint32_t t = a; t < b && status == FMT_OK; t++) {
      const uint32_t e = ldu(in.propsKv + t);
      const uint32_t key = e >> 16;
      const bool adjust = (e & 0xFFFFu) == FMT_MT_VALUE_ADJUST;
      uint32_t pos = cnt;
      for (uint32_t k = 0; k < cnt; k++)
        if ((uni(L->kvWork[k]) >> 16) == key) pos = k;
      const uint32_t before = pos < cnt ? uni(L->kvWork[pos]) & 0xFFFFu : 0u;
      uint32_t after = e & 0xFFFFu;
      if (adjust) {
        if (++t >= b) {
          fail(FMT_E_DATA);
          return;
        }
        after = fmt_mt::adjustFold(in.adj, in.doc, before, ldu(in.propsKv + t));
        if (after == fmt_mt::kAdjFailData || after == fmt_mt::kAdjFailCap) {
          fail(after == fmt_mt::kAdjFailData ? FMT_E_DATA : FMT_E_CAPACITY);
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
      cnt = workSet(cnt, key, after);  // the working set follows the change
    }
    pmUpdateMsn(leaf, minSeq);
  }

  // ------------------------------------------------------------------ op pieces
  // splitLeafSegment (mergeTree.ts:1768-1796) of leaf (b, k) at offset o (0 < o < len): the right part
  // follows it in the same block, with a fresh id; a window leaf's right part joins the window table.
  // R: the block in registers (loaded here); on return *rb/*rk locate the right part.
  FMT_DEV bool splitLeaf(BlockRegs& R, uint32_t b, int k, int o, uint32_t* rightId, uint32_t* rb, int* rk) {
    ProfScope ps_(prof[14]);
    invalidate();
    loadBlock(b, R);
    Leaf x = regLeaf(R, k);
    if (nextId >= S.idCap) return fail(FMT_E_CAPACITY);
    Leaf y = x;
    y.id = nextId++;
    if (rightId) *rightId = y.id;
    y.len = x.len - static_cast<uint32_t>(o);
    y.text = x.text + static_cast<uint32_t>(o);
    x.len = static_cast<uint32_t>(o);
    const uint32_t w = readlane(R.wi, k);
    uint32_t wy = kNone;
    if (w != kNone) {
      wSet(w, 2, x.len);
      wy = winAdd(y.id, y.ins, y.rm, y.len, ldu(wWord3(w)) & kWMetaMask, R.g, b, y.mlo, y.mhi);
    } else {
      st1(S.winIdx + y.id, kNone);
    }
    setLane(R.f[0], k, x.len);
    regsInsert(R, k + 1, y, wy);
    st1(S.leafBlk + y.id, b);
    obRefsMove(x.id, y.id, o, -o);  // the right part takes the references at/after the split
    if (S.hiMask != nullptr) hiPut(y.id, hiGet(x.id));
    if constexpr (Adj) {
      if (pmN > 0) pmCopy(x.id, y.id);  // copyTo (segmentPropertiesManager.ts:300-316)
    }
    if constexpr (Rm) {
      if (rmN > 0 && y.rm != kNotRemoved) {  // its remove-order entries, copied in rmFlush
        if (rmPendN >= 2) return fail(FMT_E_DATA);  // an op splits at most twice (its two boundaries)
        if (rmPendN == 0) {
          rmPendFrom0 = x.id;
          rmPendTo0 = y.id;
        } else {
          rmPendFrom1 = x.id;
          rmPendTo1 = y.id;
        }
        rmPendN++;
      }
    }
    const uint32_t nb = commitBlock(R);
    if (nb != kNone && k + 1 >= kMaxNodes / 2) {
      *rb = nb;
      *rk = k + 1 - kMaxNodes / 2;
    } else {
      *rb = b;
      *rk = k + 1;
    }
    if (nb != kNone) R.b = kNone;  // the registers no longer describe one block
    return status == FMT_OK;
  }

  // Where leaf `id` is now (its block from leafBlk, its slot by id).
  FMT_DEV void locate(uint32_t id, uint32_t* b, int* k) const {
    const uint32_t bb = ldu(S.leafBlk + id);
    const uint32_t cnt = ldu(S.bCount + bb);
    Lane<bool> q;
    FOR_LANES(l) { LANE(q) = l < static_cast<int>(cnt) && rd(S.lId + (li(bb, l))) == id; }
    const uint64_t m = ballot(q);
    *b = bb;
    *k = m ? ctz64(m) : -1;
  }

  // The leaf block after b in document order (kNone at the end).
  FMT_DEV uint32_t nextBlockOf(uint32_t b) const { return nextBlockAt(ldu(S.bGroup + b), ldu(S.bSlot + b)); }
  FMT_DEV uint32_t nextBlockAt(uint32_t g, uint32_t s) const {  // after slot s of group g
    s++;
    if (s < L->gCount[g]) return ldu(slotBlkPtr(g) + s);
    for (int k = groupPos(g) + 1; k < nGroups; k++) {
      g = L->gOrder[k];
      if (L->gCount[g] > 0) return ldu(slotBlkPtr(g));
    }
    return kNone;
  }

  // insertSegments (mergeTree.ts:1484-1517): ensureIntervalBoundary(p) then the inserting walk, both
  // from one search: the new leaf goes before the first qualifying leaf at p, or before the right part
  // of the leaf that strictly contained p.
  // A body-chunk segment's stamps (loadBodySegment): its insert client, whether its insertSegments
  // call splits at the position (the first of a batch), and specToSegment's remove stamps folded.
  struct LoadStamp {
    int client;
    bool boundary;
    int32_t rm;
    uint32_t mlo, mhi, firstRm;
    HiSet hs;  // (remove clients 64..253)
    bool moreRm;
  };
  FMT_DEV void insertText(const fmt_mt_op& op, const LoadStamp* ld = nullptr) {
    ProfScope ps_(prof[12]);
    const int r = op.ref_seq, c = ld ? ld->client : op.client, p = op.pos1;
    const Hit h = find(p, r, c);
    uint32_t b;
    int k;
    BlockRegs R;
    R.b = kNone;
    if (h.found) {
      if (h.st < p && ld != nullptr && !ld->boundary) {  // (a loader batch's later segment: before the leaf holding p)
        b = h.blk;
        k = h.k;
      } else if (h.st < p) {
        if (!splitLeaf(R, h.blk, h.k, p - h.st, nullptr, &b, &k)) return;
      } else {
        b = h.blk;
        k = h.k;
      }
    } else {
      if (p != totalView()) {  // "MergeTree insert failed" (mergeTree.ts:1629)
        fail(FMT_E_DATA);
        return;
      }
      if (lastBlk == kNone) {
        // empty document: the root, childless, takes the segment (insertRecursive's `_pos === 0`
        // leaf, mergeTree.ts:1935-1943) and becomes a leaf block, the first slot of the first group
        const uint32_t rb = static_cast<uint32_t>(root);
        if (ldu(S.bCount + rb) != 0 || L->gCount[L->gOrder[0]] != 0) {
          fail(FMT_E_DATA);
          return;
        }
        FOR_LANES(l) {
          if (l == 0) S.bLeaf[rb] = 1;
        }
        waveSync();
        if (!slotInsert(L->gOrder[0], 0, rb, 0)) return;
        lastBlk = rb;
      }
      b = lastBlk;
      k = -1;
    }
    const uint32_t opLen = op.len | (op.flags & FMT_MT_F_LEN_HI_MASK);
    if (opLen == 0) return;
    if (nextId >= S.idCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    uint32_t insProps = kNoProps;  // seg {text, props}: properties = clone(props) (textSegment.ts:41-52)
    if (op.pos2 > 0) {
      if (static_cast<uint32_t>(op.pos2 - 1) >= in.nPropsOps) {
        fail(FMT_E_DATA);
        return;
      }
      insProps = applyProps(kNoProps, static_cast<uint32_t>(op.pos2 - 1));
      if (status != FMT_OK) return;
    }
    if (R.b != b) loadBlock(b, R);  // (after a split without overflow the block is still in registers)
    if (k < 0) k = R.cnt;
    Leaf x;
    x.len = opLen;
    x.ins = op.seq;
    x.rm = ld ? ld->rm : kNotRemoved;
    x.mlo = ld ? ld->mlo : 0u;
    x.mhi = ld ? ld->mhi : 0u;
    x.id = nextId++;
    x.text = op.payload;
    x.meta = mkMeta(c, insProps) | ((op.flags & FMT_MT_F_MARKER) != 0 ? kMetaMarker : 0u);
    // a window entry unless every stamp is at or below minSeq (a loaded segment can be: its length
    // is then the same in every perspective and goes to the stable sums)
    const bool win = x.ins > minSeq || (x.rm != kNotRemoved && x.rm > minSeq);
    uint32_t wx = kNone;
    if (win) {
      const uint32_t wm = (mkMeta(c, 0) & 0xFFu) | (ld ? (ld->firstRm << 8) | (ld->moreRm ? 1u << 16 : 0u) : 0u);
      wx = winAdd(x.id, x.ins, x.rm, x.len, wm, R.g, b, x.mlo, x.mhi);
    } else {
      st1(S.winIdx + x.id, kNone);
    }
    if ((op.flags & FMT_MT_F_MARKER) != 0) markerAdd(x.id);
    if (S.hiMask != nullptr) {
      HiSet none;
      none.clear();
      hiPut(x.id, ld ? ld->hs : none);
    }
    regsInsert(R, k, x, wx);
    st1(S.leafBlk + x.id, b);
    const uint32_t nb = commitBlock(R);
    if (status != FMT_OK) return;
    // (a block split recounts both halves' stable sums from the registers)
    if (!win && nb == kNone && x.rm == kNotRemoved) addStable(b, static_cast<int>(x.len));
    if (obStartN > 0) obliterateOnInsert(x.id, r, c);
    if (status != FMT_OK) return;
    lru(nb != kNone && k >= kMaxNodes / 2 ? nb : b, x.id, op.seq);
    if (cuRec) {  // the new segment, unless obliterated on arrival (mergeTree.ts:1497-1508)
      uint32_t xb;
      int xk;
      locate(x.id, &xb, &xk);
      if (ldi(S.lRm + li(xb, xk)) == kNotRemoved) cuPush(x.id);
    }
  }

  // SnapshotLoader.loadBody's append of one body-chunk segment (FMT_MT_F_LOADSEG,
  // snapshotLoader.ts:277-309; mt_engine.h loadBodySegment): insertSegments at the local length
  // (every leaf not removed) from PriorPerspective(UniversalSequenceNumber, client) with stamp
  // {seq, client}, a batch of universal segments splitting only at its first; the segment keeps
  // specToSegment's remove stamps (the batch's merge-info row op.pos1, snapshotLoader.ts:105-175).
  FMT_DEV void loadBodySegment(const fmt_mt_op& op) {
    if (in.infoAll == nullptr || in.stamps == nullptr || op.pos1 < 0 || static_cast<uint64_t>(op.pos1) >= in.nInfoAll) {
      fail(FMT_E_DATA);
      return;
    }
    LoadStamp ld;
    ld.client = op.client == FMT_MT_CLIENT_NONCOLLAB ? FMT_NON_COLLAB_CLIENT : static_cast<int>(op.client);
    ld.boundary = (op.flags & FMT_MT_F_GROUP_CONT) == 0;
    ld.rm = kNotRemoved;
    ld.firstRm = 0;
    uint64_t mask = 0;
    ld.hs.clear();
    const fmt_mt_snapshot_info inf = in.infoAll[op.pos1];
    for (uint32_t t = 0; t < inf.rm_count; t++) {
      const fmt_mt_stamp st = in.stamps[inf.rm_first + t];
      const int sc = uni(st.client);
      if (sc < 0 || sc > kMaxClient || (sc > 63 && S.hiMask == nullptr)) {
        fail(FMT_E_UNSUPPORTED);
        return;
      }
      if (uni(st.seq) < ld.rm) {
        ld.rm = uni(st.seq);
        ld.firstRm = static_cast<uint32_t>(sc);
      }
      if (sc < 64) mask |= 1ull << sc;
      else ld.hs.add(sc);
    }
    ld.mlo = static_cast<uint32_t>(mask);
    ld.mhi = static_cast<uint32_t>(mask >> 32);
    ld.moreRm = __builtin_popcountll(mask) + ld.hs.count() > 1;
    invalidate();
    groupCorrections(kLocalSeq, ld.client);  // the local length: every leaf not removed
    const int local = totalView();
    invalidate();
    fmt_mt_op o = op;
    o.pos1 = local;
    o.ref_seq = 0;
    insertText(o, &ld);
  }

  // View lengths of the leaves of block b (lane k = leaf k) from PriorPerspective(r, c).
  FMT_DEV Lane<uint32_t> blockVis(uint32_t b, uint32_t cnt, int r, int c) const {
    Lane<uint32_t> vis;
    FOR_LANES(l) {
      // (all 8 slots loaded, masked by the count after; a stale slot's id indexes nothing: visAny reads
      // the hiMask side table by id only for the block's own leaves)
      const size_t i = li(b, l & 7);
      const uint32_t len = rd(S.lLen + i), mlo = rd(S.lMlo + i), mhi = rd(S.lMhi + i), meta = rd(S.lMeta + i);
      const int32_t ins = rd(S.lIns + i), rm = rd(S.lRm + i);
      const uint32_t id = c < 64 ? 0u : rd(S.lId + i);
      uint32_t v = 0;
      if (l < static_cast<int>(cnt)) v = static_cast<uint32_t>(visAny(len, ins, rm, mlo, mhi, mClient(meta), r, c, id));
      LANE(vis) = v;
    }
    return vis;
  }

  // markRangeRemoved / annotateRange (mergeTree.ts:2009-2081, 2292-2383) from one search: the leaf
  // at `start` and the leaf strictly containing `end` are found before either boundary split
  // (ensureIntervalBoundary moves no view position), then the hits are walked block by block:
  // the leaves of positive view length inside [start, end).
  FMT_DEV void applyRange(const fmt_mt_op& op) {
    ProfScope ps_(prof[13]);
    const int r = op.ref_seq, c = op.client, seq = op.seq;
    const int start = op.pos1, end = op.pos2;
    const Hit h = find(start, r, c);
    if (!h.found) return;  // nothing at or after start: no boundary, no hit
    const uint32_t idStart = ldu(S.lId + li(h.blk, h.k));
    // the leaf strictly containing end, walking from the start leaf
    uint32_t idEnd = kNone, endB = kNone;
    int offEnd = 0, endK = 0;
    {
      uint32_t b = h.blk;
      int k = h.k, pos = h.st;
      while (b != kNone && pos < end && idEnd == kNone) {
        const uint32_t cnt = ldu(S.bCount + b);
        const Lane<uint32_t> vis = blockVis(b, cnt, r, c);
        for (; k < static_cast<int>(cnt) && pos < end; k++) {
          const int v = static_cast<int>(readlane(vis, k));
          if (pos < end && end < pos + v) {
            idEnd = ldu(S.lId + li(b, k));
            offEnd = end - pos;
            endB = b;
            endK = k;
            break;
          }
          pos += v;
        }
        if (idEnd == kNone && pos < end) {
          b = nextBlockOf(b);
          k = 0;
        }
      }
    }
    // boundary splits; the leaves' positions are tracked while no split overflows a block
    BlockRegs R;
    uint32_t fb = h.blk;  // the first leaf of the range
    int fk = h.k;
    uint32_t firstIdv = idStart;
    if (h.st < start) {  // ensureIntervalBoundary(start)
      uint32_t right;
      if (!splitLeaf(R, h.blk, h.k, start - h.st, &right, &fb, &fk)) return;
      firstIdv = right;
      if (idEnd == idStart) {
        idEnd = right;
        offEnd -= start - h.st;
        endB = fb;
        endK = fk;
      } else if (R.b == kNone) {
        endB = kNone;  // moved by an overflow: locate below
      } else if (endB == h.blk) {
        endK++;
      }
    }
    if (idEnd != kNone && offEnd > 0) {  // ensureIntervalBoundary(end)
      if (endB == kNone) locate(idEnd, &endB, &endK);
      uint32_t rb;
      int rk;
      if (!splitLeaf(R, endB, endK, offEnd, nullptr, &rb, &rk)) return;
      if (R.b == kNone) locate(firstIdv, &fb, &fk);  // an overflow may have moved the first leaf
    }
    if (end <= start) return;
    uint32_t b = fb;
    int k = fk;
    int pos = start;
    while (b != kNone && pos < end) {
      // the block's leaves, their window entries and the block's list position in one round each
      const uint32_t cnt = ldu(S.bCount + b);
      const uint32_t g = ldu(S.bGroup + b), s = ldu(S.bSlot + b);
      bool scour = ldi(S.bScour + b) == 1;
      Lane<uint32_t> f[8], wi, vis;
      FOR_LANES(l) {
        const size_t i = li(b, l & 7);  // (all 8 slots: the loads do not wait for the count)
        LANE(f[0]) = rd(S.lLen + i);
        LANE(f[1]) = static_cast<uint32_t>(rd(S.lIns + i));
        LANE(f[2]) = static_cast<uint32_t>(rd(S.lRm + i));
        LANE(f[3]) = rd(S.lMlo + i);
        LANE(f[4]) = rd(S.lMhi + i);
        LANE(f[5]) = rd(S.lId + i);
        LANE(f[6]) = rd(S.lText + i);
        LANE(f[7]) = rd(S.lMeta + i);
      }
      FOR_LANES(l) {
        // (slots past the count hold stale fields, possibly never-written memory: no index from them)
        LANE(wi) = l < static_cast<int>(cnt) ? rd(S.winIdx + LANE(f[5])) : kNone;
        LANE(vis) = l < static_cast<int>(cnt)
                        ? static_cast<uint32_t>(visAny(LANE(f[0]), static_cast<int32_t>(LANE(f[1])), static_cast<int32_t>(LANE(f[2])),
                                                       LANE(f[3]), LANE(f[4]), mClient(LANE(f[7])), r, c, LANE(f[5])))
                        : 0u;
      }
      int stableDelta = 0;
      for (; k < static_cast<int>(cnt) && pos < end; k++) {
        const int v = static_cast<int>(readlane(vis, k));
        if (v > 0) {
          Leaf x;
          x.len = readlane(f[0], k);
          x.ins = static_cast<int32_t>(readlane(f[1], k));
          x.rm = static_cast<int32_t>(readlane(f[2], k));
          x.mlo = readlane(f[3], k);
          x.mhi = readlane(f[4], k);
          x.id = readlane(f[5], k);
          x.text = readlane(f[6], k);
          x.meta = readlane(f[7], k);
          if (op.type == FMT_MT_REMOVE) {
            stableDelta += removeLeaf(b, k, x, seq, c, readlane(wi, k), g);
          } else {
            annotateLeaf(b, k, x, op.payload, seq);
            if (cuRec && x.rm == kNotRemoved) cuPush(x.id);  // deltaSegments: annotated, not removed (:2045-2047)
          }
          if (status != FMT_OK) return;
          if (!scour && seq > curSeq) {  // addToLRUSet (mergeTree.ts:812-822), once per block
            st1(S.bScour + b, 1);
            heapAdd(seq, x.id);
            scour = true;
            if (status != FMT_OK) return;
          }
        }
        pos += v;
      }
      if (stableDelta) addStableAt(g, s, stableDelta);
      if (pos < end) {
        b = nextBlockAt(g, s);
        k = 0;
      }
    }
  }

  // Remove leaf (b, j) (window entry w, block group g); returns the change of b's stable sum.
  FMT_DEV int removeLeaf(uint32_t b, int j, Leaf& x, int seq, int c, uint32_t w, uint32_t g) {
    const bool was = x.rm != kNotRemoved;
    if (!was) {
      x.rm = seq;
      if (cuRec) cuPush(x.id);  // removedSegments: hits not removed before this op (mergeTree.ts:2314-2321)
    } else if constexpr (Rm) {
      if (rmRec) rmPushHit(x.id);  // a later remove stamp (stamps.ts:144-158), recorded in rmFlush
    }
    if (c < 32) x.mlo |= 1u << c;
    else if (c < 64) x.mhi |= 1u << (c - 32);
    else hiSet(x.id, c);
    putLeaf(b, j, x);
    invalidate();
    if (w == kNone) {  // a stable leaf enters the window: its length leaves the stable sums
      winAdd(x.id, x.ins, x.rm, x.len, (mkMeta(mClient(x.meta), 0) & 0xFFu) | (static_cast<uint32_t>(c) << 8), g, b, x.mlo, x.mhi);
      return -static_cast<int>(x.len);
    }
    if (!was) {
      const uint32_t m3 = ldu(wWord3(w));
      wSet(w, 1, static_cast<uint32_t>(x.rm));
      wSet(w, 3, (m3 & ~(kWMetaMask ^ 0xFFu)) | (static_cast<uint32_t>(c) << 8));
    } else {
      wSet(w, 3, ldu(wWord3(w)) | (1u << 16));  // a later remover
    }
    wSetMask(w, x.mlo, x.mhi);
    return 0;
  }

  FMT_DEV void annotateLeaf(uint32_t b, int j, Leaf& x, uint32_t opId, int seq) {
    if constexpr (Adj) {  // the leaf's PropertiesManager first (handleProperties, :188-238)
      if (in.adj != nullptr) {
        pmAnnotate(x.id, mProps(x.meta), opId, seq);
        if (status != FMT_OK) return;
      }
    }
    const uint32_t np = applyProps(mProps(x.meta), opId, true);
    if (status != FMT_OK) return;
    x.meta = (x.meta & ~(0xFFFFu << 8)) | (np << 8);
    putLeaf(b, j, x);
  }

  // ------------------------------------------------------------------ obliterates (f1)
  // Obliterates (mergeTree.ts:515-635, 2083-2290), the same rules as mt_engine.h. A reference's
  // "ordinal" is its leaf's document order — (group position, slot, index in block) here — or ""
  // (smallest, -1) once the leaf is gone from the tree or the reference was removed.
  FMT_DEV int64_t ordOf(uint32_t id) const {
    if (id == 0) return -1;
    if (ldu(S.leafBlk + id) == kNone) return -1;
    uint32_t b;
    int k;
    locate(id, &b, &k);
    if (k < 0) return -1;
    return (static_cast<int64_t>(groupPos(ldu(S.bGroup + b))) << 16) | (static_cast<int64_t>(ldu(S.bSlot + b)) << 3) | k;
  }
  FMT_DEV static int ordinalCompare(int64_t a, int64_t b) {
    if (a < 0 || b < 0) return (a < 0) == (b < 0) ? 0 : (a < 0 ? -1 : 1);
    return a < b ? -1 : (a > b ? 1 : 0);
  }
  // ---- the live-obliterate table in HBM (HugeState::obRec ...): fields of slot `slot`
  enum : int { kObStartId = 0, kObStartOff = 1, kObEndId = 2, kObEndOff = 3, kObSeq = 4, kObClient = 5 };
  FMT_DEV uint32_t obF(int slot, int f) const { return ldu(S.obRec + 6 * static_cast<size_t>(slot) + f); }
  FMT_DEV int obU(const uint32_t* p, int i) const { return static_cast<int>(ldu(p + i)); }
  // p[at + 1 .. n] = p[at .. n - 1] (one entry opens at `at`), 64 entries per step from the top
  FMT_DEV void listOpen(uint32_t* p, int at, int n) {
    for (int hi = n; hi > at; hi -= 64) {
      const int lo = hi - 64 > at ? hi - 64 : at;  // destinations (lo, hi]
      Lane<uint32_t> v;
      FOR_LANES(l) { LANE(v) = lo + 1 + l <= hi ? rd(p + lo + l) : 0u; }
      waveSync();
      FOR_LANES(l) {
        if (lo + 1 + l <= hi) p[lo + 1 + l] = LANE(v);
      }
      waveSync();
    }
  }
  // p[at .. n - 2] = p[at + 1 .. n - 1] (entry `at` closes), 64 entries per step from the bottom
  FMT_DEV void listClose(uint32_t* p, int at, int n) {
    for (int lo = at; lo + 1 < n; lo += 64) {
      const int hi = lo + 64 < n - 1 ? lo + 64 : n - 1;  // destinations [lo, hi)
      Lane<uint32_t> v;
      FOR_LANES(l) { LANE(v) = lo + l < hi ? rd(p + lo + l + 1) : 0u; }
      waveSync();
      FOR_LANES(l) {
        if (lo + l < hi) p[lo + l] = LANE(v);
      }
      waveSync();
    }
  }
  FMT_DEV int startCompare(int a, int b) const {  // SortedSegmentSet.compare on start references
    const int c = ordinalCompare(ordOf(obF(a, kObStartId)), ordOf(obF(b, kObStartId)));
    return c != 0 ? c : static_cast<int>(obF(a, kObStartOff)) - static_cast<int>(obF(b, kObStartOff));
  }
  // SortedSet.findItemPosition + SortedSegmentSet.onFindEquivalent, verbatim: the array is only as
  // sorted as the ordinals were at insertion.
  FMT_DEV int findStart(int slot, bool* exists) const {
    *exists = false;
    if (obStartN == 0) return 0;
    int start = 0, end = obStartN - 1, index = -1;
    while (start <= end) {
      index = start + (end - start) / 2;
      const int at = obU(S.obStart, index);
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
        for (int b = index - 1; b >= 0 && startCompare(slot, obU(S.obStart, b)) == 0; b--)
          if (obU(S.obStart, b) == slot) {
            *exists = true;
            return b;
          }
        for (; index < obStartN && startCompare(slot, obU(S.obStart, index)) == 0; index++)
          if (obU(S.obStart, index) == slot) {
            *exists = true;
            return index;
          }
        return index;
      }
    }
    return index;
  }

  // References on leaf `from` at offset >= minOff move to leaf `to`, offset += add (split: the right
  // part; zamboni append: every reference of the appended leaf). Lane l takes slots l, l + 64, ...
  // up to the highest slot ever taken.
  FMT_DEV void obRefsMove(uint32_t from, uint32_t to, int minOff, int add) {
    if (obLive == 0) return;
    for (int base = 0; base < obSlotsHi; base += 64) {
      FOR_LANES(l) {
        const int k = base + l;
        if (k < obSlotsHi && rd(S.obUsed + k) != 0u) {
          uint32_t* e = S.obRec + 6 * static_cast<size_t>(k);
          const uint32_t sId = rd(e + kObStartId), eId = rd(e + kObEndId);
          const int sOff = static_cast<int>(rd(e + kObStartOff)), eOff = static_cast<int>(rd(e + kObEndOff));
          if (sId == from && sOff >= minOff) {
            e[kObStartId] = to;
            e[kObStartOff] = static_cast<uint32_t>(sOff + add);
          }
          if (eId == from && eOff >= minOff) {
            e[kObEndId] = to;
            e[kObEndOff] = static_cast<uint32_t>(eOff + add);
          }
        }
      }
    }
    waveSync();
  }

  FMT_DEV bool obAdd(uint32_t sId, int sOff, uint32_t eId, int eOff, int seq, int client) {
    int slot = -1;
    const int cap = static_cast<int>(S.obCap);
    for (int base = 0; base < cap && slot < 0; base += 64) {
      Lane<bool> q;
      FOR_LANES(l) { LANE(q) = base + l < cap && rd(S.obUsed + base + l) == 0u; }
      const uint64_t m = ballot(q);
      if (m) slot = base + ctz64(m);
    }
    if (slot < 0 || obSeqN >= cap) return fail(FMT_E_CAPACITY);
    FOR_LANES(l) {
      if (l == 0) {
        S.obUsed[slot] = 1u;
        uint32_t* e = S.obRec + 6 * static_cast<size_t>(slot);
        e[kObStartId] = sId;
        e[kObStartOff] = static_cast<uint32_t>(sOff);
        e[kObEndId] = eId;
        e[kObEndOff] = static_cast<uint32_t>(eOff);
        e[kObSeq] = static_cast<uint32_t>(seq);
        e[kObClient] = static_cast<uint32_t>(client);
        S.obSeq[obSeqN] = static_cast<uint32_t>(slot);
      }
    }
    waveSync();
    if (slot + 1 > obSlotsHi) obSlotsHi = slot + 1;
    obLive++;
    obSeqN++;
    bool exists;
    const int at = findStart(slot, &exists);
    if (!exists) {
      if (obStartN >= cap) return fail(FMT_E_CAPACITY);
      listOpen(S.obStart, at, obStartN);
      st1(S.obStart + at, static_cast<uint32_t>(slot));
      waveSync();
      obStartN++;
    }
    return true;
  }

  // Obliterates.setMinSeq (mergeTree.ts:537-545): drop obliterates at/below minSeq from both lists
  // and remove their references.
  FMT_DEV void obSetMinSeq() {
    int k = 0;
    for (; k < obSeqN && static_cast<int>(obF(obU(S.obSeq, k), kObSeq)) <= minSeq; k++) {
      const int slot = obU(S.obSeq, k);
      bool exists;
      const int at = findStart(slot, &exists);
      if (exists) {
        listClose(S.obStart, at, obStartN);
        obStartN--;
      }
      FOR_LANES(l) {  // removeLocalReferencePosition
        if (l == 0) {
          S.obRec[6 * static_cast<size_t>(slot) + kObStartId] = 0u;
          S.obRec[6 * static_cast<size_t>(slot) + kObEndId] = 0u;
        }
      }
      waveSync();
      if (!exists) continue;  // still listed in startOrdered: its slot stays taken
      st1(S.obUsed + slot, 0u);
      waveSync();
      obLive--;
    }
    if (k > 0) {
      for (int i = 0; i < k; i++) listClose(S.obSeq, 0, obSeqN - i);  // (k is almost always 1)
      obSeqN -= k;
    }
  }

  // blockInsert's obliterate branch (mergeTree.ts:1642-1746) for the new leaf `id`: every overlapping
  // obliterate the inserter had not seen (seq > refSeq); when one is from another client and the
  // newest is not the inserter's own, the leaf starts out removed by those other clients' ones.
  FMT_DEV void obliterateOnInsert(uint32_t id, int refSeq, int client) {
    const int64_t k = ordOf(id);
    int minSeqOther = kNotRemoved, newestSeq = -1, newestClient = -1, firstCl = 0;
    uint32_t mlo = 0, mhi = 0;
    HiSet hs;
    hs.clear();
    bool any = false;
    for (int i = 0; i < obStartN; i++) {  // Obliterates.findOverlapping (:566-582)
      const int slot = obU(S.obStart, i);
      const int64_t si = ordOf(obF(slot, kObStartId));
      if (!(si >= 0 && si <= k)) break;
      const int64_t ei = ordOf(obF(slot, kObEndId));
      if (!(ei >= 0 && ei >= k)) continue;
      const int oseq = static_cast<int>(obF(slot, kObSeq)), ocl = static_cast<int>(obF(slot, kObClient));
      if (oseq <= refSeq) continue;
      if (ocl != client) {
        any = true;
        if (ocl < 32) mlo |= 1u << ocl;
        else if (ocl < 64) mhi |= 1u << (ocl - 32);
        else hs.add(ocl);
        if (oseq < minSeqOther) {
          minSeqOther = oseq;
          firstCl = ocl;
        }
      }
      if (oseq > newestSeq) {
        newestSeq = oseq;
        newestClient = ocl;
      }
    }
    if (!(any && newestClient != client)) return;
    if constexpr (Rm) {
    if (rmRec) {  // SnapshotV1: every stamp but the first (rm_seq) is a remove-order entry (mergeTree.ts:1715-1725)
      bool firstSkipped = false;
      for (int i = 0; i < obStartN && status == FMT_OK; i++) {
        const int slot = obU(S.obStart, i);
        const int64_t si = ordOf(obF(slot, kObStartId));
        if (!(si >= 0 && si <= k)) break;
        const int64_t ei = ordOf(obF(slot, kObEndId));
        if (!(ei >= 0 && ei >= k)) continue;
        const int oseq = static_cast<int>(obF(slot, kObSeq)), ocl = static_cast<int>(obF(slot, kObClient));
        if (oseq <= refSeq || ocl == client) continue;
        if (!firstSkipped && oseq == minSeqOther) {
          firstSkipped = true;
          continue;
        }
        rmAppend(id, ocl, oseq, FMT_MT_RM_SLICE);
      }
    }
    }
    uint32_t b;
    int kk;
    locate(id, &b, &kk);
    const size_t i = li(b, kk);
    st1(S.lRm + i, static_cast<int32_t>(minSeqOther));
    st1(S.lMlo + i, mlo);
    st1(S.lMhi + i, mhi);
    if (S.hiMask != nullptr) hiPut(id, hs);
    const uint32_t w = ldu(S.winIdx + id);  // (a new leaf: always a window entry)
    const bool more = __builtin_popcount(mlo) + __builtin_popcount(mhi) + hs.count() > 1;
    wSet(w, 1, static_cast<uint32_t>(minSeqOther));
    wSet(w, 3, (ldu(wWord3(w)) & ~(kWMetaMask ^ 0xFFu)) | (static_cast<uint32_t>(firstCl) << 8) | (more ? 1u << 16 : 0u));
    wSetMask(w, mlo, mhi);
    invalidate();
  }

  // ensureIntervalBoundary (mergeTree.ts:1798-1808): split the leaf that strictly contains pos in
  // the op's view.
  FMT_DEV bool splitAt(int pos, int r, int c) {
    const Hit h = find(pos, r, c);
    if (!h.found || h.st >= pos) return status == FMT_OK;
    BlockRegs R;
    uint32_t rb;
    int rk;
    return splitLeaf(R, h.blk, h.k, pos - h.st, nullptr, &rb, &rk);
  }

  // obliterateRangeSided (mergeTree.ts:2083-2260). Places {pos, before?}: a non-sided op is
  // {pos1, Before} .. {pos2 - 1, After} (:2282-2286); a sided one carries its sides in flags. The
  // boundaries are the places' Before edges (:2090-2091). nodeMap(start.pos, end.pos + 1) under
  // RemoteObliteratePerspective visits a leaf when it has length in the op's view or is not removed
  // at all (so concurrent inserts strictly inside are caught): st < end.pos + 1, start.pos < st + vis;
  // markRemoved skips the exclusive endpoints (:2145-2152). Endpoint references go to the leaves
  // holding start.pos and end.pos in the op's view (getContainingSegment, :858-886).
  FMT_DEV void applyObliterate(const fmt_mt_op& op) {
    ProfScope ps_(prof[13]);
    const int r = op.ref_seq, c = op.client, seq = op.seq;
    const bool sided = op.type == FMT_MT_OBLITERATE_SIDED;
    const bool sB = !sided || (op.flags & FMT_MT_F_START_BEFORE) != 0;
    const bool eB = sided && (op.flags & FMT_MT_F_END_BEFORE) != 0;
    const int sPl = op.pos1, ePl = sided ? op.pos2 : op.pos2 - 1;
    const int startPos = sB ? sPl : sPl + 1, endPos = eB ? ePl : ePl + 1, endW = ePl + 1;
    if (!splitAt(startPos, r, c) || !splitAt(endPos, r, c)) return;
    const Hit h = find(sPl, r, c);  // every leaf before it ends at or before sPl: no hit
    if (!h.found) {
      fail(FMT_E_DATA);  // "segments cannot be undefined"
      return;
    }
    uint32_t sId = 0, eId = 0;
    int sOff = 0, eOff = 0;
    uint32_t b = h.blk;
    int k = h.k, pos = h.st;
    while (b != kNone && pos < endW) {
      const uint32_t cnt = ldu(S.bCount + b);
      const uint32_t g = ldu(S.bGroup + b), s = ldu(S.bSlot + b);
      bool scour = ldi(S.bScour + b) == 1;
      Lane<uint32_t> f[8], wi, vis;
      FOR_LANES(l) {
        const size_t i = li(b, l & 7);  // (all 8 slots: the loads do not wait for the count)
        LANE(f[0]) = rd(S.lLen + i);
        LANE(f[1]) = static_cast<uint32_t>(rd(S.lIns + i));
        LANE(f[2]) = static_cast<uint32_t>(rd(S.lRm + i));
        LANE(f[3]) = rd(S.lMlo + i);
        LANE(f[4]) = rd(S.lMhi + i);
        LANE(f[5]) = rd(S.lId + i);
        LANE(f[6]) = rd(S.lText + i);
        LANE(f[7]) = rd(S.lMeta + i);
      }
      FOR_LANES(l) {
        // (slots past the count hold stale fields, possibly never-written memory: no index from them)
        LANE(wi) = l < static_cast<int>(cnt) ? rd(S.winIdx + LANE(f[5])) : kNone;
        LANE(vis) = l < static_cast<int>(cnt)
                        ? static_cast<uint32_t>(visAny(LANE(f[0]), static_cast<int32_t>(LANE(f[1])), static_cast<int32_t>(LANE(f[2])),
                                                       LANE(f[3]), LANE(f[4]), mClient(LANE(f[7])), r, c, LANE(f[5])))
                        : 0u;
      }
      int stableDelta = 0;
      for (; k < static_cast<int>(cnt) && pos < endW; k++) {
        const int v = static_cast<int>(readlane(vis, k));
        const uint32_t len = readlane(f[0], k);
        const bool removed = static_cast<int32_t>(readlane(f[2], k)) != kNotRemoved;
        if (v > 0 && sId == 0 && pos <= sPl && sPl < pos + v) {
          sId = readlane(f[5], k);
          sOff = sPl - pos;
        }
        if (v > 0 && eId == 0 && pos <= ePl && ePl < pos + v) {
          eId = readlane(f[5], k);
          eOff = ePl - pos;
        }
        const bool excl = (!sB && startPos == pos + static_cast<int>(len)) || (eB && endPos == pos && v > 0);
        if (!(v == 0 && removed) && !excl && sPl < pos + v) {
          Leaf x;
          x.len = len;
          x.ins = static_cast<int32_t>(readlane(f[1], k));
          x.rm = static_cast<int32_t>(readlane(f[2], k));
          x.mlo = readlane(f[3], k);
          x.mhi = readlane(f[4], k);
          x.id = readlane(f[5], k);
          x.text = readlane(f[6], k);
          x.meta = readlane(f[7], k);
          stableDelta += removeLeaf(b, k, x, seq, c, readlane(wi, k), g);
          if (status != FMT_OK) return;
          if (!scour && seq > curSeq) {  // addToLRUSet (mergeTree.ts:812-822), once per block
            st1(S.bScour + b, 1);
            heapAdd(seq, x.id);
            scour = true;
            if (status != FMT_OK) return;
          }
        }
        pos += v;
      }
      if (stableDelta) addStableAt(g, s, stableDelta);
      if (pos < endW) {
        b = nextBlockAt(g, s);
        k = 0;
      }
    }
    if (sId == 0 || eId == 0) {
      fail(FMT_E_DATA);
      return;
    }
    obAdd(sId, sOff, eId, eOff, seq, c);
  }

  // ------------------------------------------------------------------ remove order (SnapshotV1)
  // As mt_engine.h rmAppend / rmFlush: an FMT_MT_F_RMORDER REMOVE or obliterate that hits an
  // already-removed leaf adds the op's stamp to it; the right part of a split leaf inherits the left
  // part's entries; obliterate-on-insert adds every overlapping stamp past the first. Entries hold
  // leaf ids until writeOutputs turns them into output indices (FMT_MT_LEAF_GONE once dropped).
  FMT_DEV void rmAppend(uint32_t id, int client, int seq, uint32_t kind) {
    if (in.rmOrder == nullptr || rmN >= in.rmOrderCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    FOR_LANES(l) {
      if (l == 0) {
        fmt_mt_remove_order e;
        e.leaf = id;
        e.client = client;
        e.seq = seq;
        e.kind = kind;
        in.rmOrder[rmN] = e;
      }
    }
    waveSync();
    rmN++;
  }
  FMT_DEV void rmPushHit(uint32_t id) {
    if (rmHitN >= S.idCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    st1(S.rmIds + rmHitN, id);
    rmHitN++;
  }
  FMT_DEV void rmFlush(int client, int seq) {
    for (int q = 0; q < rmPendN && status == FMT_OK; q++) {
      const uint32_t from = q == 0 ? rmPendFrom0 : rmPendFrom1, to = q == 0 ? rmPendTo0 : rmPendTo1;
      const uint32_t n0 = rmN;
      for (uint32_t k = 0; k < n0 && status == FMT_OK; k++) {
        const uint32_t* e = reinterpret_cast<const uint32_t*>(in.rmOrder + k);
        if (ldu(e) == from) rmAppend(to, ldi(reinterpret_cast<const int32_t*>(e + 1)),
                                     ldi(reinterpret_cast<const int32_t*>(e + 2)), ldu(e + 3));
      }
    }
    rmPendN = 0;
    for (uint32_t q = 0; q < rmHitN && status == FMT_OK; q++) rmAppend(ldu(S.rmIds + q), client, seq, rmKind);
    rmHitN = 0;
  }

  // ------------------------------------------------------------------ relative positions
  // posFromRelativePos (mergeTree.ts:1462-1483), as mt_engine.h: the marker whose "markerId" holds
  // the id (the last inserted one when several do), -1 when none does or it is removed; else its start
  // in the op's perspective, then the side and offset. Markers are found through the document's
  // marker list (every marker leaf inserted or loaded, dropped ones skipped), positioned through the
  // group / slot index as the catch-up ranges are.
  FMT_DEV void markerAdd(uint32_t id) {
    if (S.mkIds == nullptr) return;
    if (mkN >= S.mkCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    st1(S.mkIds + mkN, id);
    mkN++;
  }
  FMT_DEV bool setHas(uint32_t p, uint32_t want) const {  // (lane-level) prop set p holds entry want
    if (p == kNoProps) return false;
    const uint32_t n = rd(S.props + p * kPropWords);
    bool f = false;
    for (uint32_t k = 0; k < n && k < FMT_MT_PROPS_KEYS_MAX; k++) f = f || setKv(p, k) == want;
    return f;
  }
  // View start of leaf `id` from PriorPerspective(r, c)
  FMT_DEV int viewStart(uint32_t id, int r, int c) {
    uint32_t b;
    int k;
    locate(id, &b, &k);
    invalidate();
    groupCorrections(r, c);
    const uint32_t g = ldu(S.bGroup + b), s = ldu(S.bSlot + b);
    const int gp = groupPos(g);
    int base = 0;
    for (int q = 0; q < gp; q += 64) {
      const Lane<uint32_t> len = groupLens(q);
      Lane<uint32_t> part;
      FOR_LANES(l) { LANE(part) = q + l < gp ? LANE(len) : 0u; }
      uint32_t tot;
      waveExclusiveSum(part, &tot);
      base += static_cast<int>(tot);
    }
    slotLengths(g, r, c);
    for (uint32_t q = 0; q < s; q += 64) {
      Lane<uint32_t> part;
      FOR_LANES(l) { LANE(part) = q + l < s ? static_cast<uint32_t>(L->sLen[q + l]) : 0u; }
      uint32_t tot;
      waveExclusiveSum(part, &tot);
      base += static_cast<int>(tot);
    }
    const Lane<uint32_t> vis = blockVis(b, ldu(S.bCount + b), r, c);
    Lane<uint32_t> part;
    FOR_LANES(l) { LANE(part) = l < k ? LANE(vis) : 0u; }
    uint32_t tot;
    waveExclusiveSum(part, &tot);
    invalidate();
    return base + static_cast<int>(tot);
  }
  FMT_DEV int posFromRelativePos(uint32_t idx, int r, int c) {
    const uint32_t mid = ldu(&in.relpos[idx].marker_id);
    const int offset = ldi(reinterpret_cast<const int32_t*>(&in.relpos[idx].offset));
    const bool before = (ldu(&in.relpos[idx].flags) & FMT_MT_REL_BEFORE) != 0;
    if (mid == FMT_MT_NO_MARKER || in.markerKey == FMT_MT_NO_MARKER || mid > 0xFFFFu || S.mkIds == nullptr) return -1;
    const uint32_t want = (in.markerKey << 16) | mid;
    uint32_t best = kNone;
    int bestIns = -1;
    int64_t bestOrd = -1;
    for (uint32_t base = 0; base < mkN; base += 64) {
      Lane<bool> hit;
      Lane<uint32_t> ids;
      FOR_LANES(l) {
        bool h = false;
        uint32_t id = 0;
        if (base + l < mkN) {
          id = rd(S.mkIds + base + l);
          const uint32_t b = rd(S.leafBlk + id);
          if (b != kNone) {
            const uint32_t cnt = rd(S.bCount + b);
            for (uint32_t k = 0; k < cnt && k < static_cast<uint32_t>(kMaxNodes); k++)
              if (rd(S.lId + li(b, static_cast<int>(k))) == id) h = setHas(mProps(rd(S.lMeta + li(b, static_cast<int>(k)))), want);
          }
        }
        LANE(hit) = h;
        LANE(ids) = id;
      }
      for (uint64_t m = ballot(hit); m != 0; m &= m - 1) {  // the last inserted (ties: the later in the document)
        const uint32_t id = readlane(ids, ctz64(m));
        uint32_t b;
        int k;
        locate(id, &b, &k);
        const int ins = ldi(S.lIns + li(b, k));
        const int64_t ord = ordOf(id);
        if (ins > bestIns || (ins == bestIns && ord > bestOrd)) {
          best = id;
          bestIns = ins;
          bestOrd = ord;
        }
      }
    }
    if (best == kNone) return -1;
    uint32_t b;
    int k;
    locate(best, &b, &k);
    if (ldi(S.lRm + li(b, k)) != kNotRemoved) return -1;
    int pos = viewStart(best, r, c);
    if (before) pos -= offset;
    else pos += static_cast<int>(ldu(S.lLen + li(b, k))) + offset;
    return pos;
  }
  // getValidOpRange (client.ts:758-767): an undefined pos1 / pos2 comes from relativePos1 / 2.
  FMT_DEV bool resolveRelative(fmt_mt_op& op) {
    for (int k = 0; k < 2; k++) {
      if ((op.flags & (k == 0 ? FMT_MT_F_REL1 : FMT_MT_F_REL2)) == 0) continue;
      const int32_t idx = k == 0 ? op.pos1 : op.pos2;
      const int pos = idx >= 0 && static_cast<uint32_t>(idx) < in.nRelpos && in.relpos != nullptr
                          ? posFromRelativePos(static_cast<uint32_t>(idx), op.ref_seq, op.client)
                          : -1;
      if (pos < 0) {
        fail(FMT_E_DATA);
        return false;
      }
      if (k == 0) op.pos1 = pos;
      else op.pos2 = pos;
    }
    invalidate();
    return true;
  }

  // ------------------------------------------------------------------ catch-up ranges
  // The delta event of an FMT_MT_F_CATCHUP op regenerated as position ranges (sequence.ts:395-452),
  // positions in the local view right after the op, before its zamboni pass (Client.getPosition):
  // INSERT [pos, pos + len) of the new leaf; REMOVE / OBLITERATE the newly removed leaves, merged
  // while they start at the same position; ANNOTATE the annotated leaves not removed, merged while
  // contiguous. The local view counts every leaf not removed: perspective (kLocalSeq, any client).
  static constexpr int kLocalSeq = 0x7FFFFFFE;
  FMT_DEV void cuPush(uint32_t id) {
    if (cuIdN >= S.idCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    st1(S.cuIds + cuIdN, id);
    cuIdN++;
  }
  FMT_DEV void cuEmit(int p1, int p2, int type) {
    if (cuN >= in.catchupCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    FOR_LANES(l) {
      if (l == 0) {
        fmt_mt_catchup_range r;
        r.op = opIdx;
        r.pos1 = p1;
        r.pos2 = p2;
        r.type = static_cast<uint32_t>(type);
        in.catchup[cuN] = r;
      }
    }
    cuN++;
  }
  FMT_DEV void recordCatchup(int type) {
    if (cuIdN == 0) return;
    waveSync();
    invalidate();
    groupCorrections(kLocalSeq, 0);
    uint32_t b;
    int k0;
    locate(ldu(S.cuIds), &b, &k0);
    if (k0 < 0) {
      fail(FMT_E_DATA);
      return;
    }
    // local start of block b: the groups before its group, then the slots before its slot
    const uint32_t g = ldu(S.bGroup + b), s = ldu(S.bSlot + b);
    const int gp = groupPos(g);
    int base = 0;
    for (int k = 0; k < gp; k += 64) {
      const Lane<uint32_t> len = groupLens(k);
      Lane<uint32_t> part;
      FOR_LANES(l) { LANE(part) = k + l < gp ? LANE(len) : 0u; }
      uint32_t tot;
      waveExclusiveSum(part, &tot);
      base += static_cast<int>(tot);
    }
    slotLengths(g, kLocalSeq, 0);
    for (uint32_t q = 0; q < s; q += 64) {
      Lane<uint32_t> part;
      FOR_LANES(l) { LANE(part) = q + l < s ? static_cast<uint32_t>(L->sLen[q + l]) : 0u; }
      uint32_t tot;
      waveExclusiveSum(part, &tot);
      base += static_cast<int>(tot);
    }
    int p1 = 0, p2 = 0;
    bool open = false;
    uint32_t q = 0;
    while (q < cuIdN) {
      if (b == kNone) {
        fail(FMT_E_DATA);
        return;
      }
      const int cnt = static_cast<int>(ldu(S.bCount + b));
      Lane<uint32_t> loc, ids;
      FOR_LANES(l) {
        const size_t i = li(b, l < cnt ? l : 0);
        LANE(ids) = l < cnt ? rd(S.lId + i) : 0u;
        LANE(loc) = l < cnt && rd(S.lRm + i) == kNotRemoved ? rd(S.lLen + i) : 0u;
      }
      uint32_t tot;
      const Lane<uint32_t> ex = waveExclusiveSum(loc, &tot);
      for (; q < cuIdN; q++) {
        const uint32_t id = ldu(S.cuIds + q);
        Lane<bool> hit;
        FOR_LANES(l) { LANE(hit) = l < cnt && LANE(ids) == id; }
        const uint64_t m = ballot(hit);
        if (m == 0) break;
        const int lane = ctz64(m);
        const int pos = base + static_cast<int>(readlane(ex, lane));
        const int len = static_cast<int>(ldu(S.lLen + li(b, lane)));
        if (open && (((type == FMT_MT_REMOVE || type == FMT_MT_OBLITERATE) && p1 == pos) || (type == FMT_MT_ANNOTATE && p2 == pos))) {
          p2 += len;
          continue;
        }
        if (open) cuEmit(p1, p2, type);
        p1 = pos;
        p2 = pos + len;
        open = true;
      }
      base += static_cast<int>(tot);
      if (q < cuIdN) b = nextBlockOf(b);
    }
    if (open) cuEmit(p1, p2, type);
    invalidate();
  }

  // ------------------------------------------------------------------ minSeq
  // Window entries whose insert and first remove are both at/below minSeq graduate into the stable
  // sums (mergeTree.ts:1147-1166 moves the window; their length is now the same for every view).
  FMT_DEV void graduate() {
    ProfScope ps_(prof[4]);
    uint32_t w = 0;
    while (w < nWin) {
      const uint32_t base = w;
      Lane<bool> q;
      FOR_LANES(l) {
        const uint32_t i = base + l;
        bool g = false;
        if (i < nWin) {
          const u32x4 x = wRecOf(i);
          const int32_t rm = static_cast<int32_t>(x[1]);
          g = static_cast<int32_t>(x[0]) <= minSeq && (rm == kNotRemoved || rm <= minSeq);
        }
        LANE(q) = g;
      }
      const uint64_t m = ballot(q);
      if (!m) {
        w += 64;
        continue;
      }
      const uint32_t e = base + static_cast<uint32_t>(ctz64(m));
      const int32_t rm = static_cast<int32_t>(ldu(wWord(e, 1)));
      const uint32_t len = ldu(wWord(e, 2)), blk = ldu(S.wBlk + e);
      winRemove(e);  // the entry moved into e is examined next
      if (rm == kNotRemoved) addStable(blk, static_cast<int>(len));
      w = e;
    }
    invalidate();
  }

  // ------------------------------------------------------------------ zamboni (zamboni.ts:33-213)
  // Leaves of up to 8 leaf blocks in one vector load per field: lane 8i + k = leaf k of blocks[i]
  // (cntL: block i's leaf count in every lane of its octet), plus each leaf's last text unit.
  FMT_DEV void loadOctets(const Lane<uint32_t>& blk, const Lane<int>& cntL, Lane<uint32_t>* f, Lane<uint32_t>& lastCh) const {
    FOR_LANES(l) {
      const int k = l & 7;
      const bool on = k < LANE(cntL);
      const size_t i = li(LANE(blk), on ? k : 0);
      LANE(f[0]) = on ? rd(S.lLen + i) : 0u;
      LANE(f[1]) = static_cast<uint32_t>(rd(S.lIns + i));
      LANE(f[2]) = static_cast<uint32_t>(rd(S.lRm + i));
      LANE(f[3]) = rd(S.lMlo + i);
      LANE(f[4]) = rd(S.lMhi + i);
      LANE(f[5]) = rd(S.lId + i);
      LANE(f[6]) = rd(S.lText + i);
      LANE(f[7]) = rd(S.lMeta + i);
      const uint32_t ln = LANE(f[0]);
      LANE(lastCh) = ln > 0 ? textAt(LANE(f[6]) + ln - 1) : 0u;
    }
  }

  // scourNode decisions (zamboni.ts:141-213) over loaded octets, serial per block: dst[s] = output
  // index taken by source lane s (-1: dropped); a leaf appended onto the previous kept leaf takes its
  // run head's output. Merged runs are consecutive source lanes, so their text, concatenated in lane
  // order, is written to the merge area at mergeBase (lane s's units at mergeBase + flat[s]).
  struct ScourPlan {
    Lane<int> dst, srcOf;
    Lane<uint32_t> outLen, flat;
    uint64_t heads;  // bit j: output j is a merged run
    int total;
    uint32_t mergeBase;
  };

  // LocalReferenceCollection.append (localReference.ts:233-251) for a scour plan: the references of a
  // leaf appended onto its run head move to the head, offset by the run's length before the leaf.
  FMT_DEV void obRefsFromPlan(const ScourPlan& P, const Lane<uint32_t>* f) {
    if (obLive == 0 || P.heads == 0) return;
    Lane<uint32_t> srcU;
    Lane<int> dd;
    FOR_LANES(l) {
      LANE(srcU) = static_cast<uint32_t>(LANE(P.srcOf));
      LANE(dd) = LANE(P.dst) < 0 ? 0 : LANE(P.dst);
    }
    const Lane<uint32_t> headSrc = gather(srcU, dd);
    Lane<int> hs;
    Lane<bool> mv;
    FOR_LANES(l) {
      LANE(hs) = static_cast<int>(LANE(headSrc));
      const int d = LANE(P.dst);
      LANE(mv) = d >= 0 && ((P.heads >> d) & 1ull) != 0 && LANE(headSrc) != static_cast<uint32_t>(l);
    }
    const Lane<uint32_t> headId = gather(f[5], hs), headFlat = gather(P.flat, hs);
    uint64_t m = ballot(mv);
    while (m) {
      const int s = ctz64(m);
      m &= m - 1;
      obRefsMove(readlane(f[5], s), readlane(headId, s), 0, static_cast<int>(readlane(P.flat, s) - readlane(headFlat, s)));
    }
  }
  FMT_DEV bool scourPlan(const Lane<uint32_t>* f, const Lane<uint32_t>& lastCh, const Lane<int>& cntL, int nBlk, ScourPlan& P) {
    if (!scourDecideWide(f, lastCh, cntL, P)) scourDecideSerial(f, lastCh, cntL, nBlk, P);
    return scourText(f, P);
  }
  // The same plan once the merge area was compacted: a run that still does not fit is a capacity
  // failure (the half holds twice the document's text, so only an undersized arena gets here).
  FMT_DEV bool scourPlanAfterCompaction(const Lane<uint32_t>* f, const Lane<uint32_t>& lastCh, const Lane<int>& cntL, int nBlk,
                                        ScourPlan& P) {
    textFull = false;
    if (scourPlan(f, lastCh, cntL, nBlk, P)) return true;
    textFull = false;
    return fail(FMT_E_CAPACITY);
  }

  // The decisions lane-parallel. Leaf s appends onto its run iff it and leaf s-1 (same block) are
  // acked, not removed and non-empty, s-1 does not end in '\n', their props match, and (s's length
  // <= TextSegmentGranularity or its run so far is): the last condition is decided here only when
  // s is short; otherwise (returns false) the serial rule decides.
  FMT_DEV bool scourDecideWide(const Lane<uint32_t>* f, const Lane<uint32_t>& lastCh, const Lane<int>& cntL, ScourPlan& P) {
    Lane<uint32_t> ak, cls;
    Lane<bool> dropL;
    FOR_LANES(l) {
      const bool valid = (l & 7) < LANE(cntL);
      const int32_t ins = static_cast<int32_t>(LANE(f[1])), rm = static_cast<int32_t>(LANE(f[2]));
      LANE(ak) = (valid && rm == kNotRemoved && ins <= minSeq && LANE(f[0]) > 0 && !mMarker(LANE(f[7]))) ? 1u : 0u;  // acked, kept, non-empty text
      LANE(dropL) = valid && rm != kNotRemoved && rm <= minSeq;
      LANE(cls) = propClass(mProps(LANE(f[7])));
    }
    const Lane<uint32_t> akP = shflUp1(ak), lastP = shflUp1(lastCh), clsP = shflUp1(cls);
    Lane<bool> app, longApp;
    FOR_LANES(l) {
      const bool a = (l & 7) != 0 && LANE(ak) && LANE(akP) && LANE(lastP) != 10u && LANE(clsP) == LANE(cls);
      LANE(app) = a;
      LANE(longApp) = a && LANE(f[0]) > static_cast<uint32_t>(kGranularity);
    }
    if (ballot(longApp)) return false;
    // output index of each opening lane (kept, not appended), and the latest opener at/before each lane
    Lane<uint32_t> opens;
    FOR_LANES(l) { LANE(opens) = ((l & 7) < LANE(cntL) && !LANE(dropL) && !LANE(app)) ? 1u : 0u; }
    uint32_t total;
    const Lane<uint32_t> outIdx = waveExclusiveSum(opens, &total);
    Lane<int32_t> op;
    FOR_LANES(l) { LANE(op) = LANE(opens) ? static_cast<int32_t>(LANE(outIdx)) : -1; }
    const Lane<int32_t> lastOpen = waveExclusiveMax(op, -1);
    FOR_LANES(l) {
      LANE(P.dst) = LANE(opens) ? static_cast<int>(LANE(outIdx)) : (LANE(app) ? LANE(lastOpen) : -1);
      if (l < kMaxNodes * kMaxNodes) L->tmp[l] = 0u;
    }
    waveSync();
    FOR_LANES(l) {
      if (LANE(opens)) L->tmp[64 + LANE(outIdx)] = static_cast<uint32_t>(l);
      if (LANE(P.dst) >= 0) atomicAddLds(reinterpret_cast<int32_t*>(&L->tmp[LANE(P.dst)]), static_cast<int>(LANE(f[0])));
    }
    waveSync();
    FOR_LANES(l) {
      LANE(P.srcOf) = l < static_cast<int>(total) ? static_cast<int>(L->tmp[64 + l]) : 0;
      LANE(P.outLen) = l < static_cast<int>(total) ? L->tmp[l] : 0u;
    }
    waveSync();
    // output j is a merged run iff the lane after its opener appended
    Lane<uint32_t> appU;
    FOR_LANES(l) { LANE(appU) = LANE(app) ? 1u : 0u; }
    const Lane<uint32_t> nextApp = shflDown1(appU);
    const Lane<uint32_t> headJ = gather(nextApp, P.srcOf);
    Lane<bool> hb;
    FOR_LANES(l) { LANE(hb) = l < static_cast<int>(total) && LANE(headJ) != 0; }
    P.heads = ballot(hb);
    P.total = static_cast<int>(total);
    return true;
  }

  FMT_DEV void scourDecideSerial(const Lane<uint32_t>* f, const Lane<uint32_t>& lastCh, const Lane<int>& cntL, int nBlk, ScourPlan& P) {
    FOR_LANES(l) {
      LANE(P.dst) = -1;
      LANE(P.srcOf) = 0;
      LANE(P.outLen) = 0;
    }
    P.heads = 0;
    P.total = 0;
    for (int i = 0; i < nBlk; i++) {
      const int cnt = readlane(cntL, 8 * i);
      int prev = -1;
      uint32_t prevLen = 0, prevProps = 0, prevLast = 0;
      for (int k = 0; k < cnt; k++) {
        const int s = 8 * i + k;
        const uint32_t len = readlane(f[0], s);
        const int32_t ins = static_cast<int32_t>(readlane(f[1], s)), rm = static_cast<int32_t>(readlane(f[2], s));
        if (rm == kNotRemoved && ins <= minSeq) {
          const uint32_t props = mProps(readlane(f[7], s)), lc = readlane(lastCh, s);
          const bool marker = mMarker(readlane(f[7], s));  // Marker: canAppend false both ways
          const bool canAppend = prev >= 0 && len > 0 && !marker && prevLast != 10u &&
                                 (prevLen <= static_cast<uint32_t>(kGranularity) || len <= static_cast<uint32_t>(kGranularity)) &&
                                 propsMatch(prevProps, props);
          if (canAppend) {
            setLane(P.dst, s, prev);
            prevLen += len;
            prevLast = lc;
            setLane(P.outLen, prev, prevLen);
            P.heads |= 1ull << prev;
          } else {
            setLane(P.dst, s, P.total);
            setLane(P.srcOf, P.total, s);
            setLane(P.outLen, P.total, len);
            prev = len > 0 && !marker ? P.total : -1;
            prevLen = len;
            prevProps = props;
            prevLast = lc;
            P.total++;
          }
        } else {
          if (!(rm != kNotRemoved && rm <= minSeq)) {
            setLane(P.dst, s, P.total);
            setLane(P.srcOf, P.total, s);
            setLane(P.outLen, P.total, len);
            P.total++;
          }
          prev = -1;
        }
      }
    }
  }

  // The merge area's half is full: copy the text of every leaf in the tree that lives in it, in
  // document order, into the other half (zamboni appends copy whole runs, so a long run that keeps
  // absorbing short acked leaves would otherwise fill any fixed arena). Eight blocks per step.
  FMT_DEV bool compactText() {
    const uint64_t half = (S.textCap - S.textLen) / 2;
    const uint64_t lo = mergeLo == S.textLen ? S.textLen + half : S.textLen;
    uint64_t top = lo;
    prof[22]++;
    for (int k = 0; k < nGroups && status == FMT_OK; k++) {
      const uint32_t g = L->gOrder[k];
      const int cnt = static_cast<int>(L->gCount[g]);
      const uint32_t* sb = slotBlkPtr(g);
      for (int s0 = 0; s0 < cnt; s0 += 8) {
        Lane<uint32_t> mv, tx;
        Lane<size_t> idx;
        FOR_LANES(l) {
          const int s = s0 + l / 8, j = l % 8;
          uint32_t n = 0, t = 0;
          size_t i = 0;
          if (s < cnt) {
            const uint32_t b = rd(sb + s);
            if (j < static_cast<int>(rd(S.bCount + b))) {
              i = li(b, j);
              t = rd(S.lText + i);
              if (t >= mergeLo && t < mergeHi) n = rd(S.lLen + i);
            }
          }
          LANE(mv) = n;
          LANE(tx) = t;
          LANE(idx) = i;
        }
        uint32_t total;
        const Lane<uint32_t> ex = waveExclusiveSum(mv, &total);
        if (top + total > lo + half) {
          fail(FMT_E_CAPACITY);
          break;
        }
        FOR_LANES(l) {
          if (LANE(mv)) S.lText[LANE(idx)] = static_cast<uint32_t>(top + LANE(ex));
        }
        // unit t of this step comes from the last lane whose start ex <= t (gathers, as scourText)
        for (uint32_t base = 0; base < total; base += 64) {
          Lane<int> pos;
          FOR_LANES(l) { LANE(pos) = 0; }
          for (int step = 32; step >= 1; step >>= 1) {
            Lane<int> cand;
            FOR_LANES(l) { LANE(cand) = LANE(pos) + step; }
            const Lane<uint32_t> v = gather(ex, cand);
            FOR_LANES(l) {
              if (LANE(v) <= base + static_cast<uint32_t>(l)) LANE(pos) = LANE(cand);
            }
          }
          const Lane<uint32_t> st = gather(ex, pos), sx = gather(tx, pos);
          Lane<uint32_t> v;
          FOR_LANES(l) {
            const uint32_t t = base + l;
            LANE(v) = t < total ? textAt(LANE(sx) + (t - LANE(st))) : 0u;
          }
          FOR_LANES(l) {
            const uint32_t t = base + l;
            if (t < total) S.text[top + t] = static_cast<uint16_t>(LANE(v));
          }
        }
        waveSync();
        top += total;
      }
    }
    mergeLo = lo;
    mergeHi = lo + half;
    textTop = top;
    return status == FMT_OK;
  }

  // The merged runs' text, concatenated in lane order, into the merge area.
  FMT_DEV bool scourText(const Lane<uint32_t>* f, ScourPlan& P) {
    Lane<uint32_t> member;
    FOR_LANES(l) {
      const int d = LANE(P.dst);
      LANE(member) = (d >= 0 && ((P.heads >> d) & 1ull)) ? LANE(f[0]) : 0u;
    }
    uint32_t need = 0;
    P.flat = waveExclusiveSum(member, &need);
    P.mergeBase = static_cast<uint32_t>(textTop);
    if (!need) return true;
    if (textTop + need > mergeHi) {  // the caller compacts the merge area and plans again
      textFull = true;
      return false;
    }
    for (uint32_t base = 0; base < need; base += 64) {
      // source lane of unit t: the last lane whose flat start is <= t (binary search by gathers;
      // flat is non-decreasing over lanes)
      Lane<int> pos;
      FOR_LANES(l) { LANE(pos) = 0; }
      for (int step = 32; step >= 1; step >>= 1) {
        Lane<int> cand;
        FOR_LANES(l) { LANE(cand) = LANE(pos) + step; }
        const Lane<uint32_t> v = gather(P.flat, cand);
        FOR_LANES(l) {
          if (LANE(v) <= base + static_cast<uint32_t>(l)) LANE(pos) = LANE(cand);
        }
      }
      const Lane<uint32_t> st = gather(P.flat, pos), tx = gather(f[6], pos);
      Lane<uint32_t> v;
      FOR_LANES(l) {
        const uint32_t t = base + l;
        LANE(v) = t < need ? textAt(LANE(tx) + (t - LANE(st))) : 0u;
      }
      waveSync();
      FOR_LANES(l) {
        const uint32_t t = base + l;
        if (t < need) S.text[textTop + t] = static_cast<uint16_t>(LANE(v));
      }
      waveSync();
    }
    textTop += need;
    return true;
  }

  // Source lanes whose leaf left the tree (dropped, or appended onto its run head): for each, the
  // callback's leaf id gets parent = undefined (leafBlk kNone).
  FMT_DEV void unlinkGone(const ScourPlan& P, const Lane<uint32_t>* f, const Lane<int>& cntL) {
    Lane<uint32_t> srcU;
    Lane<int> dd;
    FOR_LANES(l) {
      LANE(srcU) = static_cast<uint32_t>(LANE(P.srcOf));
      LANE(dd) = LANE(P.dst) < 0 ? 0 : LANE(P.dst);
    }
    const Lane<uint32_t> headSrc = gather(srcU, dd);
    Lane<bool> gone;
    FOR_LANES(l) {
      const bool valid = (l & 7) < LANE(cntL);
      LANE(gone) = valid && (LANE(P.dst) < 0 || LANE(headSrc) != static_cast<uint32_t>(l));
      if (LANE(gone)) S.leafBlk[LANE(f[5])] = kNone;
    }
    if constexpr (Adj) {
      if (pmN > 0) {  // appended and unlinked leaves take their managers with them
        waveSync();
        for (uint64_t m = ballot(gone); m != 0 && status == FMT_OK; m &= m - 1) pmDropLeaf(readlane(f[5], ctz64(m)));
      }
    }
  }

  // scourNode over leaf block b: drops leaves removed at/below minSeq, appends acked same-props
  // appendable leaves onto the previous kept leaf. Returns the new leaf count.
  FMT_DEV int scourLeaves(uint32_t b, int cnt) {
    ProfScope ps_(prof[8]);
    if (cnt == 0) return 0;
    Lane<uint32_t> blk, f[8], lastCh;
    Lane<int> cntL;
    FOR_LANES(l) {
      LANE(blk) = b;
      LANE(cntL) = l < 8 ? cnt : 0;
    }
    loadOctets(blk, cntL, f, lastCh);
    ScourPlan P;
    if (!scourPlan(f, lastCh, cntL, 1, P)) {
      if (!textFull || !compactText()) return cnt;  // (compaction moved the octets' text: reload)
      loadOctets(blk, cntL, f, lastCh);
      if (!scourPlanAfterCompaction(f, lastCh, cntL, 1, P)) return cnt;
    }
    if (P.total == cnt) return cnt;  // nothing dropped or appended
    obRefsFromPlan(P, f);
    Lane<uint32_t> g8[8];
#pragma unroll
    for (int x = 0; x < 8; x++) g8[x] = gather(f[x], P.srcOf);
    const Lane<uint32_t> runSt = gather(P.flat, P.srcOf);
    waveSync();
    FOR_LANES(l) {
      if (l < P.total) {
        const size_t i = li(b, l);
        const bool merged = ((P.heads >> l) & 1ull) != 0;
        S.lLen[i] = merged ? LANE(P.outLen) : LANE(g8[0]);
        S.lIns[i] = static_cast<int32_t>(LANE(g8[1]));
        S.lRm[i] = static_cast<int32_t>(LANE(g8[2]));
        S.lMlo[i] = LANE(g8[3]);
        S.lMhi[i] = LANE(g8[4]);
        S.lId[i] = LANE(g8[5]);
        S.lText[i] = merged ? P.mergeBase + LANE(runSt) : LANE(g8[6]);
        S.lMeta[i] = LANE(g8[7]);
      }
    }
    unlinkGone(P, f, cntL);
    waveSync();
    st1(S.bCount + b, static_cast<uint32_t>(P.total));
    return P.total;
  }

  FMT_DEV static void setLane(Lane<uint32_t>& x, int idx, uint32_t v) {
    FOR_LANES(l) {
      if (l == idx) LANE(x) = v;
    }
  }
  FMT_DEV static void setLane(Lane<int>& x, int idx, int v) {
    FOR_LANES(l) {
      if (l == idx) LANE(x) = v;
    }
  }

  // packParent (zamboni.ts:83-139) at the leaf level: every child leaf block of p is scoured, the held
  // leaves are redistributed into min(7, total / 4) (>= 1) blocks. The first of p's old blocks are
  // reused for the new ones (block identity is not observable); the rest are freed and unlisted.
  // All children are scoured together: lane 8i + k holds leaf k of child i (≤ 7 x 7 leaves), so the
  // whole pack is a handful of dependent memory rounds instead of one scour per child.
  FMT_DEV void packLeafParent(uint32_t p) {
    ProfScope ps_(prof[9]);
    const int pc = static_cast<int>(ldu(S.bCount + p));
    Lane<uint32_t> chl, f[8], lastCh;
    Lane<int> cntL;
    FOR_LANES(l) { LANE(chl) = (l >> 3) < pc ? rd(S.bChild + (static_cast<size_t>(p) * 8 + (l >> 3))) : 0u; }
    FOR_LANES(l) { LANE(cntL) = (l >> 3) < pc ? static_cast<int>(rd(S.bCount + LANE(chl))) : 0; }
    loadOctets(chl, cntL, f, lastCh);
    ScourPlan P;
    if (!scourPlan(f, lastCh, cntL, pc, P)) {
      if (!textFull || !compactText()) return;
      loadOctets(chl, cntL, f, lastCh);
      if (!scourPlanAfterCompaction(f, lastCh, cntL, pc, P)) return;
    }
    obRefsFromPlan(P, f);
    const int total = P.total;
    const uint64_t heads = P.heads;
    const Lane<int>& srcOf = P.srcOf;
    const Lane<uint32_t>& outLen = P.outLen;
    const uint32_t mergeBase = P.mergeBase;
    // redistribution: nb blocks, the first `rem` of them one leaf longer
    int nb = 0;
    if (total > 0) {
      nb = total / (kMaxNodes / 2);
      if (nb > kMaxNodes - 1) nb = kMaxNodes - 1;
      if (nb < 1) nb = 1;
    }
    const int base = nb ? total / nb : 0;
    const int rem = nb ? total % nb : 0;
    // new block ids: the old blocks' ids (and slots) first, extra blocks listed after the previous one
    Lane<uint32_t> blkQ;
    FOR_LANES(l) { LANE(blkQ) = 0u; }
    uint32_t prevB = kNone;
    for (int q = 0; q < nb; q++) {
      uint32_t b;
      if (q < pc) {
        b = readlane(chl, 8 * q);
      } else {
        b = allocBlk(1);
        if (b == kNone) return;
        const uint32_t g = ldu(S.bGroup + prevB);
        st1(S.bGroup + b, g);
        st1(S.bCount + b, 0u);
        if (!slotInsert(g, static_cast<int>(ldu(S.bSlot + prevB)) + 1, b, 0)) return;
      }
      setLane(blkQ, q, b);
      prevB = b;
    }
    // output j -> block q, slot kq
    Lane<int> qOf, kOf;
    FOR_LANES(l) {
      const int j = l;
      const int big = rem * (base + 1);
      int q = 0, kq = 0;
      if (j < total) {
        if (j < big) {
          q = j / (base + 1);
          kq = j - q * (base + 1);
        } else {
          q = rem + (j - big) / base;
          kq = (j - big) - (q - rem) * base;
        }
      }
      LANE(qOf) = q;
      LANE(kOf) = kq;
    }
    Lane<uint32_t> g8[8];
#pragma unroll
    for (int x = 0; x < 8; x++) g8[x] = gather(f[x], srcOf);
    const Lane<uint32_t> blkJ = gather(blkQ, qOf), runSt = gather(P.flat, srcOf);
    FOR_LANES(l) {
      if (l < kMaxNodes) L->tmp[l] = 0u;
    }
    waveSync();
    FOR_LANES(l) {
      if (l < total) {
        const uint32_t b = LANE(blkJ);
        const size_t x = li(b, LANE(kOf));
        const bool merged = ((heads >> l) & 1ull) != 0;
        const uint32_t id = LANE(g8[5]);
        const uint32_t len = merged ? LANE(outLen) : LANE(g8[0]);
        S.lLen[x] = len;
        S.lIns[x] = static_cast<int32_t>(LANE(g8[1]));
        S.lRm[x] = static_cast<int32_t>(LANE(g8[2]));
        S.lMlo[x] = LANE(g8[3]);
        S.lMhi[x] = LANE(g8[4]);
        S.lId[x] = id;
        S.lText[x] = merged ? mergeBase + LANE(runSt) : LANE(g8[6]);
        S.lMeta[x] = LANE(g8[7]);
        S.leafBlk[id] = b;
        const uint32_t w = rd(S.winIdx + id);
        if (w != kNone) wRetag(w, b, rd(S.bGroup + b));
        const int c = (w == kNone && static_cast<int32_t>(LANE(g8[2])) == kNotRemoved) ? static_cast<int>(len) : 0;
        atomicAddLds(reinterpret_cast<int32_t*>(&L->tmp[LANE(qOf)]), c);
      }
    }
    waveSync();
    unlinkGone(P, f, cntL);
    waveSync();
    // block records and slot stable sums (lane q)
    FOR_LANES(l) {
      if (l < nb) {
        const uint32_t b = LANE(blkQ);
        const int cnt = l < rem ? base + 1 : base;
        S.bCount[b] = static_cast<uint32_t>(cnt);
        S.bLeaf[b] = 1u;
        S.bParent[b] = p;
        S.bScour[b] = -1;
        S.bChild[static_cast<size_t>(p) * 8 + l] = b;
        const uint32_t g = rd(S.bGroup + b), s0 = rd(S.bSlot + b);
        int32_t* sp = S.gSlotStable + static_cast<size_t>(g) * kSlotCap + s0;
        const int32_t stB = static_cast<int32_t>(L->tmp[l]);
        const int32_t old = rd(sp);
        *sp = stB;
        atomicAddLds(&L->gStable[g], stB - old);
        atomicAddLds(&L->cStable[L->gPos[g] >> 5], stB - old);
      }
    }
    waveSync();
    // unlist and free the old blocks past nb (consecutive slots, possibly in two groups)
    for (int i = nb; i < pc; i++) {
      const uint32_t b = readlane(chl, 8 * i);
      const uint32_t g = ldu(S.bGroup + b);
      const int s0 = static_cast<int>(ldu(S.bSlot + b));
      int run = 1;  // the following old blocks in the same group are the next slots
      while (i + run < pc && ldu(S.bGroup + readlane(chl, 8 * (i + run))) == g) run++;
      slotRemove(g, s0, run);
      for (int k = 0; k < run; k++) {
        const uint32_t ob = readlane(chl, 8 * (i + k));
        st1(S.bCount + ob, 0u);
        freeBlock(ob);
      }
      i += run - 1;
    }
    // (a parent left childless stays; packParent empties it, zamboni.ts:129-132. When that is the
    // root, no leaf block is listed any more, and the next insert makes the root a leaf block again
    // as in an empty document, insertText)
    st1(S.bCount + p, static_cast<uint32_t>(nb));
    if (lastBlk != kNone) updateLastBlk();
    invalidate();
  }

  FMT_DEV void updateLastBlk() {
    lastBlk = kNone;
    for (int k = nGroups - 1; k >= 0 && lastBlk == kNone; k--) {
      const uint32_t g = L->gOrder[k];
      const uint32_t cnt = L->gCount[g];
      if (cnt > 0) lastBlk = ldu(slotBlkPtr(g) + cnt - 1);
    }
  }

  // packParent above the leaf level: grandchildren blocks redistributed (no leaf moves). Lane 8i + k
  // holds grandchild k of child i; output j (document order) goes to block q, slot kq.
  FMT_DEV void packInterior(uint32_t p) {
    ProfScope ps_(prof[15]);
    const int pc = static_cast<int>(ldu(S.bCount + p));
    Lane<uint32_t> chl, gc, one;
    Lane<int> cc;
    FOR_LANES(l) { LANE(chl) = (l >> 3) < pc ? rd(S.bChild + (static_cast<size_t>(p) * 8 + (l >> 3))) : 0u; }
    FOR_LANES(l) { LANE(cc) = (l >> 3) < pc ? static_cast<int>(rd(S.bCount + LANE(chl))) : 0; }
    FOR_LANES(l) {
      const bool on = (l & 7) < LANE(cc);
      LANE(gc) = on ? rd(S.bChild + (static_cast<size_t>(LANE(chl)) * 8 + (l & 7))) : 0u;
      LANE(one) = on ? 1u : 0u;
    }
    // output index of each grandchild (document order), and the source lane of each output
    uint32_t nU;
    const Lane<uint32_t> outIdx = waveExclusiveSum(one, &nU);
    const int n = static_cast<int>(nU);
    FOR_LANES(l) {
      if (LANE(one)) L->tmp[LANE(outIdx)] = static_cast<uint32_t>(l);
    }
    waveSync();
    Lane<int> src;
    FOR_LANES(l) { LANE(src) = l < n ? static_cast<int>(L->tmp[l]) : 0; }
    waveSync();
    int nb = 0;
    if (n > 0) {
      nb = n / (kMaxNodes / 2);
      if (nb > kMaxNodes - 1) nb = kMaxNodes - 1;
      if (nb < 1) nb = 1;
    }
    const int base = nb ? n / nb : 0;
    const int rem = nb ? n % nb : 0;
    Lane<uint32_t> blkQ;
    FOR_LANES(l) { LANE(blkQ) = 0u; }
    for (int q = 0; q < nb; q++) {
      const uint32_t b = q < pc ? readlane(chl, 8 * q) : allocBlk(0);
      if (b == kNone) return;
      setLane(blkQ, q, b);
    }
    Lane<int> qOf, kOf;
    FOR_LANES(l) {
      const int big = rem * (base + 1);
      int q = 0, kq = 0;
      if (l < n) {
        if (l < big) {
          q = l / (base + 1);
          kq = l - q * (base + 1);
        } else {
          q = rem + (l - big) / base;
          kq = (l - big) - (q - rem) * base;
        }
      }
      LANE(qOf) = q;
      LANE(kOf) = kq;
    }
    const Lane<uint32_t> held = gather(gc, src), blkJ = gather(blkQ, qOf);
    waveSync();
    FOR_LANES(l) {
      if (l < n) {
        S.bChild[static_cast<size_t>(LANE(blkJ)) * 8 + LANE(kOf)] = LANE(held);
        S.bParent[LANE(held)] = LANE(blkJ);
      }
      if (l < nb) {
        const uint32_t b = LANE(blkQ);
        S.bLeaf[b] = 0u;
        S.bCount[b] = static_cast<uint32_t>(l < rem ? base + 1 : base);
        S.bScour[b] = -1;
        S.bChild[static_cast<size_t>(p) * 8 + l] = b;
        S.bParent[b] = p;
      }
    }
    waveSync();
    for (int i = nb; i < pc; i++) freeBlock(readlane(chl, 8 * i));
    st1(S.bCount + p, static_cast<uint32_t>(nb));
  }

  FMT_DEV void zamboni() {
    ProfScope ps_(prof[3]);
    for (int i = 0; i < 2; i++) {
      if (heapN == 0) break;
      if constexpr (Adj) {  // segmentToScour?.segment?.propertyManager?.updateMsn(minSeq) (zamboni.ts:44)
        if (pmN > 0) pmUpdateMsn(uni(L->heap[1].leafId), minSeq);
      }
      if (heapSeq(1) > minSeq) break;
      const HeapEnt e = heapGet();
      const uint32_t b = ldu(S.leafBlk + e.leafId);
      if (b == kNone) continue;  // unlinked or appended
      // (the block's flag, count and parent in one memory round trip; the scour changes no parent)
      const int32_t flag = ldi(S.bScour + b);
      const int oldCount = static_cast<int>(ldu(S.bCount + b));
      const uint32_t parent = ldu(S.bParent + b);
      if (flag == 0) continue;
      const int kept = scourLeaves(b, oldCount);
      if (status != FMT_OK) return;
      st1(S.bScour + b, 0);
      if (kept >= oldCount) continue;
      if (kept >= kMaxNodes / 2 || parent == kNone) continue;
      packLeafParent(parent);
      if (status != FMT_OK) return;
      uint32_t p = parent;
      for (;;) {
        const uint32_t pp = ldu(S.bParent + p);
        if (ldu(S.bCount + p) >= static_cast<uint32_t>(kMaxNodes / 2) || pp == kNone) break;
        p = pp;
        packInterior(p);
        if (status != FMT_OK) return;
      }
    }
  }

  // ------------------------------------------------------------------ load (f3)
  // reloadFromSegments (mergeTree.ts:751-800) of the header chunk: 7 leaves per block, layer by
  // layer; then SnapshotLoader.loadBody's appends of the body chunk (snapshotLoader.ts:277-309), each
  // through the inserting walk at the end — the last leaf's block, split 4 / 4 at MaxNodesInBlock
  // (mergeTree.ts:1946-1987) — whose resulting shape the runtime passes in in.shape. Every loaded
  // segment is stamped {UniversalSequenceNumber, NonCollabClient} (snapshotLoader.ts:180-186) and
  // keeps its spec's properties (a clone, as TextSegment.fromJSONObject does). Blocks are numbered
  // leaf level first; groups take kFill leaf blocks each.
  FMT_DEV uint32_t shapeLevels() const {
    if (in.shape != nullptr) return ldu(in.shape);
    uint32_t L = 1;
    for (uint32_t n = (in.nSegs + 6) / 7; n > 1; n = (n + 6) / 7) L++;
    return L;
  }
  FMT_DEV uint32_t shapeCount(uint32_t lvl) const {
    if (in.shape != nullptr) return ldu(in.shape + 1 + lvl);
    uint32_t n = (in.nSegs + 6) / 7;
    for (uint32_t l = 0; l < lvl; l++) n = (n + 6) / 7;
    return n;
  }
  // node q of a level (pairs: that level's first (start, count) record; below: the level's size)
  FMT_DEV void shapeNode(const uint32_t* pairs, uint32_t below, uint32_t q, uint32_t* st, uint32_t* c) const {
    if (pairs != nullptr) {
      *st = rd(pairs + 2 * static_cast<size_t>(q));
      *c = rd(pairs + 2 * static_cast<size_t>(q) + 1);
    } else {
      *st = 7 * q;
      *c = below - 7 * q < 7 ? below - 7 * q : 7;
    }
  }

  FMT_DEV void load() {
    ProfScope ps_(prof[5]);
    const uint32_t N = in.nSegs;
    if (N == 0) {  // an empty document: the root block alone, no leaf block listed yet (insertText)
      if (S.blockCap < 1) {
        fail(FMT_E_CAPACITY);
        return;
      }
      FOR_LANES(l) {
        if (l == 0) {
          S.bCount[0] = 0;
          S.bLeaf[0] = 0;
          S.bScour[0] = -1;
          S.bParent[0] = kNone;
        }
      }
      L->gOrder[0] = 0;
      L->gStable[0] = 0;
      L->gCount[0] = 0;
      L->gCorr[0] = 0;
      waveSync();
      nGroups = 1;
      root = 0;
      nextBlock = 1;
      nextId = 1;
      lastBlk = kNone;
      minSeq = in.snapMinSeq;
      curSeq = in.snapSeq;
      chunksRebuild();
      return;
    }
    const uint32_t nLv = shapeLevels();
    const uint32_t nLeafBlk = shapeCount(0);
    const uint32_t* pairs = in.shape != nullptr ? in.shape + 1 + nLv : nullptr;
    if (nLeafBlk > S.blockCap || N + 1 > S.idCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    // kFill leaf blocks per group, more when that would take over 3/4 of the groups (a body appended
    // 4 per block: 10M segments make 2.5M leaf blocks), leaving room for group splits either way
    uint32_t fill = kFill;
    if (nLeafBlk > static_cast<uint32_t>(kGroupCap / 4 * 3) * kFill)
      fill = (nLeafBlk + kGroupCap / 4 * 3 - 1) / (kGroupCap / 4 * 3);
    if (fill > static_cast<uint32_t>(kSlotCap) / 8 * 7) {
      fail(FMT_E_CAPACITY);
      return;
    }
    nGroups = static_cast<int>((nLeafBlk + fill - 1) / fill);
    if (nGroups > kGroupCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    // leaf blocks (lane = block): their leaves, count, stable sum, group slot
    Lane<bool> winL, wideL;  // some leaf stamped above minSeq; a writer past 63 (merge info)
    FOR_LANES(l) {
      LANE(winL) = false;
      LANE(wideL) = false;
    }
    for (uint32_t base = 0; base < nLeafBlk; base += 64) {
      FOR_LANES(l) {
        const uint32_t b = base + l;
        if (b < nLeafBlk) {
          uint32_t st, c;
          shapeNode(pairs, N, b, &st, &c);
          int sum = 0;
          for (uint32_t k = 0; k < c; k++) {
            const uint32_t j = st + k;
            const size_t i = static_cast<size_t>(b) * 8 + k;
            const fmt_mt_snapshot_seg sg = in.segs[j];
            const uint32_t len = sg.len & ~FMT_MT_SEG_MARKER;
            int32_t ins = 0, rm = kNotRemoved, client = in.initClient;
            uint64_t mask = 0;
            HiSet hs;
            hs.clear();
            if (in.info != nullptr) {  // merge info: the insert stamp, the remove stamps folded
              const fmt_mt_snapshot_info inf = in.info[j];
              ins = inf.ins_seq;
              client = inf.ins_client;
              for (uint32_t t = 0; t < inf.rm_count; t++) {
                const fmt_mt_stamp st = in.stamps[inf.rm_first + t];
                rm = st.seq < rm ? st.seq : rm;
                if (st.client < 0 || st.client > kMaxClient || (st.client > 63 && S.hiMask == nullptr)) LANE(wideL) = true;
                else if (st.client < 64) mask |= 1ull << st.client;
                else hs.add(st.client);
              }
              if (client > kMaxClient) LANE(wideL) = true;
            }
            if (S.hiMask != nullptr)
              for (int q = 0; q < kHiWords; q++) S.hiMask[kHiWords * static_cast<size_t>(j + 1) + q] = hs.w[q];
            S.lLen[i] = len;
            S.lIns[i] = ins;
            S.lRm[i] = rm;
            S.lMlo[i] = static_cast<uint32_t>(mask);
            S.lMhi[i] = static_cast<uint32_t>(mask >> 32);
            S.lId[i] = j + 1;
            S.lText[i] = sg.text;
            S.lMeta[i] = mkMeta(client, kNoProps) | ((sg.len & FMT_MT_SEG_MARKER) != 0 ? kMetaMarker : 0u);
            S.leafBlk[j + 1] = b;
            S.winIdx[j + 1] = kNone;
            // (a leaf stamped above minSeq is a window entry, added below; a removed one counts nowhere)
            const bool win = ins > in.snapMinSeq || (rm != kNotRemoved && rm > in.snapMinSeq);
            if (win) LANE(winL) = true;
            else if (rm == kNotRemoved) sum += static_cast<int>(len);
          }
          S.bCount[b] = c;
          S.bLeaf[b] = 1;
          S.bScour[b] = -1;
          S.bParent[b] = kNone;
          const uint32_t g = b / fill, s = b % fill;
          S.bGroup[b] = g;
          S.bSlot[b] = s;
          S.gSlotBlk[static_cast<size_t>(g) * kSlotCap + s] = b;
          S.gSlotStable[static_cast<size_t>(g) * kSlotCap + s] = sum;
        }
      }
    }
    nextId = N + 1;
    waveSync();
    if (ballot(wideL) != 0) {
      fail(FMT_E_CAPACITY);
      return;
    }
    const bool anyWin = ballot(winL) != 0;
    loadProps(nLeafBlk, pairs);
    if (status != FMT_OK) return;
    for (int g = 0; g < nGroups; g++) {
      const uint32_t lo = static_cast<uint32_t>(g) * fill, hi = lo + fill < nLeafBlk ? lo + fill : nLeafBlk;
      Lane<uint32_t> acc;
      FOR_LANES(l) { LANE(acc) = 0; }
      for (uint32_t base = lo; base < hi; base += 64) {
        FOR_LANES(l) {
          if (base + l < hi) LANE(acc) += static_cast<uint32_t>(rd(S.gSlotStable + (static_cast<size_t>(g) * kSlotCap + (base + l - lo))));
        }
      }
      uint32_t tot;
      waveExclusiveSum(acc, &tot);
      L->gOrder[g] = static_cast<uint16_t>(g);
      L->gStable[g] = static_cast<int32_t>(tot);
      L->gCount[g] = static_cast<uint16_t>(hi - lo);
      L->gCorr[g] = 0;
      waveSync();
    }
    // interior levels (lane = block)
    uint32_t lo = 0, next = nLeafBlk, below = nLeafBlk;
    const uint32_t* lvPairs = pairs;
    for (uint32_t lvl = 1; lvl < nLv; lvl++) {
      const uint32_t nb = shapeCount(lvl);
      if (lvPairs != nullptr) lvPairs += 2 * static_cast<size_t>(below);
      if (next + nb > S.blockCap) {
        fail(FMT_E_CAPACITY);
        return;
      }
      for (uint32_t base = 0; base < nb; base += 64) {
        FOR_LANES(l) {
          const uint32_t q = base + l;
          if (q < nb) {
            uint32_t st, c;
            shapeNode(lvPairs, below, q, &st, &c);
            const uint32_t id = next + q;
            S.bCount[id] = c;
            S.bLeaf[id] = 0;
            S.bScour[id] = -1;
            S.bParent[id] = kNone;
            for (uint32_t k = 0; k < c; k++) {
              S.bChild[static_cast<size_t>(id) * 8 + k] = lo + st + k;
              S.bParent[lo + st + k] = id;
            }
          }
        }
      }
      waveSync();
      lo = next;
      next += nb;
      below = nb;
    }
    root = static_cast<int>(lo);
    nextBlock = next;
    lastBlk = nLeafBlk - 1;
    chunksRebuild();
    minSeq = in.snapMinSeq;
    curSeq = in.snapSeq;
    if (anyWin) loadWindow(nLeafBlk);
    if (S.mkIds != nullptr) loadMarkers(nLeafBlk);
  }

  // The large tier's state at its checkpoint (huge_ckpt.h) in the paged layout: the same B+tree —
  // block ids kept, leaf blocks listed in document order kFill per group as a load lists them (a
  // large document has at most 1023 blocks: one group) —, the same leaf ids, the LRU heap in its array order, the free-block
  // list, the collab window and the live obliterates; its prop sets are interned again in their id
  // order and its text goes to the merge area. Returns the op (batch index) to resume at.
  FMT_DEV uint64_t loadFromLarge() {
    namespace K = fmt_ckpt;
    ProfScope ps_(prof[5]);
    const uint32_t* ck = in.ck;
    const uint64_t next = ldu(ck + K::kNextLo) | (static_cast<uint64_t>(ldu(ck + K::kNextHi)) << 32);
    const int n = static_cast<int>(ldu(ck + K::kN));
    const uint32_t nChars = ldu(ck + K::kNChars);
    const int nPropsL = static_cast<int>(ldu(ck + K::kNProps));
    const int heapL = static_cast<int>(ldu(ck + K::kHeapN));
    const uint32_t nextIdL = ldu(ck + K::kNextId);
    if (n <= 0 || static_cast<uint32_t>(K::kBlocks) > S.blockCap || nextIdL > S.idCap || heapL > kHeapCap ||
        nChars > (S.textCap - S.textLen) / 2) {
      fail(FMT_E_CAPACITY);
      return 0;
    }
    // prop sets, in id order (a wide set spans records: FMT_MT_PROPS_CONT), their new ids in sBlk
    uint32_t* pmap = L->sBlk;
    for (int p = 0; p < nPropsL && status == FMT_OK;) {
      const uint32_t cnt = ldu(&in.ckProps[p].n);
      if (cnt == FMT_MT_PROPS_CONT || cnt > static_cast<uint32_t>(FMT_MT_PROPS_KEYS_MAX) || p >= kSlotCap) {
        fail(FMT_E_DATA);
        return 0;
      }
      for (int c = 0; c * 64 < static_cast<int>(cnt); c++) {
        FOR_LANES(l) {
          const int k = c * 64 + l;
          if (k < static_cast<int>(cnt)) L->kvWork[k] = rd(&in.ckProps[p + k / FMT_MT_PROPS_MAX].kv[k % FMT_MT_PROPS_MAX]);
        }
      }
      waveSync();
      const uint32_t id = internWork(cnt);
      FOR_LANES(l) {
        if (l == 0) pmap[p] = id;
      }
      waveSync();
      p += cnt > FMT_MT_PROPS_MAX ? static_cast<int>((cnt + FMT_MT_PROPS_MAX - 1) / FMT_MT_PROPS_MAX) : 1;
    }
    if (status != FMT_OK) return 0;
    // (device memory starts arbitrary: the ids of leaves zamboni dropped before the checkpoint, which
    // remove-order entries and PropertiesManager records may still name, read as no leaf)
    FOR_LANES(l) {
      for (uint32_t k = static_cast<uint32_t>(l); k < nextIdL; k += 64) {
        S.leafBlk[k] = kNone;
        S.winIdx[k] = kNone;
      }
    }
    waveSync();
    minSeq = static_cast<int>(ldu(ck + K::kMinSeq));
    curSeq = static_cast<int>(ldu(ck + K::kCurSeq));
    // the text, into the merge area
    const uint64_t tb = textTop;
    FOR_LANES(l) {
      for (uint32_t t = static_cast<uint32_t>(l); t < nChars; t += 64) S.text[tb + t] = static_cast<uint16_t>(loadWg(in.ckChars + t));
    }
    textTop = tb + nChars;
    // every block's tree fields (free ones too: nothing reaches them)
    FOR_LANES(l) {
      for (int b = l; b < K::kBlocks; b += 64) {
        const uint32_t* o = ck + K::kBlk + K::kBlkWords * b;
        const uint32_t w0 = rd(o), par = rd(o + 1);
        const uint32_t cnt = w0 & 0xFFu;
        S.bCount[b] = cnt;
        S.bLeaf[b] = (w0 >> 8) & 0xFFu;
        S.bScour[b] = static_cast<int32_t>(static_cast<int8_t>((w0 >> 16) & 0xFFu));
        S.bParent[b] = par == K::kNoParent ? kNone : par;
        if (((w0 >> 8) & 0xFFu) == 0)
          for (uint32_t c = 0; c < cnt && c < 8; c++) S.bChild[static_cast<size_t>(b) * 8 + c] = rd(o + 2 + c);
      }
    }
    waveSync();
    // leaf blocks in document order (a run of leaves per block), kFill per group as a load fills
    // them: ordinal o is slot o % kFill of group o / kFill; the run's first leaf is parked in the
    // slot's stable-sum word until the leaves are placed
    const auto slotOf = [](uint32_t o) -> size_t { return static_cast<size_t>(o / kFill) * kSlotCap + o % kFill; };
    uint32_t nLeafBlk = 0;
    for (int base = 0; base < n; base += 64) {
      FOR_LANES(l) {
        const int j = base + l;
        if (j < n) {
          const uint32_t b = rd(ck + K::kLeafBlk + j);
          if (j == 0 || rd(ck + K::kLeafBlk + j - 1) != b) {
            const fmt_mt_leaf x = in.ckLeaves[j];
            const uint32_t o = static_cast<uint32_t>(x.block) | (static_cast<uint32_t>(x.pad & 0x7FFFu) << 16);
            S.gSlotBlk[slotOf(o)] = b;
            S.gSlotStable[slotOf(o)] = j;
          }
        }
      }
    }
    {
      const fmt_mt_leaf x = in.ckLeaves[n - 1];
      nLeafBlk = uni(static_cast<uint32_t>(x.block) | (static_cast<uint32_t>(x.pad & 0x7FFFu) << 16)) + 1u;
    }
    nGroups = static_cast<int>((nLeafBlk + kFill - 1) / kFill);
    if (nGroups > kGroupCap) {
      fail(FMT_E_CAPACITY);
      return 0;
    }
    waveSync();
    Lane<bool> winL;
    FOR_LANES(l) { LANE(winL) = false; }
    for (uint32_t base = 0; base < nLeafBlk; base += 64) {
      FOR_LANES(l) {
        const uint32_t o = base + l;
        if (o < nLeafBlk) {
          const uint32_t b = rd(S.gSlotBlk + slotOf(o));
          const int start = rd(S.gSlotStable + slotOf(o));
          const uint32_t c = rd(S.bCount + b);
          int sum = 0;
          for (uint32_t k = 0; k < c && k < 8; k++) {
            const int j = start + static_cast<int>(k);
            const fmt_mt_leaf x = in.ckLeaves[j];
            const uint32_t w4 = rd(ck + K::kLeafW4 + j);
            const uint32_t id = w4 & 0x7FFFFFu;
            const size_t i = li(b, static_cast<int>(k));
            const uint32_t props = x.props == 0xFFFFu ? kNoProps : L->sBlk[x.props];
            S.lLen[i] = x.len;
            S.lIns[i] = x.ins_seq;
            S.lRm[i] = x.rm_seq;
            S.lMlo[i] = static_cast<uint32_t>(x.rm_clients);
            S.lMhi[i] = static_cast<uint32_t>(x.rm_clients >> 32);
            S.lId[i] = id;
            S.lText[i] = static_cast<uint32_t>(tb + x.char_off);
            S.lMeta[i] = mkMeta(x.ins_client, props) | ((w4 & (1u << 23)) != 0 ? kMetaMarker : 0u);
            S.leafBlk[id] = b;
            S.winIdx[id] = kNone;
            if (S.hiMask != nullptr)
              for (int q = 0; q < kHiWords; q++) S.hiMask[kHiWords * static_cast<size_t>(id) + q] = 0u;
            const bool win = x.ins_seq > minSeq || (x.rm_seq != kNotRemoved && x.rm_seq > minSeq);
            if (win) LANE(winL) = true;
            else if (x.rm_seq == kNotRemoved) sum += static_cast<int>(x.len);
          }
          S.bGroup[b] = o / kFill;
          S.bSlot[b] = o % kFill;
          S.gSlotStable[slotOf(o)] = sum;
        }
      }
    }
    waveSync();
    for (int g = 0; g < nGroups; g++) {
      const uint32_t lo = static_cast<uint32_t>(g) * kFill, hi = lo + kFill < nLeafBlk ? lo + kFill : nLeafBlk;
      Lane<uint32_t> acc;
      FOR_LANES(l) { LANE(acc) = 0; }
      for (uint32_t base = lo; base < hi; base += 64) {
        FOR_LANES(l) {
          if (base + l < hi) LANE(acc) += static_cast<uint32_t>(rd(S.gSlotStable + slotOf(base + l)));
        }
      }
      uint32_t tot;
      waveExclusiveSum(acc, &tot);
      L->gOrder[g] = static_cast<uint16_t>(g);
      L->gStable[g] = static_cast<int32_t>(tot);
      L->gCount[g] = static_cast<uint16_t>(hi - lo);
      L->gCorr[g] = 0;
      waveSync();
    }
    chunksRebuild();
    root = static_cast<int>(ldu(ck + K::kRoot));
    nextBlock = K::kBlocks;
    nFree = static_cast<uint32_t>(ldu(ck + K::kNFree));
    FOR_LANES(l) {
      for (uint32_t k = static_cast<uint32_t>(l); k < nFree; k += 64) S.freeBlk[k] = rd(ck + K::kFree + k);
      for (int k = l; k <= heapL; k += 64) {
        HeapEnt e;
        e.maxSeq = static_cast<int32_t>(rd(ck + K::kHeapOff + 2 * k));
        e.leafId = rd(ck + K::kHeapOff + 2 * k + 1);
        L->heap[k] = e;
      }
    }
    waveSync();
    heapN = heapL;
    lastBlk = ldu(S.gSlotBlk + slotOf(nLeafBlk - 1));
    nextId = nextIdL;
    cuN = ldu(ck + K::kCuN);
    // the window: leaves stamped above minSeq, in document order
    if (ballot(winL) != 0) {
      for (uint32_t base = 0; base < nLeafBlk * 8 && status == FMT_OK; base += 64) {
        Lane<bool> w;
        FOR_LANES(l) {
          const uint32_t x = base + l, o = x >> 3, k = x & 7;
          bool v = false;
          if (o < nLeafBlk) {
            const uint32_t b = rd(S.gSlotBlk + slotOf(o));
            if (k < rd(S.bCount + b)) {
              const size_t i = li(b, static_cast<int>(k));
              const int32_t ins = rd(S.lIns + i), rm = rd(S.lRm + i);
              v = ins > minSeq || (rm != kNotRemoved && rm > minSeq);
            }
          }
          LANE(w) = v;
        }
        for (uint64_t m = ballot(w); m != 0 && status == FMT_OK; m &= m - 1) {
          const uint32_t x = base + static_cast<uint32_t>(ctz64(m));
          const uint32_t b = ldu(S.gSlotBlk + slotOf(x >> 3));
          const Leaf y = getLeaf(b, static_cast<int>(x & 7));
          const uint64_t mask = static_cast<uint64_t>(y.mlo) | (static_cast<uint64_t>(y.mhi) << 32);
          // window meta: insert client | first remover << 8 | more removers << 16 (the large tier keeps
          // the set, not which remover came first: the lowest id stands in; the passes read neither)
          const uint32_t first = mask != 0 ? static_cast<uint32_t>(__builtin_ctzll(mask)) : 0u;
          const uint32_t meta = (static_cast<uint32_t>(mClient(y.meta)) & 0xFFu) | (first << 8) |
                                (__builtin_popcountll(mask) > 1 ? 1u << 16 : 0u);
          winAdd(y.id, y.ins, y.rm, y.len, meta, (x >> 3) / kFill, b, y.mlo, y.mhi);
        }
      }
    }
    // live obliterates (same slots)
    const uint32_t obc = ldu(ck + K::kObCounts);
    const uint64_t used = ldu(ck + K::kObUsedLo) | (static_cast<uint64_t>(ldu(ck + K::kObUsedHi)) << 32);
    if (used != 0 || obc != 0) {
      if (S.obCap < static_cast<uint32_t>(K::kObSlots)) {
        fail(FMT_E_CAPACITY);
        return 0;
      }
      obSeqN = static_cast<int>(obc & 0xFFFFu);
      obStartN = static_cast<int>(obc >> 16);
      obLive = __builtin_popcountll(used);
      obSlotsHi = K::kObSlots;
      FOR_LANES(l) {
        const int k = l;  // (kObSlots == 64: one slot per lane)
        const uint32_t* o = ck + K::kOb + 6 * k;
        uint32_t* e = S.obRec + 6 * static_cast<size_t>(k);
        e[kObStartId] = rd(o);
        e[kObEndId] = rd(o + 1);
        e[kObStartOff] = rd(o + 2);
        e[kObEndOff] = rd(o + 3);
        e[kObSeq] = rd(o + 4);
        e[kObClient] = rd(o + 5);
        S.obUsed[k] = static_cast<uint32_t>((used >> k) & 1u);
        S.obSeq[k] = rd(ck + K::kObSeq + k);
        S.obStart[k] = rd(ck + K::kObStart + k);
      }
      waveSync();
    }
    // relative positions: every Marker leaf still in the tree joins the marker list (in document
    // order; the engine's pick among markers with one id does not depend on the list's order, and a
    // marker zamboni unlinked before the checkpoint is one the list skips anyway)
    if (S.mkIds != nullptr) {
      for (uint32_t base = 0; base < nLeafBlk * 8 && status == FMT_OK; base += 64) {
        Lane<bool> mk;
        Lane<uint32_t> ids;
        FOR_LANES(l) {
          const uint32_t x = base + l, o = x >> 3, k = x & 7;
          bool v = false;
          uint32_t id = 0;
          if (o < nLeafBlk) {
            const uint32_t b = rd(S.gSlotBlk + slotOf(o));
            if (k < rd(S.bCount + b)) {
              const size_t i = li(b, static_cast<int>(k));
              v = mMarker(rd(S.lMeta + i));
              id = rd(S.lId + i);
            }
          }
          LANE(mk) = v;
          LANE(ids) = id;
        }
        for (uint64_t m = ballot(mk); m != 0 && status == FMT_OK; m &= m - 1) markerAdd(readlane(ids, ctz64(m)));
      }
    }
    // annotate-adjust: the PropertiesManager records stay in the document's slab (same layout), and
    // its computed numbers with their count in theirs
    if constexpr (Adj) {
      pmN = static_cast<int>(ldu(ck + K::kPmN));
      if (pmN < 0 || pmN > pmCap()) {
        fail(FMT_E_DATA);
        return 0;
      }
    }
    // remove order: the large tier's entries stay in the document's slab with their leaf ids (ids are
    // kept across the checkpoint; one of a leaf zamboni dropped before it is in no block: GONE at output)
    if constexpr (Rm) {
      rmN = ldu(ck + K::kRmN);
      if (rmN > 0 && (in.rmOrder == nullptr || rmN > in.rmOrderCap)) {
        fail(FMT_E_DATA);
        return 0;
      }
    }
    invalidate();
    return next;
  }

  // Loaded Markers join the marker list (relative positions), in document order.
  FMT_DEV void loadMarkers(uint32_t nLeafBlk) {
    for (uint32_t base = 0; base < nLeafBlk * 8 && status == FMT_OK; base += 64) {
      Lane<bool> mk;
      Lane<uint32_t> ids;
      FOR_LANES(l) {
        const uint32_t x = base + l, b = x >> 3, k = x & 7;
        bool v = false;
        uint32_t id = 0;
        if (b < nLeafBlk && k < rd(S.bCount + b)) {
          const size_t i = li(b, static_cast<int>(k));
          v = mMarker(rd(S.lMeta + i));
          id = rd(S.lId + i);
        }
        LANE(mk) = v;
        LANE(ids) = id;
      }
      for (uint64_t m = ballot(mk); m != 0 && status == FMT_OK; m &= m - 1) markerAdd(readlane(ids, ctz64(m)));
    }
  }

  // Loaded leaves whose merge info is above minSeq enter the window table (their lengths differ
  // between perspectives), in document order; the stable sums above left them out.
  FMT_DEV void loadWindow(uint32_t nLeafBlk) {
    for (uint32_t base = 0; base < nLeafBlk * 8 && status == FMT_OK; base += 64) {
      Lane<bool> w;
      FOR_LANES(l) {
        const uint32_t x = base + l, b = x >> 3, k = x & 7;
        bool v = false;
        if (b < nLeafBlk && k < rd(S.bCount + b)) {
          const size_t i = li(b, static_cast<int>(k));
          const int32_t ins = rd(S.lIns + i), rm = rd(S.lRm + i);
          v = ins > minSeq || (rm != kNotRemoved && rm > minSeq);
        }
        LANE(w) = v;
      }
      for (uint64_t m = ballot(w); m != 0 && status == FMT_OK; m &= m - 1) {
        const uint32_t x = base + static_cast<uint32_t>(ctz64(m)), b = x >> 3;
        const Leaf y = getLeaf(b, static_cast<int>(x & 7));
        const uint64_t mask = static_cast<uint64_t>(y.mlo) | (static_cast<uint64_t>(y.mhi) << 32);
        // window meta: insert client | first remover << 8 | more removers << 16 (as removeLeaf leaves it)
        uint32_t first = 0;
        if (y.rm != kNotRemoved) {
          const fmt_mt_snapshot_info inf = in.info[y.id - 1];
          for (uint32_t t = 0; t < inf.rm_count; t++) {
            const fmt_mt_stamp st = in.stamps[inf.rm_first + t];
            if (st.seq == y.rm) {
              first = static_cast<uint32_t>(st.client);
              break;
            }
          }
        }
        const uint32_t meta = (static_cast<uint32_t>(mClient(y.meta)) & 0xFFu) | (first << 8) |
                              (__builtin_popcountll(mask) + hiCount(y.id) > 1 ? 1u << 16 : 0u);
        winAdd(y.id, y.ins, y.rm, y.len, meta, ldu(S.bGroup + b), b, y.mlo, y.mhi);
      }
    }
    invalidate();
  }

  // The loaded segments' properties (IJSONTextSegment.props: the segment's properties are a clone of
  // them, textSegment.ts:41-52): interned once per distinct props op, 64 segments a step.
  FMT_DEV void loadProps(uint32_t nLeafBlk, const uint32_t* pairs) {
    if (!in.segProps) return;
    uint32_t lastOp = kNone, lastSet = kNoProps;
    for (uint32_t base = 0; base < nLeafBlk * 8; base += 64) {
      Lane<uint32_t> op;
      FOR_LANES(l) {
        const uint32_t x = base + l, b = x >> 3, k = x & 7;
        uint32_t v = FMT_MT_NO_PROPS;
        if (b < nLeafBlk) {
          uint32_t st, c;
          shapeNode(pairs, in.nSegs, b, &st, &c);
          if (k < c) v = in.segs[st + k].props;
        }
        LANE(op) = v;
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
        if (id != lastOp) {
          lastSet = applyProps(kNoProps, id);
          if (status != FMT_OK) return;
          lastOp = id;
        }
        FOR_LANES(l) {
          if (LANE(op) == id) {
            const uint32_t x = base + l;
            const size_t i = li(x >> 3, static_cast<int>(x & 7));
            S.lMeta[i] = (rd(S.lMeta + i) & (0xFFu | kMetaMarker)) | (lastSet << 8);  // (the insert client stays)
            LANE(op) = FMT_MT_NO_PROPS;
          }
        }
      }
    }
    waveSync();
  }

  // ------------------------------------------------------------------ driver
  FMT_DEV Lane<uint32_t> fetchOp(uint64_t i) const {
    Lane<uint32_t> x;
    if (i < in.end) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(in.ops + i);
      FOR_LANES(l) { LANE(x) = l < 8 ? p[l] : 0u; }
    } else {
      FOR_LANES(l) { LANE(x) = 0u; }
    }
    return x;
  }
  FMT_DEV static fmt_mt_op decodeOp(const Lane<uint32_t>& rec) {
    fmt_mt_op op;
    op.seq = static_cast<int32_t>(readlane(rec, 0));
    op.ref_seq = static_cast<int32_t>(readlane(rec, 1));
    op.min_seq = static_cast<int32_t>(readlane(rec, 2));
    op.pos1 = static_cast<int32_t>(readlane(rec, 3));
    op.pos2 = static_cast<int32_t>(readlane(rec, 4));
    op.payload = readlane(rec, 5);
    const uint32_t lct = readlane(rec, 6);
    op.len = static_cast<uint16_t>(lct & 0xFFFF);
    op.client = static_cast<uint8_t>((lct >> 16) & 0xFF);
    op.type = static_cast<uint8_t>(lct >> 24);
    op.flags = readlane(rec, 7);
    return op;
  }

  FMT_DEV void replay(uint64_t first) {
    ProfScope ps_(prof[0]);
    Lane<uint32_t> rec0 = fetchOp(first), rec1 = fetchOp(first + 1);
    for (uint64_t i = first; i < in.end; i++) {
      fmt_mt_op op = decodeOp(rec0);
      rec0 = rec1;
      rec1 = fetchOp(i + 2);
      invalidate();
#ifdef FMT_HUGE_CHECK
      checkPerspective(op.seq, op.ref_seq, op.client);
#endif
      cuRec = (op.flags & FMT_MT_F_CATCHUP) != 0 && in.catchup != nullptr && S.cuIds != nullptr;
      cuIdN = 0;
      if constexpr (Rm) rmRec = (op.flags & FMT_MT_F_RMORDER) != 0 && in.rmOrder != nullptr && S.rmIds != nullptr;
      rmKind = op.type == FMT_MT_REMOVE ? FMT_MT_RM_SET : FMT_MT_RM_SLICE;
      rmHitN = 0;
      opIdx = static_cast<uint32_t>(i - in.begin);
      const bool loader = (op.flags & FMT_MT_F_LOADSEG) != 0;
      if (loader) {
        if (op.type != FMT_MT_INSERT || (op.client > kMaxClient && op.client != FMT_MT_CLIENT_NONCOLLAB)) fail(FMT_E_UNSUPPORTED);
        else loadBodySegment(op);
      } else if (op.client > kMaxClient || (op.client > 63 && S.hiMask == nullptr)) fail(FMT_E_UNSUPPORTED);
      else if ((op.flags & (FMT_MT_F_REL1 | FMT_MT_F_REL2)) != 0 && !resolveRelative(op)) {
      } else if (op.type == FMT_MT_INSERT) insertText(op);
      else if (op.type == FMT_MT_REMOVE || op.type == FMT_MT_ANNOTATE) {
        if (op.type == FMT_MT_ANNOTATE && op.payload >= in.nPropsOps) fail(FMT_E_DATA);
        else applyRange(op);
      } else if (op.type == FMT_MT_OBLITERATE || op.type == FMT_MT_OBLITERATE_SIDED) {
        applyObliterate(op);
      } else {
        fail(FMT_E_UNSUPPORTED);
      }
      if (((op.flags & FMT_MT_F_RMORDER) != 0 && !rmRec) || ((op.flags & FMT_MT_F_CATCHUP) != 0 && !cuRec)) fail(FMT_E_UNSUPPORTED);
      if (cuRec && status == FMT_OK) recordCatchup(op.type == FMT_MT_OBLITERATE_SIDED ? FMT_MT_OBLITERATE : op.type);
      if constexpr (Rm) {
        if ((rmPendN > 0 || rmHitN > 0) && status == FMT_OK) rmFlush(op.client, op.seq);
      }
      cuRec = rmRec = false;
      // (a loader segment updates no collab window; a batch of them is no GROUP message)
      const bool lastMember =
          !loader && (i + 1 == in.end || (readlane(rec0, 7) & (FMT_MT_F_GROUP_CONT | FMT_MT_F_LOADSEG)) != FMT_MT_F_GROUP_CONT);
      for (int z = 0; z < 2 && status == FMT_OK; z++) {
        if (z == 1) {
          if (!lastMember) break;
          if (curSeq > op.seq || op.min_seq > op.seq || minSeq > op.min_seq) {
            fail(FMT_E_DATA);
            break;
          }
          curSeq = op.seq;
          if (op.min_seq <= minSeq) break;
          minSeq = op.min_seq;
          graduate();
          if (obSeqN > 0) obSetMinSeq();
        }
        zamboni();
      }
#ifdef FMT_HUGE_CHECK
      if (status == FMT_OK) checkInvariants(op.seq);
#endif
      if (status != FMT_OK) {
        failSeq = op.seq;
        break;
      }
    }
  }

#ifdef FMT_HUGE_CHECK
  // Host emulation only: the perspective lengths of groups and slots equal the leaves' sums.
  void checkPerspective(int seq, int r, int c) {
    groupCorrections(r, c);
    for (int k = 0; k < nGroups; k++) {
      const uint32_t g = L->gOrder[k];
      long brute = 0;
      slotLengths(g, r, c);
      for (uint32_t s = 0; s < L->gCount[g]; s++) {
        const uint32_t b = S.gSlotBlk[static_cast<size_t>(g) * kSlotCap + s];
        long bl = 0;
        for (uint32_t j = 0; j < S.bCount[b]; j++) {
          const size_t i = li(b, static_cast<int>(j));
          bl += visAny(S.lLen[i], S.lIns[i], S.lRm[i], S.lMlo[i], S.lMhi[i], mClient(S.lMeta[i]), r, c, S.lId[i]);
        }
        if (bl != L->sLen[s]) {
          std::fprintf(stderr, "seq %d: slot %u of group %u (block %u) view %ld, index %d (stable %d) r=%d c=%d minSeq=%d\n", seq, s, g, b, bl,
                       L->sLen[s], S.gSlotStable[static_cast<size_t>(g) * kSlotCap + s], r, c, minSeq);
          for (uint32_t j = 0; j < S.bCount[b]; j++) {
            const size_t i = li(b, static_cast<int>(j));
            const uint32_t w = S.winIdx[S.lId[i]];
            std::fprintf(stderr, "  leaf id %u len %u ins %d rm %d mask %x:%x ic %d vis %d win %d", S.lId[i], S.lLen[i], S.lIns[i], S.lRm[i],
                         S.lMhi[i], S.lMlo[i], mClient(S.lMeta[i]),
                         visAny(S.lLen[i], S.lIns[i], S.lRm[i], S.lMlo[i], S.lMhi[i], mClient(S.lMeta[i]), r, c, S.lId[i]), w == kNone ? -1 : (int)w);
            if (w != kNone) std::fprintf(stderr, " | w ins %d rm %d len %u meta %x grp %u blk %u", S.wRec[4 * w], S.wRec[4 * w + 1], S.wRec[4 * w + 2], S.wRec[4 * w + 3] & kWMetaMask, S.wRec[4 * w + 3] >> kWGroupShift, S.wBlk[w]);
            std::fprintf(stderr, "\n");
          }
          fail(FMT_E_DATA);
          return;
        }
        brute += bl;
      }
      if (brute != L->gStable[g] + L->gCorr[g]) {
        std::fprintf(stderr, "seq %d: group %u view %ld, index %d + %d\n", seq, g, brute, L->gStable[g], L->gCorr[g]);
        fail(FMT_E_DATA);
        return;
      }
    }
    invalidate();
  }

  // Host emulation only (tests/emu/huge_emu.cpp): every index structure agrees with the leaves.
  void checkInvariants(int seq) {
    auto bad = [&](const char* what, long a, long b) {
      std::fprintf(stderr, "seq %d: %s (%ld vs %ld)\n", seq, what, a, b);
      fail(FMT_E_DATA);
    };
    long nw = 0;
    for (int k = 0; k < nGroups; k++) {
      const uint32_t g = L->gOrder[k];
      long sum = 0;
      for (uint32_t s = 0; s < L->gCount[g]; s++) {
        const uint32_t b = S.gSlotBlk[static_cast<size_t>(g) * kSlotCap + s];
        if (S.bGroup[b] != g || S.bSlot[b] != s) return bad("block group/slot", b, s);
        long st = 0;
        for (uint32_t j = 0; j < S.bCount[b]; j++) {
          const size_t i = li(b, static_cast<int>(j));
          const uint32_t id = S.lId[i];
          if (S.leafBlk[id] != b) return bad("leafBlk", id, b);
          const bool shouldWin = S.lIns[i] > minSeq || (S.lRm[i] != kNotRemoved && S.lRm[i] > minSeq);
          const uint32_t w = S.winIdx[id];
          if (shouldWin != (w != kNone)) return bad("window membership", id, shouldWin);
          if (w != kNone) {
            nw++;
            if (S.wLeaf[w] != id || S.wBlk[w] != b || (S.wRec[4 * w + 3] >> kWGroupShift) != g || S.wRec[4 * w + 2] != S.lLen[i] ||
                static_cast<int32_t>(S.wRec[4 * w]) != S.lIns[i] || static_cast<int32_t>(S.wRec[4 * w + 1]) != S.lRm[i] ||
                S.wMask[2 * w] != S.lMlo[i] || S.wMask[2 * w + 1] != S.lMhi[i])
              return bad("window entry", id, w);
          } else if (S.lRm[i] == kNotRemoved) {
            st += S.lLen[i];
          }
        }
        if (st != S.gSlotStable[static_cast<size_t>(g) * kSlotCap + s]) return bad("slot stable", st, S.gSlotStable[static_cast<size_t>(g) * kSlotCap + s]);
        sum += st;
      }
      if (sum != L->gStable[g]) return bad("group stable", sum, L->gStable[g]);
    }
    if (nw != static_cast<long>(nWin)) bad("window count", nw, nWin);
    for (uint32_t w = 0; w < nWin && w < kWinLds; w++) {  // the LDS mirror of the window table
      for (int f = 0; f < 4; f++)
        if (L->wRecL[4 * w + f] != S.wRec[4 * w + f]) return bad("window mirror", w, f);
      if (L->wMaskL[2 * w] != S.wMask[2 * w] || L->wMaskL[2 * w + 1] != S.wMask[2 * w + 1]) return bad("window mirror mask", w, 0);
    }
    for (int c = 0; c * 32 < nGroups; c++) {  // the group scan's chunk sums and positions
      long sum = 0;
      for (int k = c * 32; k < c * 32 + 32 && k < nGroups; k++) {
        if (L->gPos[L->gOrder[k]] != k) return bad("group position", L->gOrder[k], k);
        sum += L->gStable[L->gOrder[k]];
      }
      if (sum != L->cStable[c]) return bad("chunk stable", sum, L->cStable[c]);
    }
  }
#endif

  // Converged state in document order: fmt_mt_leaf records (block = leaf-block ordinal, low 16 bits,
  // pad = high 16 bits), the text of every leaf (tombstones included), the prop sets, the header.
  // Eight leaf blocks per wave step: lane l handles slot l % 8 of block l / 8.
  // getAtSeq(properties, minSeq) (segmentPropertiesManager.ts:328-344) of every leaf with a manager,
  // as mt_engine.h: its current properties with each pending key set to the value its changes at or
  // below minSeq leave (null: deleted; a key the properties lack goes last, in the manager's key
  // order), interned; outLegacy[output index] already holds every leaf's current set.
  FMT_DEV void pmLegacyProps(uint16_t* outLegacy) {
    const uint32_t* R = pmBase();
    for (;;) {
      if (status != FMT_OK) return;
      int h = -1;  // the next head of a leaf not handled yet (a handled head's seq word gets bit 31)
      for (int base = 0; base < pmN && h < 0; base += 64) {
        Lane<bool> p;
        FOR_LANES(l) {
          const int i = base + l;
          LANE(p) = i < pmN && rd(R + 4 * i) != 0u && (rd(R + 4 * i + 1) & 0x10000u) == 0u &&
                    (rd(R + 4 * i + 2) & 0x80000000u) == 0u;
        }
        const uint64_t m = ballot(p);
        if (m != 0) h = base + ctz64(m);
      }
      if (h < 0) return;
      const uint32_t leaf = pmWord(h, 0);
      int j = -1;
      uint32_t cnt = 0;
      if (ldu(S.leafBlk + leaf) != kNone) {
        uint32_t b;
        int k;
        locate(leaf, &b, &k);
        if (k >= 0) {
          j = static_cast<int>(ldu(S.outIdx + leaf));
          cnt = loadWork(mProps(ldu(S.lMeta + li(b, k))));
        }
      }
      for (int g = h; g >= 0 && status == FMT_OK; g = pmFind(leaf, 0u, 0x10000u, g + 1)) {
        pmSet(g, 2, 0x80000000u);  // (done: a head's seq word is otherwise unused)
        if (j < 0) continue;
        const uint32_t key = pmWord(g, 1) & 0xFFFFu;
        uint32_t v = pmWord(g, 3);
        for (int c = pmFind(leaf, key | 0x10000u, 0x1FFFFu, g + 1); c >= 0; c = pmFind(leaf, key | 0x10000u, 0x1FFFFu, c + 1)) {
          if (static_cast<int>(pmWord(c, 2)) > minSeq) break;  // (a key's changes are in seq order)
          v = pmWord(c, 3);
        }
        cnt = workSet(cnt, key, v);
      }
      if (j >= 0 && status == FMT_OK) {
        const uint32_t id = internWork(cnt);
        if (status != FMT_OK) return;
        st1(outLegacy + j, static_cast<uint16_t>(id));
      }
    }
  }

  FMT_DEV void writeOutputs(fmt_mt_doc_result* hdr, fmt_mt_leaf* outLeaves, uint64_t capLeaves, uint16_t* outChars,
                            uint64_t capChars, fmt_mt_propset* outProps, uint16_t* outLegacy = nullptr,
                            uint64_t* outHi = nullptr) {
    uint64_t nLeaves = 0, nChars = 0, visible = 0;
    uint32_t nBlocks = 0;
    for (int k = 0; k < nGroups && status == FMT_OK; k++) {
      const uint32_t g = L->gOrder[k];
      const int cnt = static_cast<int>(L->gCount[g]);
      const uint32_t* sb = slotBlkPtr(g);
      for (int s0 = 0; s0 < cnt; s0 += 8) {
        Lane<uint32_t> valid, len, vlen, blockStart;
        Lane<size_t> idx;
        FOR_LANES(l) {
          const int s = s0 + l / 8, j = l % 8;
          uint32_t v = 0, ln = 0, vl = 0, bs = 0;
          size_t i = 0;
          if (s < cnt) {
            const uint32_t b = rd(sb + s);
            const uint32_t bc = rd(S.bCount + b);
            bs = (j == 0 && bc > 0) ? 1u : 0u;
            if (j < static_cast<int>(bc)) {
              i = li(b, j);
              v = 1;
              ln = rd(S.lLen + i);
              vl = rd(S.lRm + i) == kNotRemoved ? ln : 0u;
            }
          }
          LANE(valid) = v;
          LANE(len) = ln;
          LANE(vlen) = vl;
          LANE(blockStart) = bs;
          LANE(idx) = i;
        }
        uint32_t tv, tl, tvl, tb;
        const Lane<uint32_t> ev = waveExclusiveSum(valid, &tv);
        const Lane<uint32_t> el = waveExclusiveSum(len, &tl);
        const Lane<uint32_t> eb = waveExclusiveSum(blockStart, &tb);
        waveExclusiveSum(vlen, &tvl);
        if (nLeaves + tv > capLeaves || nChars + tl > capChars) {
          fail(FMT_E_CAPACITY);
          break;
        }
        FOR_LANES(l) {
          if (LANE(valid)) {
            const size_t i = LANE(idx);
            const uint64_t o = nLeaves + LANE(ev);
            const uint64_t co = nChars + LANE(el);
            const uint32_t blk = nBlocks + LANE(eb) - ((l % 8) != 0 ? 1u : 0u);  // this block's ordinal
            fmt_mt_leaf x;
            x.ins_seq = rd(S.lIns + i);
            x.rm_seq = rd(S.lRm + i);
            x.rm_clients = static_cast<uint64_t>(rd(S.lMlo + i)) | (static_cast<uint64_t>(rd(S.lMhi + i)) << 32);
            if (outHi != nullptr) {  // (remove clients 64..253: kHiOutWords 64-bit words per leaf)
              const size_t q = kHiWords * static_cast<size_t>(rd(S.lId + i));
              for (int k = 0; k < kHiOutWords; k++)
                outHi[kHiOutWords * o + k] = static_cast<uint64_t>(rd(S.hiMask + q + 2 * k)) |
                                             (static_cast<uint64_t>(rd(S.hiMask + q + 2 * k + 1)) << 32);
            }
            x.char_off = static_cast<uint32_t>(co);
            x.len = LANE(len);
            const uint32_t m = rd(S.lMeta + i);
            x.ins_client = static_cast<int16_t>(mClient(m));
            x.props = static_cast<uint16_t>(mProps(m));
            x.block = static_cast<uint16_t>(blk & 0xFFFFu);
            x.pad = static_cast<uint16_t>((blk >> 16) | (mMarker(m) ? FMT_MT_LEAF_MARKER : 0u));
            outLeaves[o] = x;
            if constexpr (Rm) {
              if (S.rmIds != nullptr) S.rmIds[rd(S.lId + i)] = static_cast<uint32_t>(o);  // (remove-order entries)
            }
            if constexpr (Adj) {
              if (outLegacy != nullptr) {  // (annotate-adjust: getAtSeq below)
                S.outIdx[rd(S.lId + i)] = static_cast<uint32_t>(o);
                outLegacy[o] = static_cast<uint16_t>(mProps(m));
              }
            }
            const uint32_t t = rd(S.lText + i);
            for (uint32_t c = 0; c < LANE(len); c++) outChars[co + c] = static_cast<uint16_t>(textAt(t + c));
          }
        }
        nLeaves += tv;
        nChars += tl;
        visible += tvl;
        nBlocks += tb;
      }
    }
    if constexpr (Adj) {
      if (outLegacy != nullptr && S.outIdx != nullptr && status == FMT_OK) {
        waveSync();
        if (pmN > 0) pmLegacyProps(outLegacy);
        if (status != FMT_OK) {
          // the legacy getAtSeq view did not fit the prop-set table: the replay state stands, only
          // its legacy summary is unavailable (kLegacyUnavailable: summaryRunsKernel and
          // fmt_mt_fetch_legacy_props report FMT_E_CAPACITY for this document)
          status = FMT_OK;
          for (uint64_t base = 0; base < nLeaves; base += 64) {
            FOR_LANES(l) {
              if (base + l < nLeaves) outLegacy[base + l] = fmt_mt::kLegacyUnavailable;
            }
          }
          waveSync();
        }
      }
    }
    FOR_LANES(l) {
      for (int p = l; p < nProps; p += 64) {
        fmt_mt_propset ps;
        ps.n = rd(S.props + p * kPropWords);
        for (int k = 0; k < FMT_MT_PROPS_MAX; k++) ps.kv[k] = rd(S.props + p * kPropWords + 1 + k);
        outProps[p] = ps;
      }
    }
    waveSync();
    // remove-order entries: leaf id -> output index, FMT_MT_LEAF_GONE once zamboni dropped the leaf
    for (uint32_t base = 0; Rm && status == FMT_OK && S.rmIds != nullptr && base < rmN; base += 64) {
      FOR_LANES(l) {
        const uint32_t k = base + l;
        if (k < rmN) {
          uint32_t* e = reinterpret_cast<uint32_t*>(in.rmOrder + k);
          const uint32_t id = rd(e);
          e[0] = rd(S.leafBlk + id) == kNone ? FMT_MT_LEAF_GONE : rd(S.rmIds + id);
        }
      }
    }
    const int d = status == FMT_OK ? depth() : 0;
    FOR_LANES(l) {
      if (l == 0) {
        fmt_mt_doc_result h;
        h.status = status;
        h.fail_seq = failSeq;
        h.cur_seq = curSeq;
        h.min_seq = minSeq;
        h.n_leaves = static_cast<uint32_t>(nLeaves);
        h.n_chars = static_cast<uint32_t>(nChars);
        h.n_props = static_cast<uint32_t>(nProps);
        h.n_blocks = nBlocks;
        h.depth = static_cast<uint32_t>(d);
        h.visible_len = static_cast<uint32_t>(visible);
        h.n_catchup = cuN;
        h.n_rm_order = rmN;
        *hdr = h;
      }
    }
  }

  FMT_DEV int depth() const {
    int d = 1;
    for (uint32_t b = static_cast<uint32_t>(root); ldu(S.bLeaf + b) == 0 && ldu(S.bCount + b) > 0; b = childAt(b, 0)) d++;
    return d;
  }

  FMT_DEV void run(const HugeInputs& inputs) {
    in = inputs;
    heapN = 0;
    nWin = 0;
    cuN = cuIdN = 0;
    cuRec = false;
    rmN = rmHitN = 0;
    rmRec = false;
    rmPendN = 0;
    mkN = 0;
    pmN = 0;
    nFree = 0;
    nProps = 0;
    if (inputs.nPropsOps > 0 || inputs.segProps != 0) {  // (empty prop-set hash tables)
      FOR_LANES(l) {
        for (uint32_t k = static_cast<uint32_t>(l); k < 2 * kPropHash; k += 64) S.pHead[k] = 0u;
      }
      waveSync();
    }
    textTop = S.textLen;
    mergeLo = S.textLen;
    mergeHi = S.textLen + (S.textCap - S.textLen) / 2;
    status = FMT_OK;
    obLive = obSeqN = obStartN = obSlotsHi = 0;
    for (uint32_t base = 0; base < S.obCap; base += 64) {
      FOR_LANES(l) {
        if (base + l < S.obCap) S.obUsed[base + l] = 0u;
      }
    }
    waveSync();
    uint64_t first = in.begin;
    if (in.ck != nullptr) {
      first = loadFromLarge();  // (an index into the batch's ops, as in.begin)
      prof[24] = first - in.begin;
    } else {
      load();
    }
    if (status == FMT_OK) replay(first);
  }
};

using HugeDoc = HugeDocT<false>;

}  // namespace fmt_huge
