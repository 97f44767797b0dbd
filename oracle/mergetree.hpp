// oracle/mergetree.hpp — TEST INFRASTRUCTURE ONLY (parity oracle for the merge-tree replay path).
//
// A CPU restatement of the reference merge-tree for a client that never submits ops while
// collaborating (an observer: every sequenced message is remote), plus the detached local-op path
// used to build the SharedString snapshot fixtures. Every function cites the reference code it
// follows (paths relative to /root/reference/packages/dds/merge-tree/src unless stated).
//
// What is restated exactly (it decides the segmentation that summaries expose):
//   - the 8-slot B+tree, its 4/4 split and root growth (mergeTree.ts:1846-1987, 1313-1320)
//   - the inserting walk with breakTie / theUnfinishedNode (mergeTree.ts:1811-1972)
//   - ensureIntervalBoundary splits (mergeTree.ts:1768-1808), nodeMap (mergeTree.ts:2961-3020)
//   - remove / annotate stamping (mergeTree.ts:2009-2081, 2292-2383; stamps.ts:144-158)
//   - the zamboni LRU heap, scour and packParent (zamboni.ts:33-213; core-utils heap.ts:54-182)
//   - raw-property LWW (segmentPropertiesManager.ts:188-238) and the legacy summary
//     (snapshotlegacy.ts:74-262, snapshotChunks.ts:85-204)
// What is replaced: PartialSequenceLengths is only an index; block lengths under a remote
// perspective are evaluated directly as the sum of leaf lengths, which is exactly the invariant the
// reference's strict checker asserts (partialLengths.ts:1189-1240).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../include/fmt.h"

namespace orc {

constexpr int kUnassignedSeq = -1;  // constants.ts:21
constexpr int kTreeMaintSeq = -2;   // constants.ts:26
constexpr int kLocalClientId = -1;  // constants.ts:31
constexpr int kNonCollabClient = -2;  // constants.ts:36
constexpr int kMaxNodesInBlock = 8;   // mergeTreeNodes.ts:248
constexpr int kTextGranularity = 256;  // textSegment.ts:21
constexpr int kUndefinedLen = -1;      // "length undefined": removed at or below minSeq
constexpr int kZamboniMax = 2;         // zamboni.ts:25

struct DataError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
// A local op whose range is invalid in the local view (client.ts:797-810 "RangeOutOfBounds",
// thrown with usageError: true): FMT_E_USAGE.
struct UsageError : DataError {
  using DataError::DataError;
};

// A remove stamp's kind (stamps.ts RemoveOperationStamp.type): 0 = "setRemove" (markRangeRemoved),
// 1 = "sliceRemove" (obliterate, incl. obliterate-on-insert). Insert stamps leave it 0.
// localSeq (stamps.ts:47): defined (> 0) iff the stamp is a local op pending its ack (seq -1).
struct Stamp {
  int seq;
  int client;
  int kind = 0;
  int localSeq = 0;
};

// stamps.ts:87-121 (lessThan / greaterThan / lte): acked before unacked; unacked by localSeq.
inline bool stampGreater(const Stamp& a, const Stamp& b) {
  if (a.seq == kUnassignedSeq) return b.seq != kUnassignedSeq || a.localSeq > b.localSeq;
  if (b.seq == kUnassignedSeq) return false;
  return a.seq > b.seq;
}
inline bool stampLess(const Stamp& a, const Stamp& b) {
  if (a.seq == kUnassignedSeq) return b.seq == kUnassignedSeq && a.localSeq < b.localSeq;
  if (b.seq == kUnassignedSeq) return true;
  return a.seq < b.seq;
}
inline bool stampLte(const Stamp& a, const Stamp& b) { return !stampGreater(a, b); }
inline bool isLocal(const Stamp& a) { return a.seq == kUnassignedSeq; }  // stamps.ts:125-127

// perspective.ts:80-93 (PriorPerspective), :103-118 (LocalReconnectingPerspective) and :174-184
// (LocalDefaultPerspective). mergeTreeNodes.ts:325-327 seqLTE excludes UnassignedSequenceNumber.
struct Perspective {
  bool everything;  // LocalDefaultPerspective: every op has occurred
  int refSeq;
  int client;
  int localSeq = 0;  // > 0: LocalReconnectingPerspective(refSeq, client, localSeq)
  bool hasOccurred(const Stamp& s) const {
    if (everything) return true;
    const bool viaRefSeq = s.seq != kUnassignedSeq && s.seq <= refSeq;
    if (localSeq > 0) return viaRefSeq || (s.localSeq > 0 && s.localSeq <= localSeq);
    return viaRefSeq || s.client == client;
  }
};

// A property map with JS insertion order (keys interned as ids by the host driver).
struct PropMap {
  bool defined = false;  // `seg.properties` is undefined until the first annotate
  std::vector<std::pair<uint16_t, uint16_t>> kv;  // (key id, value id), insertion order
};
bool matchProperties(const PropMap& a, const PropMap& b);  // properties.ts:32-61

// PropertiesManager (segmentPropertiesManager.ts:140-345) of a segment, for an observer: per key (in
// the order its entry was created, a JS Map) the msnConsensus value and the remote changes not yet
// folded into it. Only adjusts make the list grow: a raw change folds straight into msnConsensus
// while the list is empty (:213-221). Values are value ids (0 = null).
struct PropChangeRec {
  int seq;
  bool adjust;
  uint16_t value;  // raw value id
  int32_t row;     // adjust row
};
struct PropPending {
  uint16_t key;
  uint16_t msnConsensus;
  std::vector<PropChangeRec> remote;
  std::vector<PropChangeRec> local;  // the local client's unacked changes (segmentPropertiesManager.ts:209-211)
};
struct PropManager {
  std::vector<PropPending> changes;
};

struct Block;
struct Node {
  explicit Node(bool leaf) : isLeaf(leaf) {}
  Block* parent = nullptr;
  int index = 0;
  const bool isLeaf;
};

struct LRef;
struct Seg;
// mergeTreeNodes.ts:234-240 SegmentGroup: the segments one local op touched, pending its ack. `type`
// and `payload` are the op's (FMT_MT_* and its props-op id / insert props-op id + 1, what ackOp and
// regeneratePendingOp read from the op they are handed); previousProps (annotate: the keys' values
// before the op, null = 0) parallel to segments.
struct SegmentGroup {
  std::vector<Seg*> segments;
  bool hasPrevious = false;
  std::vector<std::vector<std::pair<uint16_t, uint16_t>>> previousProps;
  int localSeq = 0;
  int refSeq = 0;
  uint32_t type = 0;
  int32_t payload = 0;
  int32_t pos2 = 0;      // (insert: props-op id + 1 of the original op's seg props)
  uint32_t flags = 0;    // (insert: FMT_MT_F_MARKER)
  // the refSeq its op was submitted at (SharedSegmentSequence.inFlightRefSeqs, sequence.ts:468-499,
  // 666; a resubmitted op keeps its original one, :782-790)
  int inflightRef = 0;
};

struct Seg : Node {
  Seg() : Node(true) {}
  std::u16string text;  // a Marker's one unit is its refType
  bool marker = false;  // Marker segment (mergeTreeNodes.ts:495-564): cachedLength 1, never appends
  Stamp ins{0, 0};
  std::vector<Stamp> removes;  // sorted by stamps.compare (spliceIntoList)
  PropMap props;
  std::unique_ptr<PropManager> pm;  // segment.propertyManager (created by the first annotate)
  std::vector<LRef*> refs;     // local references on this segment (localReference.ts)
  std::vector<SegmentGroup*> groups;  // segmentGroups (segmentGroupCollection.ts): pending local ops
  int len() const { return static_cast<int>(text.size()); }
  bool removed() const { return !removes.empty(); }
};

// A StayOnRemove local reference (localReference.ts): stays on its segment when the segment is
// removed, follows the text across splitAt (LocalReferenceCollection.split) and zamboni appends
// (LocalReferenceCollection.append), and keeps pointing at a segment zamboni unlinks.
struct ObliterateInfo;
struct LRef {
  Seg* seg = nullptr;  // nullptr once removed (removeLocalReferencePosition)
  int offset = 0;
  ObliterateInfo* ob = nullptr;
};

// mergeTree.ts ObliterateInfo: the obliterated range's endpoint references and the op's stamp.
struct ObliterateInfo {
  LRef start, end;
  Stamp stamp;
  int refSeq = 0;
};

// Length index of a block for remote perspectives (what PartialSequenceLengths is to the
// reference, partialLengths.ts:180-230, 973-1005; only an index: its value is Σ leaf lengths,
// partialLengths.ts:1189-1240). A leaf w contributes len·[ins ≤ r ∧ rm1 > r ∧ c ∉ R] +
// len·[ins > r ∧ ic = c ∧ rm1 > r ∧ c ∉ R] to PriorPerspective(r, c), r ≥ minSeq. The first term is
// len·([ins ≤ r] − [max(ins, rm1) ≤ r]): a +len event at ins and a −len event at max(ins, rm1),
// kept in seq order with prefix sums (events at or below the fold point are constants in k0);
// the second and the c ∈ R correction come from the few leaves each client inserted or removed in
// the collaboration window, evaluated from the leaves themselves.
struct BlockIdx {
  int64_t k0 = 0;                          // folded events
  std::vector<int> evSeq;                  // event seqs, non-decreasing
  std::vector<int64_t> evCum;              // prefix sums of the event deltas
  std::vector<std::pair<int, std::vector<struct Seg*>>> clients;  // client → leaves (inserted by it or
                                                                  // removed by it, in the window)
};

struct Block : Node {
  Block() : Node(false) {}
  int childCount = 0;
  Node* children[kMaxNodesInBlock] = {};
  int needsScour = -1;  // -1 undefined, 0 false, 1 true (mergeTreeNodes.ts MergeBlock.needsScour)
  std::unique_ptr<BlockIdx> idx;  // remote-perspective length index (MergeTree::enableIndex)
  bool idxDirty = true;           // rebuilt from the children before its next use
};

// core-utils/src/heap.ts:54-182 with LRUSegmentComparer (mergeTree.ts:144-147). Ported as an
// algorithm because ties between equal maxSeq are resolved by its exact sift order.
class LruHeap {
 public:
  struct Entry {
    Seg* seg;
    int maxSeq;
  };
  LruHeap() { L_.push_back({nullptr, -2}); }
  int count() const { return static_cast<int>(L_.size()) - 1; }
  const Entry& peek() const { return L_[1]; }
  Entry get();
  void add(Entry e);

 private:
  bool gtParent(int k) const { return k > 1 && L_[k >> 1].maxSeq - L_[k].maxSeq > 0; }
  void fixup(int k);
  void fixdown(int k);
  std::vector<Entry> L_;
};

struct Summary {
  std::string header;
  std::string body;  // empty when no body chunk
};

class MergeTree {
 public:
  MergeTree();

  // --- collaboration window (mergeTreeNodes.ts:598-696) ---
  int clientId = kLocalClientId;
  bool collaborating = false;
  int minSeq = 0;
  int currentSeq = 0;

  // A legacy summary chunk's segment spec: text and, when the spec has "props", its properties.
  struct LoadedSeg {
    std::u16string text;
    bool marker = false;  // {"marker": {"refType"}}: text = the refType unit
    bool hasProps = false;
    std::vector<std::pair<uint16_t, uint16_t>> props;
    Stamp ins{0, kNonCollabClient};  // SnapshotV1 merge info (specToSegment, snapshotLoader.ts:105-175)
    std::vector<Stamp> removes;      // in stamp order
  };
  // SnapshotLoader (snapshotLoader.ts:59-348): header segments rebuild the tree
  // (reloadFromSegments, mergeTree.ts:751-800), collaboration starts at (minSeq, seq), body segments
  // are appended through insertSegments with stamp {UniversalSequenceNumber, NonCollabClient}.
  void loadSnapshot(const std::vector<LoadedSeg>& header, const std::vector<LoadedSeg>& body,
                    int minSeqArg, int seqArg);

  // Detached local ops (not collaborating): stamp {seq 0, client -1}, local perspective.
  void insertLocal(int pos, const std::u16string& text);
  void annotateLocal(int start, int end, const std::vector<std::pair<uint16_t, uint16_t>>& props);
  void removeLocal(int start, int end);
  // client.ts:1700-1727 → mergeTree.ts:803-810
  void startCollaboration(int localClientId, int minSeqArg, int currentSeqArg);

  // One member op of a sequenced remote message (client.ts:1291-1327).
  void applyRemote(const fmt_mt_op& op, const uint16_t* arena, const uint32_t* propsOff,
                   const uint32_t* propsKv);
  // client.ts:1381-1391 updateSeqNumbers, after the last member of a message.
  void updateSeqNumbers(int min, int seq);

  // --- f4: the local client (a Client whose own ops apply before they are
  // sequenced). Its short id is clientId (startCollaboration); every other client is remote. ---
  int localSeq = 0;  // collabWindow.localSeq (mergeTreeNodes.ts:685-695 mintNextLocalOperationStamp)
  // insertSegmentLocal / removeRangeLocal / annotateRangeLocal (client.ts:273-355): the op's positions
  // are in the local view (LocalDefaultPerspective), its stamp {UnassignedSequenceNumber, clientId,
  // ++localSeq}, its segments a new pending SegmentGroup (mergeTree.ts:1410-1447).
  void applyLocal(const fmt_mt_op& op, const uint16_t* arena, const uint32_t* propsOff, const uint32_t* propsKv);
  // The local client's own op came back sequenced (client.ts:1367-1368 ackPendingSegment →
  // mergeTree.ts:1325-1408 ackOp): the oldest pending group takes the stamp {seq, clientId}.
  void ackOp(const fmt_mt_op& op, const uint32_t* propsOff, const uint32_t* propsKv);
  // client.ts:554 → mergeTree.ts:2388-2514: undo the newest pending op.
  void rollback(const fmt_mt_op& op);
  // Reconnect (client.ts:1452-1542 regeneratePendingOp, called for every pending op in order): the
  // segments are normalized once (mergeTree.ts:2602-2818), then every pending group becomes one new
  // op per segment (resetPendingDeltaToOps, client.ts:1160-1289) at positions from
  // LocalReconnectingPerspective(currentSeq, clientId, group localSeq). The new ops are appended to
  // *out (fmt_mt_op records: seq = localSeq, ref_seq = currentSeq, insert text appended to *text
  // with payload = its offset there); squash is false (IDeltaHandler.reSubmit's default path).
  void regeneratePending(std::vector<fmt_mt_op>* out, std::u16string* text);
  size_t pendingGroups() const { return pendingSegments_.size(); }
  // the oldest in-flight op's refSeq (none: INT_MAX): SharedSegmentSequence bounds every window update
  // by it (getMinInFlightRefSeq, sequence.ts:499 → client.ts:1374-1378)
  int minInflightRef() const { return pendingSegments_.empty() ? 0x7FFFFFFF : pendingSegments_.front()->inflightRef; }
  // REGEN events applied without an explicit output (orc_mt_apply_ops) collect their ops here
  std::vector<fmt_mt_op> regenOps;
  std::u16string regenText;

  // Maintain the per-block remote length index (BlockIdx) instead of summing leaf lengths over the
  // subtree on every query: O(log window + the querying client's window leaves) per block, which
  // makes a 10M-segment document (BASELINE config 5, T3) replayable. Results are identical; only
  // valid for an observer replay (every stamp acknowledged). Call before loading or applying ops.
  void enableIndex() { indexed_ = true; }

  // Legacy catch-up ops (sequence.ts:971-1006): while set, each applied op appends the ranges of
  // the sequenceDelta event it raises, merged the way createOpsFromDelta merges them
  // (sequence.ts:395-452), tagged with catchupOp.
  std::vector<fmt_mt_catchup_range>* catchupOut = nullptr;
  uint32_t catchupOp = 0;
  // Annotate-adjust (IMergeTreeAnnotateAdjustMsg, ops.ts:187-222): the batch's adjust rows, the
  // number of each host value id (NaN: not a number), the host's numbers with their ids, and this
  // document's computed numbers (value ids FMT_MT_VALUE_COMPUTED + index, first-computed order).
  const fmt_mt_adjust* adjusts = nullptr;
  // SnapshotV1 merge info of the batch (FMT_MT_F_LOADSEG body segments name their row)
  const fmt_mt_snapshot_info* snapInfo = nullptr;
  const fmt_mt_stamp* snapStamps = nullptr;
  uint64_t nSnapInfo = 0;
  uint32_t nAdjusts = 0;
  const double* valueNum = nullptr;
  uint32_t nValues = 0;
  const std::vector<std::pair<double, uint32_t>>* hostNumbers = nullptr;  // sorted by number
  std::vector<std::pair<double, uint32_t>> docNumbers;  // hostNumbers' storage with document-local value ids
  std::vector<double> numbers;
  // One change of an annotate op, in opToChanges order (segmentPropertiesManager.ts:86-95): a raw
  // value id (0 = null), or an adjust row (adjust >= 0).
  struct PropChange {
    uint16_t key;
    uint16_t value;
    int32_t adjust;
  };
  // Legacy relative positions (FMT_MT_F_REL1/REL2): the batch's table and the "markerId" key id.
  const fmt_mt_relpos* relpos = nullptr;
  uint32_t nRelpos = 0;
  uint32_t markerIdKey = FMT_MT_NO_MARKER;

  // Readouts.
  // getMarkerFromId (mergeTree.ts:1450-1453) finds a marker with this markerId value id (not removed).
  bool markerPresent(uint32_t id) const {
    const fmt_mt_relpos rp{id, 0, 0, 0};
    return posFromRelativePos(rp, Perspective{true, 0, 0}) >= 0;
  }
  std::u16string getText() const;     // MergeTreeTextHelper.ts:28-87 (local perspective)
  int getLocalLength() const;
  void collectLeaves(std::vector<const Seg*>& out, std::vector<int>& blockOfLeaf,
                     int* nLeafBlocks, int* depth) const;
  // snapshotlegacy.ts:195-262 extractSync + :126-193 emit (header/body blob contents).
  // (not const: getAtSeq may look up computed numbers, and the answer never differs from a replay's)
  Summary summarize(const std::vector<std::string>& keyNames,
                    const std::vector<std::string>& valueJson, int chunkSize = 10000);

 private:
  struct InsertCtx {
    bool isInsert;
    Seg* candidate;
  };
  struct InsertResult {
    Block* remainder;
    bool hadChanges;
  };

  Block* makeBlock(int childCount);
  Seg* makeSeg();
  static void assignChild(Block* parent, Node* child, int index);

  Perspective localPerspective() const { return {true, 0x7fffffff, clientId}; }
  // f4 internals
  std::vector<std::unique_ptr<SegmentGroup>> groupPool_;
  std::vector<SegmentGroup*> pendingSegments_;  // mergeTree.ts:657 pendingSegments (front = oldest)
  bool lastNormSet_ = false;                    // client.ts:1414 lastNormalization
  int lastNormRefSeq_ = 0, lastNormLocalSeq_ = 0;
  SegmentGroup* addToPendingList(Seg* seg, SegmentGroup* group, int localSeqArg,
                                 const std::vector<std::pair<uint16_t, uint16_t>>* previousProps = nullptr);
  int findRollbackPosition(const Seg* seg) const;  // mergeTree.ts:2519-2536
  void normalizeSegmentsOnRebase();                // mergeTree.ts:2734-2766
  void normalizeAdjacentSegments(std::vector<Seg*>& range);  // mergeTree.ts:2613-2712
  // segmentPropertiesManager.ts:140-173 rollbackProperties (collaborating)
  void rollbackProperties(Seg* s, const std::vector<std::pair<uint16_t, uint16_t>>& props);
  static bool isRemovedAndAcked(const Seg* s) { return s->removed() && !isLocal(s->removes[0]); }
  bool minSeqHasOccurred(const Stamp& s) const {
    return (s.seq != kUnassignedSeq && s.seq <= minSeq) || s.client == kNonCollabClient;
  }
  static bool isPresent(const Seg* s, const Perspective& p);
  int leafLength(const Seg* s, const Perspective& p) const;      // mergeTree.ts:720-736
  int localBlockLength(const Block* b) const;                    // blockUpdate cachedLength
  int remoteBlockLength(const Block* b, const Perspective& p) const;  // const_cast inside when indexed
  int nodeLength(const Node* n, const Perspective& p) const;     // mergeTree.ts:1116-1145
  // mergeTree.ts:1123-1135: a local perspective that sees every local edit reads the cached lengths
  bool isLocalPerspective(const Perspective& p) const {
    return (!collaborating || clientId == p.client) &&
           (p.localSeq == 0 || (p.localSeq == localSeq && p.refSeq >= currentSeq));
  }

  void insertingWalk(int pos, const Perspective& p, Stamp stamp, InsertCtx& ctx);
  InsertResult insertRecursive(Block* block, int pos, const Perspective& p, Stamp stamp,
                               InsertCtx& ctx, bool isLastBlock);
  bool breakTie(int pos, const Node* node, const Stamp& stamp) const;
  bool hasLeafAfter(const Block* block) const;  // forwardExcursion existence (blockInsert)
  Block* split(Block* node);
  void updateRoot(Block* splitNode);
  Seg* splitAt(Seg* seg, int pos);
  void ensureIntervalBoundary(int pos, const Perspective& p);

  int getPosition(const Node* node) const;  // mergeTree.ts:835-856, local perspective
  int getPosition(const Node* node, const Perspective& p) const;
  // mergeTree.ts:1462-1483 posFromRelativePos (-1 when the id names no marker)
  int posFromRelativePos(const fmt_mt_relpos& rp, const Perspective& p) const;
  // idToMarker (mergeTree.ts:675): marker id (value id of its "markerId" property) → marker; set when
  // a marker is inserted (:1614-1620) or loaded (blockUpdate, :2833-2841), deleted when zamboni
  // unlinks a marker (unlinkMarker, :738-743; zamboni.ts:202-204)
  std::map<uint32_t, Seg*> idToMarker;
  void registerMarker(Seg* s);
  void unlinkMarker(const Seg* s);
  void recordDelta(uint32_t type, const std::vector<Seg*>& deltaSegs);

  template <class F>
  void nodeMap(const Perspective& p, int start, int end, F&& leafFn) const;

  void insertSegments(int pos, Seg* seg, const Perspective& p, Stamp stamp, bool boundary = true);
  void markRangeRemoved(int start, int end, const Perspective& p, Stamp stamp);
  // obliterateRange (mergeTree.ts:2262-2290) → obliterateRangeSided (:2083-2260) with
  // start {pos1, Before} and end {pos2 - 1, After}.
  // obliterateRangeSided: start/end InteriorSequencePlaces {pos, before?} (mergeTree.ts:2083-2260)
  void obliterateRange(int startPos, bool startBefore, int endPos, bool endBefore, const Perspective& p, Stamp stamp);
  // The obliterate branch of blockInsert (mergeTree.ts:1642-1746) for a new remote segment.
  void obliterateOnInsert(Seg* seg, const Perspective& p, Stamp stamp);
  // Obliterates (mergeTree.ts:515-625): seqOrdered + startOrdered (a SortedSegmentSet of the
  // start references, sortedSegmentSet.ts / sortedSet.ts, restated with its binary search).
  int ordinalCompare(const Seg* a, const Seg* b) const;
  int refCompare(const LRef* a, const LRef* b) const;
  std::pair<bool, size_t> findStart(const LRef* item) const;
  std::vector<ObliterateInfo*> findOverlapping(const Seg* seg) const;
  void obliteratesSetMinSeq(int min);
  void attachRef(LRef* ref, Seg* seg, int offset);
  static void detachRef(LRef* ref);
  std::pair<Seg*, int> getContainingSegment(int pos, const Perspective& p) const;
  uint16_t adjustedValue(uint16_t cur, const fmt_mt_adjust& a);  // computePropertyValue for one adjust
  // computePropertyValue(consensus, changes[0 .. n)) (segmentPropertiesManager.ts:54-78)
  uint16_t foldChanges(uint16_t consensus, const std::vector<PropChangeRec>& changes, size_t n);
  void updateMsn(PropManager& pm, int msn);                             // :275-291
  PropMap getAtSeq(const Seg* s, int seq);                              // :328-344
  double numberOfValue(uint16_t id) const;
  uint16_t valueOfNumber(double x);
  void annotateRange(int start, int end, const std::vector<PropChange>& props,
                     const Perspective& p, Stamp stamp, bool rollbackOp = false);
  void addToLRUSet(Seg* leaf, int seq);
  void setMinSeq(int min);

  void zamboniSegments();
  void scourNode(Block* node, std::vector<Node*>& hold);
  void packParent(Block* parent);

  // BlockIdx maintenance (indexed_ only)
  bool indexed_ = false;
  std::pair<Seg*, Seg*> lastSplit_{nullptr, nullptr};  // the split ensureIntervalBoundary made
  void idxMarkDirty(Block* b);
  void idxRebuild(Block* b);
  int64_t idxLength(Block* b, const Perspective& p);
  void idxAppendEvent(Block* b, int seq, int64_t delta);
  void idxAddClient(Block* b, int client, Seg* s);
  void idxOnNewLeaf(Seg* s);                  // after insertion (+ obliterateOnInsert)
  void idxOnSplit(Seg* left, Seg* right);     // right part of a split, linked after left
  void idxOnRemove(Seg* s, int client, bool wasRemoved);  // after a remove stamp was added
  void idxLeafTerms(Seg* s, BlockIdx& ix);    // a leaf's events and client entries, for rebuilds

  Block* root_;
  Block unfinished_;  // theUnfinishedNode sentinel (mergeTree.ts:656)
  LruHeap heap_;
  std::vector<std::unique_ptr<ObliterateInfo>> obPool_;
  std::vector<ObliterateInfo*> obSeq_;   // seqOrdered (front = lowest seq)
  std::vector<LRef*> obStart_;           // startOrdered
  std::vector<std::unique_ptr<Seg>> segPool_;
  std::vector<std::unique_ptr<Block>> blockPool_;
};

}  // namespace orc
