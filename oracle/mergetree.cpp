// oracle/mergetree.cpp — TEST INFRASTRUCTURE ONLY. See mergetree.hpp for scope and citations.
#include "mergetree.hpp"

#include <algorithm>
#include <list>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "common.hpp"

namespace orc {

// ------------------------------------------------------------------------------------------------
// properties.ts:32-61 matchProperties: same key set, equal values (values are interned JSON texts,
// so equal ids ⇔ equal primitive values). Order-insensitive; undefined matches {}.
// ------------------------------------------------------------------------------------------------
bool matchProperties(const PropMap& a, const PropMap& b) {
  if (a.kv.size() != b.kv.size()) return false;
  for (const auto& [k, v] : a.kv) {
    bool found = false;
    for (const auto& [k2, v2] : b.kv) {
      if (k2 == k) {
        if (v2 != v) return false;
        found = true;
        break;
      }
    }
    if (!found) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------------------
// heap.ts:54-182
// ------------------------------------------------------------------------------------------------
void LruHeap::add(Entry e) {
  L_.push_back(e);
  fixup(count());
}

LruHeap::Entry LruHeap::get() {
  std::swap(L_[1], L_[count()]);
  Entry x = L_.back();
  L_.pop_back();
  fixdown(1);
  return x;
}

void LruHeap::fixup(int k) {
  while (gtParent(k)) {
    const int parent = k >> 1;
    std::swap(L_[k], L_[parent]);
    k = parent;
  }
}

void LruHeap::fixdown(int k) {
  while ((k << 1) <= count()) {
    int j = k << 1;
    if (j < count() && L_[j].maxSeq - L_[j + 1].maxSeq > 0) j++;
    if (L_[k].maxSeq - L_[j].maxSeq <= 0) break;
    std::swap(L_[k], L_[j]);
    k = j;
  }
}

// ------------------------------------------------------------------------------------------------
// Construction and node plumbing
// ------------------------------------------------------------------------------------------------
MergeTree::MergeTree() {
  root_ = makeBlock(0);
  unfinished_.childCount = -1;
}

Block* MergeTree::makeBlock(int childCount) {
  blockPool_.push_back(std::make_unique<Block>());
  Block* b = blockPool_.back().get();
  b->childCount = childCount;
  return b;
}

Seg* MergeTree::makeSeg() {
  segPool_.push_back(std::make_unique<Seg>());
  return segPool_.back().get();
}

// mergeTreeNodes.ts:312-323 assignChild
void MergeTree::assignChild(Block* parent, Node* child, int index) {
  child->parent = parent;
  child->index = index;
  parent->children[index] = child;
}

// ------------------------------------------------------------------------------------------------
// Lengths
// ------------------------------------------------------------------------------------------------
// perspective.ts:57-71 PerspectiveBase.isSegmentPresent
bool MergeTree::isPresent(const Seg* s, const Perspective& p) {
  if (!p.hasOccurred(s->ins)) return false;
  for (const Stamp& r : s->removes)
    if (p.hasOccurred(r)) return false;
  return true;
}

// mergeTree.ts:720-736 leafLength: undefined once the first remove is at or below minSeq.
int MergeTree::leafLength(const Seg* s, const Perspective& p) const {
  if (s->removed() && minSeqHasOccurred(s->removes[0])) return kUndefinedLen;
  return isPresent(s, p) ? s->len() : 0;
}

// mergeTree.ts:2819-2879 blockUpdate: sum of the defined child lengths, undefined if none.
int MergeTree::localBlockLength(const Block* b) const {
  int len = kUndefinedLen;
  const Perspective lp = localPerspective();
  for (int i = 0; i < b->childCount; i++) {
    const Node* c = b->children[i];
    const int l = c->isLeaf ? leafLength(static_cast<const Seg*>(c), lp)
                            : localBlockLength(static_cast<const Block*>(c));
    if (l != kUndefinedLen) len = (len == kUndefinedLen ? 0 : len) + l;
  }
  return len;
}

// PartialSequenceLengths.getPartialLength ≡ Σ leaf nodeLength ?? 0 (partialLengths.ts:1189-1240).
int MergeTree::remoteBlockLength(const Block* b, const Perspective& p) const {
  if (indexed_) return static_cast<int>(const_cast<MergeTree*>(this)->idxLength(const_cast<Block*>(b), p));
  int len = 0;
  for (int i = 0; i < b->childCount; i++) {
    const Node* c = b->children[i];
    if (c->isLeaf) {
      const int l = leafLength(static_cast<const Seg*>(c), p);
      if (l != kUndefinedLen) len += l;
    } else {
      len += remoteBlockLength(static_cast<const Block*>(c), p);
    }
  }
  return len;
}

// mergeTree.ts:1116-1145 nodeLength
int MergeTree::nodeLength(const Node* n, const Perspective& p) const {
  if (n->isLeaf) return leafLength(static_cast<const Seg*>(n), p);
  const Block* b = static_cast<const Block*>(n);
  if (isLocalPerspective(p)) return localBlockLength(b);
  return remoteBlockLength(b, p);
}

int MergeTree::getLocalLength() const {
  const int l = localBlockLength(root_);
  return l == kUndefinedLen ? 0 : l;
}

// ------------------------------------------------------------------------------------------------
// Inserting walk (mergeTree.ts:1811-1987)
// ------------------------------------------------------------------------------------------------
bool MergeTree::breakTie(int pos, const Node* node, const Stamp& stamp) const {
  if (!node->isLeaf) return true;
  if (pos != 0) return false;
  const Seg* s = static_cast<const Seg*>(node);
  return stampGreater(stamp, s->ins) ||
         (s->removed() && s->removes[0].seq != kUnassignedSeq && stampGreater(s->removes[0], stamp));
}

// forwardExcursion(node, ...) visits every leaf after `node` regardless of visibility
// (mergeTreeNodeWalk.ts:123-140); blockInsert's continueFrom only asks whether one exists.
static bool subtreeHasLeaf(const Node* n) {
  if (n->isLeaf) return true;
  const Block* b = static_cast<const Block*>(n);
  for (int i = 0; i < b->childCount; i++)
    if (subtreeHasLeaf(b->children[i])) return true;
  return false;
}

bool MergeTree::hasLeafAfter(const Block* block) const {
  const Node* node = block;
  while (node->parent != nullptr) {
    const Block* p = node->parent;
    for (int i = node->index + 1; i < p->childCount; i++)
      if (subtreeHasLeaf(p->children[i])) return true;
    node = p;
  }
  return false;
}

void MergeTree::insertingWalk(int pos, const Perspective& p, Stamp stamp, InsertCtx& ctx) {
  InsertResult r = insertRecursive(root_, pos, p, stamp, ctx, true);
  if (r.remainder != nullptr) updateRoot(r.remainder);
}

MergeTree::InsertResult MergeTree::insertRecursive(Block* block, int pos, const Perspective& p,
                                                   Stamp stamp, InsertCtx& ctx, bool isLastBlock) {
  int rem = pos;
  int childIndex;
  Node* newNode = nullptr;
  bool hadChanges = false;
  for (childIndex = 0; childIndex < block->childCount; childIndex++) {
    Node* child = block->children[childIndex];
    const bool isLastChildOfLastBlock = isLastBlock && childIndex == block->childCount - 1;
    int len = nodeLength(child, p);
    if (len == kUndefinedLen) {
      if (!isLastChildOfLastBlock) continue;  // removed below minSeq: skipped
      len = 0;
    }
    if (rem < len || (rem == len && breakTie(rem, child, stamp))) {
      if (child->isLeaf) {
        Seg* seg = static_cast<Seg*>(child);
        if (ctx.isInsert) {
          // onLeaf: the candidate replaces the current slot, the old leaf moves after it.
          hadChanges = true;
          assignChild(block, ctx.candidate, childIndex);
          newNode = seg;
          childIndex++;
        } else {
          // splitLeafSegment (mergeTree.ts:1768-1796)
          if (rem > 0) {
            newNode = splitAt(seg, rem);
            lastSplit_ = {seg, static_cast<Seg*>(newNode)};
            hadChanges = true;
            childIndex++;
          } else {
            return {nullptr, hadChanges};
          }
        }
      } else {
        InsertResult r = insertRecursive(static_cast<Block*>(child), rem, p, stamp, ctx,
                                         isLastChildOfLastBlock);
        hadChanges = hadChanges || r.hadChanges;
        if (r.remainder == nullptr) return r;
        if (r.remainder == &unfinished_) {
          rem -= len;  // act as if shifted past the block
          continue;
        }
        newNode = r.remainder;
        childIndex++;
      }
      break;
    }
    rem -= len;
  }
  if (newNode == nullptr && rem == 0) {
    if (ctx.isInsert) {
      if (hasLeafAfter(block)) return {&unfinished_, hadChanges};
      newNode = ctx.candidate;
    }
  }
  if (newNode != nullptr) {
    hadChanges = true;
    for (int i = block->childCount; i > childIndex; i--) {
      block->children[i] = block->children[i - 1];
      block->children[i]->index = i;
    }
    assignChild(block, newNode, childIndex);
    block->childCount++;
    if (block->childCount < kMaxNodesInBlock) return {nullptr, hadChanges};
    return {split(block), hadChanges};
  }
  return {nullptr, hadChanges};
}

// mergeTree.ts:1974-1987: keep the first half, move the second half to a new block.
Block* MergeTree::split(Block* node) {
  constexpr int half = kMaxNodesInBlock / 2;
  idxMarkDirty(node);  // both halves are re-indexed from their children (nb is new)
  Block* nb = makeBlock(half);
  node->childCount = half;
  for (int i = 0; i < half; i++) {
    assignChild(nb, node->children[half + i], i);
    node->children[half + i] = nullptr;
  }
  return nb;
}

// mergeTree.ts:1313-1320
void MergeTree::updateRoot(Block* splitNode) {
  Block* nr = makeBlock(2);
  assignChild(nr, root_, 0);
  assignChild(nr, splitNode, 1);
  root_ = nr;
}

// mergeTreeNodes.ts:389-435 splitAt + textSegment.ts:95-103 + segmentPropertiesManager.ts:24-42.
Seg* MergeTree::splitAt(Seg* seg, int pos) {
  Seg* next = makeSeg();
  next->text = seg->text.substr(static_cast<size_t>(pos));
  seg->text.resize(static_cast<size_t>(pos));
  next->ins = seg->ins;
  next->removes = seg->removes;
  // SegmentGroupCollection.copyTo (segmentGroupCollection.ts:47-59, splitLeafSegment mergeTree.ts:1779-1782):
  // the right part joins every pending group of the left, in the left's queue order
  for (SegmentGroup* g : seg->groups) {
    next->groups.push_back(g);
    if (g->hasPrevious) {
      const size_t idx = static_cast<size_t>(std::find(g->segments.begin(), g->segments.end(), seg) - g->segments.begin());
      const bool found = idx < g->segments.size();
      g->segments.push_back(next);
      if (found) {
        auto copy = g->previousProps.at(idx);  // (push_back may reallocate)
        g->previousProps.push_back(std::move(copy));
      }
    } else {
      g->segments.push_back(next);
    }
  }
  if (seg->props.defined) {  // copyPropertiesAndManager (segmentPropertiesManager.ts:24-42, copyTo :300-316)
    next->props = seg->props;
    if (seg->pm) next->pm = std::make_unique<PropManager>(*seg->pm);
  }
  // LocalReferenceCollection.split (localReference.ts:464-483): refs at offset >= pos move over
  std::vector<LRef*> keep;
  for (LRef* r : seg->refs) {
    if (r->offset >= pos) {
      r->seg = next;
      r->offset -= pos;
      next->refs.push_back(r);
    } else {
      keep.push_back(r);
    }
  }
  seg->refs.swap(keep);
  return next;
}

// ------------------------------------------------------------------------------------------------
// Obliterate (mergeTree.ts:515-625, 1642-1746, 2083-2290)
// ------------------------------------------------------------------------------------------------
// Segment ordinals compare as strings (mergeTreeNodes.ts setOrdinal, ordinal.ts): for linked
// segments that is document order, i.e. the order of their child-index paths from the root; an
// unlinked segment's ordinal is undefined, which SortedSegmentSet reads as "" (smallest).
int MergeTree::ordinalCompare(const Seg* a, const Seg* b) const {
  const bool la = a != nullptr && a->parent != nullptr, lb = b != nullptr && b->parent != nullptr;
  if (!la || !lb) return la == lb ? 0 : (la ? 1 : -1);
  if (a == b) return 0;
  auto path = [](const Node* n) {
    std::vector<int> p;
    for (; n->parent != nullptr; n = n->parent) p.push_back(n->index);
    std::reverse(p.begin(), p.end());
    return p;
  };
  const std::vector<int> pa = path(a), pb = path(b);
  return std::lexicographical_compare(pa.begin(), pa.end(), pb.begin(), pb.end()) ? -1 : 1;
}

int MergeTree::refCompare(const LRef* a, const LRef* b) const {
  const int c = ordinalCompare(a->seg, b->seg);
  return c != 0 ? c : a->offset - b->offset;
}

// SortedSet.findItemPosition (sortedSet.ts) + SortedSegmentSet.onFindEquivalent, verbatim: the
// array is only as sorted as the ordinals were when items went in.
std::pair<bool, size_t> MergeTree::findStart(const LRef* item) const {
  if (obStart_.empty()) return {false, 0};
  long start = 0, end = static_cast<long>(obStart_.size()) - 1, index = -1;
  while (start <= end) {
    index = start + (end - start) / 2;
    const int c = refCompare(item, obStart_[index]);
    if (c < 0) {
      if (start == index) return {false, static_cast<size_t>(index)};
      end = index - 1;
    } else if (c > 0) {
      if (index == end) return {false, static_cast<size_t>(index + 1)};
      start = index + 1;
    } else {
      if (item == obStart_[index]) return {true, static_cast<size_t>(index)};
      for (long b = index - 1; b >= 0 && refCompare(item, obStart_[b]) == 0; b--)
        if (obStart_[b] == item) return {true, static_cast<size_t>(b)};
      for (; index < static_cast<long>(obStart_.size()) && refCompare(item, obStart_[index]) == 0; index++)
        if (obStart_[index] == item) return {true, static_cast<size_t>(index)};
      return {false, static_cast<size_t>(index)};
    }
  }
  return {false, static_cast<size_t>(index)};
}

// Obliterates.findOverlapping (mergeTree.ts:566-582): walk the starts in array order, stop at the
// first start that is unlinked or past the segment.
std::vector<ObliterateInfo*> MergeTree::findOverlapping(const Seg* seg) const {
  std::vector<ObliterateInfo*> out;
  for (const LRef* start : obStart_) {
    const Seg* startSeg = start->seg;
    if (startSeg != nullptr && startSeg->parent != nullptr && ordinalCompare(startSeg, seg) <= 0) {
      const Seg* endSeg = start->ob->end.seg;
      if (endSeg != nullptr && endSeg->parent != nullptr && ordinalCompare(endSeg, seg) >= 0)
        out.push_back(start->ob);
    } else {
      break;
    }
  }
  return out;
}

void MergeTree::attachRef(LRef* ref, Seg* seg, int offset) {
  ref->seg = seg;
  ref->offset = offset;
  seg->refs.push_back(ref);
}

void MergeTree::detachRef(LRef* ref) {
  if (ref->seg != nullptr) {
    auto& v = ref->seg->refs;
    v.erase(std::remove(v.begin(), v.end(), ref), v.end());
  }
  ref->seg = nullptr;
}

// Obliterates.setMinSeq (mergeTree.ts:537-545)
void MergeTree::obliteratesSetMinSeq(int min) {
  size_t k = 0;
  for (; k < obSeq_.size() && obSeq_[k]->stamp.seq <= min; k++) {
    ObliterateInfo* ob = obSeq_[k];
    const auto pos = findStart(&ob->start);
    if (pos.first) obStart_.erase(obStart_.begin() + static_cast<long>(pos.second));
    detachRef(&ob->start);
    detachRef(&ob->end);
  }
  obSeq_.erase(obSeq_.begin(), obSeq_.begin() + static_cast<long>(k));
}

// getContainingSegment (mergeTree.ts:858-886): the first leaf nodeMap visits in [pos, pos + 1).
std::pair<Seg*, int> MergeTree::getContainingSegment(int pos, const Perspective& p) const {
  Seg* found = nullptr;
  int offset = 0;
  int walkPos = 0;
  bool exit = false;
  auto walk = [&](auto&& self, const Block* b) -> void {
    for (int i = 0; i < b->childCount && !exit; i++) {
      if (pos + 1 <= walkPos) {
        exit = true;
        return;
      }
      const Node* n = b->children[i];
      const int len = nodeLength(n, p);
      const int lenAt = len == kUndefinedLen ? 0 : len;
      if (lenAt == 0) continue;
      const int nextPos = walkPos + lenAt;
      if (pos >= nextPos) {
        walkPos = nextPos;
        continue;
      }
      if (n->isLeaf) {
        found = const_cast<Seg*>(static_cast<const Seg*>(n));
        offset = pos - walkPos;
        exit = true;
        return;
      }
      self(self, static_cast<const Block*>(n));
    }
  };
  walk(walk, root_);
  return {found, offset};
}

// obliterateRangeSided (mergeTree.ts:2083-2260). `start`/`end` are the places' pos; the boundaries
// are the places' Before edges ({p, After} is the edge at p + 1, :2090-2091).
void MergeTree::obliterateRange(int start, bool startBefore, int endPlace, bool endBefore, const Perspective& p,
                                Stamp stamp) {
  stamp.kind = 1;  // sliceRemove (mergeTree.ts:2270)
  const int startPos = startBefore ? start : start + 1, endPos = endBefore ? endPlace : endPlace + 1;
  const int end = endPlace + 1;  // nodeMap(start.pos, end.pos + 1): the end reference's segment included
  ensureIntervalBoundary(startPos, p);
  ensureIntervalBoundary(endPos, p);
  obPool_.push_back(std::make_unique<ObliterateInfo>());
  ObliterateInfo* ob = obPool_.back().get();
  ob->stamp = stamp;
  ob->refSeq = p.refSeq;
  const auto s0 = getContainingSegment(start, p);
  const auto s1 = getContainingSegment(endPlace, p);
  if (s0.first == nullptr || s1.first == nullptr) throw DataError("segments cannot be undefined");  // 0xa3f
  ob->start.ob = ob;
  ob->end.ob = ob;
  attachRef(&ob->start, s0.first, s0.second);
  attachRef(&ob->end, s1.first, s1.second);
  obSeq_.push_back(ob);
  const auto at = findStart(&ob->start);
  if (!at.first) obStart_.insert(obStart_.begin() + static_cast<long>(at.second), &ob->start);

  // nodeMap(perspective, markRemoved, ..., start, end, RemoteObliteratePerspective(client)):
  // positions come from the op's view; a leaf is visited when it has length there or is not
  // removed at all (concurrent inserts included). Blocks are only skipped when wholly before start.
  std::vector<Seg*> newlyRemoved;
  int pos = 0;
  bool exit = false;
  auto walk = [&](auto&& self, Block* b) -> void {
    for (int i = 0; i < b->childCount && !exit; i++) {
      if (end <= pos) {
        exit = true;
        return;
      }
      Node* n = b->children[i];
      const int lenAt0 = nodeLength(n, p);
      const int lenAt = lenAt0 == kUndefinedLen ? 0 : lenAt0;
      if (n->isLeaf && lenAt == 0 && static_cast<Seg*>(n)->removed()) continue;
      const int nextPos = pos + lenAt;
      if (start >= nextPos) {
        pos = nextPos;
        continue;
      }
      if (n->isLeaf) {
        Seg* s = static_cast<Seg*>(n);
        // markRemoved's exclusive endpoints (:2145-2152): walked (so concurrent inserts between
        // them and the range are reached) but not removed
        if ((!startBefore && startPos == pos + s->len()) || (endBefore && endPos == pos && lenAt > 0)) {
          pos = nextPos;
          continue;
        }
        const bool wasRemoved = s->removed();
        if (!wasRemoved) {
          newlyRemoved.push_back(s);
          s->removes.push_back(stamp);
        } else {
          int k = static_cast<int>(s->removes.size()) - 1;
          for (; k >= 0; k--)
            if (stampGreater(stamp, s->removes[k])) break;
          s->removes.insert(s->removes.begin() + (k + 1), stamp);
        }
        if (indexed_) idxOnRemove(s, stamp.client, wasRemoved);
        if (collaborating) addToLRUSet(s, stamp.seq);
        pos = nextPos;
      } else {
        self(self, static_cast<Block*>(n));
      }
    }
  };
  walk(walk, root_);
  if (catchupOut) recordDelta(FMT_MT_OBLITERATE, newlyRemoved);
  if (collaborating && stamp.seq != kUnassignedSeq) zamboniSegments();
}

void MergeTree::obliterateOnInsert(Seg* seg, const Perspective& p, Stamp stamp) {
  if (obStart_.empty()) return;
  const Stamp refSeqStamp{p.refSeq, stamp.client};
  std::vector<Stamp> overlappingAcked;
  ObliterateInfo *oldest = nullptr, *newest = nullptr;
  for (ObliterateInfo* ob : findOverlapping(seg)) {
    if (stampGreater(ob->stamp, refSeqStamp)) {
      if (stamp.client != ob->stamp.client) {
        overlappingAcked.push_back(ob->stamp);
        if (oldest == nullptr || stampGreater(oldest->stamp, ob->stamp)) oldest = ob;
      }
      if (newest == nullptr || stampGreater(ob->stamp, newest->stamp)) newest = ob;
    }
  }
  // every stamp here is acked, so newestAcked === newest (mergeTree.ts:1715-1725)
  if (oldest != nullptr && newest->stamp.client != stamp.client) {
    std::stable_sort(overlappingAcked.begin(), overlappingAcked.end(),
                     [](const Stamp& a, const Stamp& b) { return a.seq < b.seq; });
    seg->removes = overlappingAcked;
  }
}

// mergeTree.ts:1798-1808
void MergeTree::ensureIntervalBoundary(int pos, const Perspective& p) {
  InsertCtx ctx{false, nullptr};
  lastSplit_ = {nullptr, nullptr};
  insertingWalk(pos, p, Stamp{kTreeMaintSeq, p.client}, ctx);
  if (indexed_ && lastSplit_.second != nullptr) idxOnSplit(lastSplit_.first, lastSplit_.second);
}

// ------------------------------------------------------------------------------------------------
// nodeMap (mergeTree.ts:2961-3020) over depthFirstNodeWalk: visits leaves of positive length
// under `p` that lie inside [start, end) after the boundaries have been ensured.
// ------------------------------------------------------------------------------------------------
template <class F>
void MergeTree::nodeMap(const Perspective& p, int start, int end, F&& leafFn) const {
  if (end == start) return;
  int pos = 0;
  bool exit = false;
  auto walk = [&](auto&& self, const Block* b) -> void {
    for (int i = 0; i < b->childCount && !exit; i++) {
      if (end <= pos) {
        exit = true;
        return;
      }
      const Node* n = b->children[i];
      const int len = nodeLength(n, p);
      const int lenAt = len == kUndefinedLen ? 0 : len;
      if (lenAt == 0) continue;  // skip
      const int nextPos = pos + lenAt;
      if (start >= nextPos) {
        pos = nextPos;
        continue;
      }
      if (n->isLeaf) {
        leafFn(const_cast<Seg*>(static_cast<const Seg*>(n)));
        pos = nextPos;
      } else {
        self(self, static_cast<const Block*>(n));
      }
    }
  };
  walk(walk, root_);
}

// ------------------------------------------------------------------------------------------------
// Operations
// ------------------------------------------------------------------------------------------------
// mergeTree.ts:812-822
void MergeTree::addToLRUSet(Seg* leaf, int seq) {
  if (leaf->parent->needsScour != 1 && seq > currentSeq) {
    leaf->parent->needsScour = 1;
    heap_.add({leaf, seq});
  }
}

// mergeTree.ts:1484-1517 insertSegments + :1555-1750 blockInsert (no obliterates in scope).
void MergeTree::insertSegments(int pos, Seg* seg, const Perspective& p, Stamp stamp, bool boundary) {
  if (boundary) ensureIntervalBoundary(pos, p);
  if (seg->len() > 0) {
    seg->ins = stamp;
    InsertCtx ctx{true, seg};
    insertingWalk(pos, p, stamp, ctx);
    if (seg->parent == nullptr) throw DataError("MergeTree insert failed");
    if (stamp.seq != kUnassignedSeq) obliterateOnInsert(seg, p, stamp);
    if (indexed_) idxOnNewLeaf(seg);
    // delta callback precedes zamboni (:1497-1516); an insert obliterated on arrival raises none
    if (catchupOut && !seg->removed()) recordDelta(FMT_MT_INSERT, {seg});
    if (collaborating) {  // saveIfLocal (mergeTree.ts:1573-1591)
      if (isLocal(seg->ins) && stamp.client == clientId)
        addToPendingList(seg, nullptr, stamp.localSeq);
      else if (stampGreater(seg->ins, Stamp{minSeq, kNonCollabClient}))
        addToLRUSet(seg, seg->ins.seq);
    }
  }
  if (collaborating && stamp.seq != kUnassignedSeq) zamboniSegments();
}

// mergeTree.ts:2292-2383 markRangeRemoved; stamps.ts:144-158 spliceIntoList.
void MergeTree::markRangeRemoved(int start, int end, const Perspective& p, Stamp stamp) {
  ensureIntervalBoundary(start, p);
  ensureIntervalBoundary(end, p);
  std::vector<Seg*> hit;
  nodeMap(p, start, end, [&](Seg* s) { hit.push_back(s); });
  std::vector<Seg*> newlyRemoved;  // removedSegments: the REMOVE delta (mergeTree.ts:2314-2321)
  SegmentGroup* group = nullptr;
  for (Seg* s : hit) {
    const bool wasRemoved = s->removed();
    if (!s->removed() || stamp.seq == kUnassignedSeq) {
      if (!s->removed()) newlyRemoved.push_back(s);
      s->removes.push_back(stamp);
    } else {
      int i = static_cast<int>(s->removes.size()) - 1;
      for (; i >= 0; i--)
        if (stampGreater(stamp, s->removes[i])) break;
      s->removes.insert(s->removes.begin() + (i + 1), stamp);
    }
    if (indexed_) idxOnRemove(s, stamp.client, wasRemoved);
    if (collaborating) {  // mergeTree.ts:2335-2347
      if (isLocal(s->removes[0]) && stamp.client == clientId) group = addToPendingList(s, group, stamp.localSeq);
      else addToLRUSet(s, stamp.seq);
    }
  }
  if (catchupOut) recordDelta(FMT_MT_REMOVE, newlyRemoved);  // mergeTree.ts:2363-2368
  if (collaborating && stamp.seq != kUnassignedSeq) zamboniSegments();
}

// segmentPropertiesManager.ts:54-78 computePropertyValue for one adjust change onto the current value
// `cur` (0: null / absent): (typeof number ? value : 0) + delta, then `adjusted > max` (a JSON null
// max compares as 0 and is assigned: null), else `adjusted < min`. Returns the result's value id.
double MergeTree::numberOfValue(uint16_t id) const {
  if (id >= FMT_MT_VALUE_COMPUTED) return numbers.at(id - FMT_MT_VALUE_COMPUTED);
  return valueNum != nullptr && id != 0 && id < nValues ? valueNum[id] : std::nan("");  // (0: null)
}

// A number's value id: the host's id of a === number, else this document's computed entry (new
// entries appended in first-computed order). -0 === 0.
uint16_t MergeTree::valueOfNumber(double x) {
  if (x == 0) x = 0;
  if (hostNumbers != nullptr) {
    auto it = std::lower_bound(hostNumbers->begin(), hostNumbers->end(), x,
                               [](const std::pair<double, uint32_t>& e, double v) { return e.first < v; });
    if (it != hostNumbers->end() && it->first == x) return static_cast<uint16_t>(it->second);
  }
  for (size_t k = 0; k < numbers.size(); k++)
    if (numbers[k] == x) return static_cast<uint16_t>(FMT_MT_VALUE_COMPUTED + k);
  if (numbers.size() >= 0x7FFF) throw DataError("more computed numbers than value ids");
  numbers.push_back(x);
  return static_cast<uint16_t>(FMT_MT_VALUE_COMPUTED + numbers.size() - 1);
}

uint16_t MergeTree::adjustedValue(uint16_t cur, const fmt_mt_adjust& a) {
  const double c = numberOfValue(cur);  // (absent: null → not a number)
  const double adjusted = (std::isnan(c) ? 0.0 : c) + a.delta;
  if ((a.flags & FMT_MT_ADJ_MAX) && adjusted > ((a.flags & FMT_MT_ADJ_MAX_NULL) ? 0.0 : a.max))
    return (a.flags & FMT_MT_ADJ_MAX_NULL) ? 0 : valueOfNumber(a.max);
  if ((a.flags & FMT_MT_ADJ_MIN) && adjusted < ((a.flags & FMT_MT_ADJ_MIN_NULL) ? 0.0 : a.min))
    return (a.flags & FMT_MT_ADJ_MIN_NULL) ? 0 : valueOfNumber(a.min);
  return valueOfNumber(adjusted);
}

uint16_t MergeTree::foldChanges(uint16_t consensus, const std::vector<PropChangeRec>& changes, size_t n) {
  uint16_t v = consensus;
  for (size_t i = 0; i < n && i < changes.size(); i++) {
    const PropChangeRec& c = changes[i];
    if (!c.adjust) {
      v = c.value;
    } else {
      if (adjusts == nullptr || static_cast<uint32_t>(c.row) >= nAdjusts) throw DataError("adjust row out of range");
      v = adjustedValue(v, adjusts[c.row]);
    }
  }
  return v;
}

// segmentPropertiesManager.ts:275-291: every key folds its remote changes at or below msn into
// msnConsensus; a key left with no pending change loses its entry.
void MergeTree::updateMsn(PropManager& pm, int msn) {
  for (size_t k = 0; k < pm.changes.size();) {
    PropPending& e = pm.changes[k];
    size_t n = 0;
    while (n < e.remote.size() && e.remote[n].seq <= msn) n++;
    e.msnConsensus = foldChanges(e.msnConsensus, e.remote, n);
    e.remote.erase(e.remote.begin(), e.remote.begin() + static_cast<std::ptrdiff_t>(n));
    if (e.remote.empty() && e.local.empty()) pm.changes.erase(pm.changes.begin() + static_cast<std::ptrdiff_t>(k));
    else k++;
  }
}

// segmentPropertiesManager.ts:328-344 getAtSeq: the current properties with every pending key set to
// its msnConsensus folded with the remote changes at or below seq (null: deleted; a key the current
// properties lack goes last, in the manager's key order).
PropMap MergeTree::getAtSeq(const Seg* s, int seq) {
  PropMap out;
  out.defined = true;  // ({...oldProps}: an object even when the properties are undefined)
  out.kv = s->props.kv;
  for (const PropPending& e : s->pm->changes) {
    size_t n = 0;
    while (n < e.remote.size() && e.remote[n].seq <= seq) n++;
    const uint16_t v = foldChanges(e.msnConsensus, e.remote, n);
    auto it = std::find_if(out.kv.begin(), out.kv.end(), [&](const auto& x) { return x.first == e.key; });
    if (v == 0) {
      if (it != out.kv.end()) out.kv.erase(it);
    } else if (it != out.kv.end()) {
      it->second = v;
    } else {
      out.kv.emplace_back(e.key, v);
    }
  }
  return out;
}

// mergeTree.ts:2009-2081 annotateRange + segmentPropertiesManager.ts:188-238 handleProperties: a
// key's entry starts at its current value (null when absent); a local change joins its local list, a
// raw remote change folds into msnConsensus while the key has no remote change pending and is queued
// otherwise (an adjust always is); properties[key] = computePropertyValue(msnConsensus, remote,
// local); null deletes the key; `seg.properties ??= createMap()` runs even if nothing changes. Then
// updateMsn(collabWindow.minSeq). A local op's segments join its pending group with their
// propertyDeltas (the keys' previous values, for rollback); rollbackOp: rollbackProperties instead
// (handleProperties' rollback branch, :196-198).
void MergeTree::annotateRange(int start, int end, const std::vector<PropChange>& props, const Perspective& p,
                              Stamp stamp, bool rollbackOp) {
  ensureIntervalBoundary(start, p);
  ensureIntervalBoundary(end, p);
  std::vector<Seg*> hit;
  nodeMap(p, start, end, [&](Seg* s) { hit.push_back(s); });
  SegmentGroup* group = nullptr;
  const bool local = isLocal(stamp);
  for (Seg* s : hit) {
    s->props.defined = true;
    if (!s->pm) s->pm = std::make_unique<PropManager>();
    PropManager& pm = *s->pm;
    if (rollbackOp) {
      std::vector<std::pair<uint16_t, uint16_t>> kv;
      for (const PropChange& ch : props) kv.emplace_back(ch.key, ch.value);
      rollbackProperties(s, kv);
    } else {
      std::vector<std::pair<uint16_t, uint16_t>> deltas;  // propertyDeltas: key -> previous value
      for (const PropChange& ch : props) {
        const uint16_t key = ch.key;
        auto it = std::find_if(s->props.kv.begin(), s->props.kv.end(),
                               [&](const auto& e) { return e.first == key; });
        const uint16_t previous = it != s->props.kv.end() ? it->second : 0;
        auto pe = std::find_if(pm.changes.begin(), pm.changes.end(), [&](const PropPending& e) { return e.key == key; });
        if (pe == pm.changes.end()) {
          pm.changes.push_back(PropPending{key, previous, {}, {}});
          pe = pm.changes.end() - 1;
        }
        const PropChangeRec rec{stamp.seq, ch.adjust >= 0, ch.value, ch.adjust};
        if (local) pe->local.push_back(rec);
        else if (!rec.adjust && pe->remote.empty()) pe->msnConsensus = rec.value;
        else pe->remote.push_back(rec);
        const uint16_t afterRemote = foldChanges(pe->msnConsensus, pe->remote, pe->remote.size());
        const uint16_t value = foldChanges(afterRemote, pe->local, pe->local.size());
        if (local || pe->local.empty() || value != previous) {
          auto d = std::find_if(deltas.begin(), deltas.end(), [&](const auto& e) { return e.first == key; });
          if (d == deltas.end()) deltas.emplace_back(key, previous);
          else d->second = previous;
        }
        if (value == 0) {  // null → delete
          if (it != s->props.kv.end()) s->props.kv.erase(it);
        } else if (it != s->props.kv.end()) {
          it->second = value;
        } else {
          s->props.kv.emplace_back(key, value);
        }
      }
      updateMsn(pm, minSeq);
      if (collaborating && local) group = addToPendingList(s, group, stamp.localSeq, &deltas);
    }
    if (collaborating && !local) addToLRUSet(s, stamp.seq);
  }
  if (catchupOut) {  // deltaSegments: annotated segments not removed (mergeTree.ts:2045-2047, 2068-2073)
    std::vector<Seg*> delta;
    for (Seg* s : hit)
      if (!s->removed()) delta.push_back(s);
    recordDelta(FMT_MT_ANNOTATE, delta);
  }
  if (collaborating && !local) zamboniSegments();
}

// segmentPropertiesManager.ts:140-173 (collaborating): each key of the op (its previous values are
// not read) drops its newest local change and takes computePropertyValue(msnConsensus, remote, local)
// again; a key left with no change loses its entry; null deletes the key.
void MergeTree::rollbackProperties(Seg* s, const std::vector<std::pair<uint16_t, uint16_t>>& props) {
  s->props.defined = true;  // applyChanges: seg.properties ??= createMap()
  if (!s->pm) s->pm = std::make_unique<PropManager>();
  PropManager& pm = *s->pm;
  for (const auto& [key, prev] : props) {
    (void)prev;
    auto pe = std::find_if(pm.changes.begin(), pm.changes.end(), [&](const PropPending& e) { return e.key == key; });
    if (pe == pm.changes.end()) throw DataError("Pending changes must exist for rollback when collaborating");  // 0xa6f
    if (!pe->local.empty()) pe->local.pop_back();
    const uint16_t value = foldChanges(foldChanges(pe->msnConsensus, pe->remote, pe->remote.size()), pe->local, pe->local.size());
    if (pe->local.empty() && pe->remote.empty()) pm.changes.erase(pe);
    auto it = std::find_if(s->props.kv.begin(), s->props.kv.end(), [&](const auto& e) { return e.first == key; });
    if (value == 0) {
      if (it != s->props.kv.end()) s->props.kv.erase(it);
    } else if (it != s->props.kv.end()) {
      it->second = value;
    } else {
      s->props.kv.emplace_back(key, value);
    }
  }
}

// mergeTree.ts:835-856 getPosition: lengths of everything before the node, walking up the parents.
int MergeTree::getPosition(const Node* node) const { return getPosition(node, localPerspective()); }

int MergeTree::getPosition(const Node* node, const Perspective& lp) const {
  int total = 0;
  const Node* prev = node;
  for (const Block* parent = node->parent; parent != nullptr; prev = parent, parent = parent->parent) {
    for (int i = 0; i < parent->childCount; i++) {
      const Node* c = parent->children[i];
      if (c == prev) break;
      const int l = nodeLength(c, lp);
      if (l > 0) total += l;  // `?? 0`
    }
  }
  return total;
}

uint32_t markerIdOf(const Seg* s, uint32_t key) {  // Marker.getId(): properties[reservedMarkerIdKey]
  if (!s->marker || key == FMT_MT_NO_MARKER) return FMT_MT_NO_MARKER;
  for (const auto& [k, v] : s->props.kv)
    if (k == key) return v;
  return FMT_MT_NO_MARKER;
}

void MergeTree::registerMarker(Seg* s) {
  const uint32_t id = markerIdOf(s, markerIdKey);
  if (id != FMT_MT_NO_MARKER) idToMarker[id] = s;
}

void MergeTree::unlinkMarker(const Seg* s) {
  const uint32_t id = markerIdOf(s, markerIdKey);
  if (id != FMT_MT_NO_MARKER) idToMarker.erase(id);
}

int MergeTree::posFromRelativePos(const fmt_mt_relpos& rp, const Perspective& p) const {
  const auto it = rp.marker_id == FMT_MT_NO_MARKER ? idToMarker.end() : idToMarker.find(rp.marker_id);
  // getMarkerFromId (mergeTree.ts:1450-1453): a removed marker is not found
  if (it == idToMarker.end() || it->second->removed()) return -1;
  int pos = getPosition(it->second, p);
  if (rp.flags & FMT_MT_REL_BEFORE) pos -= rp.offset;
  else pos += it->second->len() + rp.offset;  // cachedLength (1 for a marker)
  return pos;
}

// sequence.ts:395-452 createOpsFromDelta over one event's ranges, which SequenceDeltaEventClass
// orders by segment (document order) with position = Client.getPosition (sequenceDeltaEvent.ts:91-103).
// REMOVE merges a range that starts where the previous one started (removed text has no local
// length); ANNOTATE merges a range that starts where the previous one ended when the props match —
// they always do here: every segment's propertyDeltas holds every key of the op, and the raw value
// the segment now holds is the op's own (segmentPropertiesManager.ts:199-235 with no pending local).
void MergeTree::recordDelta(uint32_t type, const std::vector<Seg*>& deltaSegs) {
  const size_t first = catchupOut->size();
  for (const Seg* s : deltaSegs) {
    const int pos = getPosition(s);
    if (catchupOut->size() > first) {
      fmt_mt_catchup_range& last = catchupOut->back();
      if (((type == FMT_MT_REMOVE || type == FMT_MT_OBLITERATE) && last.pos1 == pos) ||
          (type == FMT_MT_ANNOTATE && last.pos2 == pos)) {
        last.pos2 += s->len();
        continue;
      }
    }
    catchupOut->push_back(fmt_mt_catchup_range{catchupOp, pos, pos + s->len(), type});
  }
}

// mergeTree.ts:1147-1166
void MergeTree::setMinSeq(int min) {
  if (min > currentSeq) throw DataError("Trying to set minSeq above currentSeq of collab window!");
  if (minSeq > min) throw DataError("minSeq of collab window > target minSeq!");
  if (min > minSeq) {
    minSeq = min;
    obliteratesSetMinSeq(min);
    zamboniSegments();
  }
}

// client.ts:1381-1391
void MergeTree::updateSeqNumbers(int min, int seq) {
  if (currentSeq > seq) throw DataError("Incoming op sequence# < local collabWindow's currentSequence#");
  currentSeq = seq;
  if (min > seq) throw DataError("Incoming op sequence# < minSequence#");
  setMinSeq(min);
}

void MergeTree::insertLocal(int pos, const std::u16string& text) {
  Seg* s = makeSeg();
  s->text = text;
  insertSegments(pos, s, localPerspective(), Stamp{collaborating ? kUnassignedSeq : 0, clientId});
}

void MergeTree::annotateLocal(int start, int end,
                              const std::vector<std::pair<uint16_t, uint16_t>>& props) {
  std::vector<PropChange> ch;
  for (const auto& [k, v] : props) ch.push_back(PropChange{k, v, -1});
  annotateRange(start, end, ch, localPerspective(),
                Stamp{collaborating ? kUnassignedSeq : 0, clientId});
}

void MergeTree::removeLocal(int start, int end) {
  markRangeRemoved(start, end, localPerspective(),
                   Stamp{collaborating ? kUnassignedSeq : 0, clientId});
}

// ------------------------------------------------------------------------------------------------
// f4: the local client
// ------------------------------------------------------------------------------------------------
// mergeTree.ts:1410-1447 addToPendingList + segmentGroupCollection.ts:25-28 enqueue.
SegmentGroup* MergeTree::addToPendingList(Seg* seg, SegmentGroup* group, int localSeqArg,
                                          const std::vector<std::pair<uint16_t, uint16_t>>* previousProps) {
  if (group == nullptr) {
    if (localSeqArg <= 0) throw DataError("Local seq should be passed when creating new segment group");  // 0xb72
    groupPool_.push_back(std::make_unique<SegmentGroup>());
    group = groupPool_.back().get();
    group->localSeq = localSeqArg;
    group->refSeq = currentSeq;
    group->hasPrevious = previousProps != nullptr;
    pendingSegments_.push_back(group);
  }
  if (group->hasPrevious != (previousProps != nullptr)) throw DataError("All segments in group should have previousProps or none");
  if (previousProps) group->previousProps.push_back(*previousProps);
  seg->groups.push_back(group);
  group->segments.push_back(seg);
  return group;
}

namespace {
std::vector<MergeTree::PropChange> opChanges(const fmt_mt_op& op, const uint32_t* propsOff, const uint32_t* propsKv) {
  std::vector<MergeTree::PropChange> kv;
  for (uint32_t i = propsOff[op.payload]; i < propsOff[op.payload + 1]; i++) {
    const uint16_t key = static_cast<uint16_t>(propsKv[i] >> 16), value = static_cast<uint16_t>(propsKv[i] & 0xffff);
    if (value == FMT_MT_VALUE_ADJUST) {
      if (i + 1 >= propsOff[op.payload + 1]) throw DataError("adjust entry without its row");
      kv.push_back(MergeTree::PropChange{key, 0, static_cast<int32_t>(propsKv[++i])});
    } else {
      kv.push_back(MergeTree::PropChange{key, value, -1});
    }
  }
  return kv;
}
}  // namespace

void MergeTree::applyLocal(const fmt_mt_op& op, const uint16_t* arena, const uint32_t* propsOff, const uint32_t* propsKv) {
  if (!collaborating) throw DataError("local op before collaboration");
  const Perspective lp = localPerspective();
  // getValidOpRange (client.ts:749-815), local branch: positions against the local length
  const int length = getLocalLength();
  const int start = op.pos1, end = op.pos2;
  if (op.type == FMT_MT_INSERT) {
    if (start < 0 || start > length) throw UsageError("RangeOutOfBounds");
  } else if (op.type == FMT_MT_REMOVE || op.type == FMT_MT_ANNOTATE) {
    if (start < 0 || start >= length || end <= start) throw UsageError("RangeOutOfBounds");
  } else {
    throw DataError("unsupported local op type");
  }
  const size_t groupsBefore = pendingSegments_.size();
  Stamp stamp{kUnassignedSeq, clientId, 0, 0};
  if (op.type == FMT_MT_INSERT) {
    const uint32_t len = fmt_mt_op_len(&op);
    if (len == 0) return;  // insertSegmentLocal: nothing to insert, no op (client.ts:348-351)
    stamp.localSeq = ++localSeq;  // mintNextLocalOperationStamp (mergeTreeNodes.ts:685-695)
    Seg* s = makeSeg();
    s->text.assign(reinterpret_cast<const char16_t*>(arena + op.payload), len);
    s->marker = (op.flags & FMT_MT_F_MARKER) != 0;
    if (op.pos2 > 0) {
      const uint32_t id = static_cast<uint32_t>(op.pos2 - 1);
      s->props.defined = true;
      for (uint32_t i = propsOff[id]; i < propsOff[id + 1]; i++) {
        const uint16_t key = static_cast<uint16_t>(propsKv[i] >> 16), value = static_cast<uint16_t>(propsKv[i] & 0xffff);
        auto it = std::find_if(s->props.kv.begin(), s->props.kv.end(), [&](const auto& e) { return e.first == key; });
        if (value == 0) {
          if (it != s->props.kv.end()) s->props.kv.erase(it);
        } else if (it != s->props.kv.end()) {
          it->second = value;
        } else {
          s->props.kv.emplace_back(key, value);
        }
      }
    }
    if (s->marker) registerMarker(s);
    insertSegments(start, s, lp, stamp);
  } else if (op.type == FMT_MT_REMOVE) {
    stamp.localSeq = ++localSeq;
    markRangeRemoved(start, end, lp, stamp);
  } else {
    const std::vector<PropChange> changes = opChanges(op, propsOff, propsKv);
    // annotateAdjustRangeLocal (client.ts:286-301): min greater than max is a UsageError, before the
    // op applies (a JSON null bound compares as 0)
    for (const PropChange& ch : changes) {
      if (ch.adjust < 0) continue;
      if (adjusts == nullptr || static_cast<uint32_t>(ch.adjust) >= nAdjusts) throw DataError("adjust row out of range");
      const fmt_mt_adjust& a = adjusts[ch.adjust];
      const double mn = (a.flags & FMT_MT_ADJ_MIN_NULL) ? 0.0 : a.min, mx = (a.flags & FMT_MT_ADJ_MAX_NULL) ? 0.0 : a.max;
      if ((a.flags & FMT_MT_ADJ_MIN) && (a.flags & FMT_MT_ADJ_MAX) && mn > mx) throw UsageError("min is greater than max");
    }
    stamp.localSeq = ++localSeq;
    annotateRange(start, end, changes, lp, stamp);
  }
  if (pendingSegments_.size() != groupsBefore + 1) throw DataError("local op created no segment group");
  SegmentGroup* g = pendingSegments_.back();
  g->type = op.type;
  g->payload = static_cast<int32_t>(op.payload);
  g->pos2 = op.type == FMT_MT_INSERT ? op.pos2 : 0;
  g->flags = op.flags & FMT_MT_F_MARKER;
  g->inflightRef = op.ref_seq;  // (the record's ref_seq: the refSeq it was submitted at)
}

// mergeTree.ts:149-215 ackSegment + :1325-1408 ackOp.
void MergeTree::ackOp(const fmt_mt_op& op, const uint32_t* propsOff, const uint32_t* propsKv) {
  if (pendingSegments_.empty()) throw DataError("ack without a pending local op");
  SegmentGroup* g = pendingSegments_.front();
  if (g->type != op.type) throw DataError("ack of a different op type than the oldest pending op");
  pendingSegments_.erase(pendingSegments_.begin());
  const Stamp stamp{op.seq, clientId};
  std::vector<PropChange> changes;
  if (op.type == FMT_MT_ANNOTATE) changes = opChanges(op, propsOff, propsKv);
  for (Seg* seg : g->segments) {
    if (seg->groups.empty() || seg->groups.front() != g) throw DataError("On ack, unexpected segmentGroup!");  // 0x043
    seg->groups.erase(seg->groups.begin());
    switch (op.type) {
      case FMT_MT_ANNOTATE: {  // PropertiesManager.ack (segmentPropertiesManager.ts:248-267)
        if (!seg->pm) throw DataError("On annotate ack, missing segment property manager!");  // 0x044
        for (const PropChange& ch : changes) {
          auto pe = std::find_if(seg->pm->changes.begin(), seg->pm->changes.end(),
                                 [&](const PropPending& e) { return e.key == ch.key; });
          if (pe == seg->pm->changes.end() || pe->local.empty()) throw DataError("must have local change to ack");  // 0xa71
          pe->local.erase(pe->local.begin());
          const PropChangeRec rec{op.seq, ch.adjust >= 0, ch.value, ch.adjust};
          if (!rec.adjust && pe->remote.empty()) pe->msnConsensus = rec.value;
          else pe->remote.push_back(rec);
        }
        updateMsn(*seg->pm, op.min_seq);  // (the acked message's minimumSequenceNumber)
        break;
      }
      case FMT_MT_INSERT:
        if (!isLocal(seg->ins)) throw DataError("On insert, seq number already assigned!");  // 0x045
        seg->ins = stamp;
        break;
      case FMT_MT_REMOVE: {
        if (!seg->removed() || !isLocal(seg->removes.back())) throw DataError("Expected last remove to be unacked");  // 0xb5d
        if (seg->removes.size() > 1 && isLocal(seg->removes[seg->removes.size() - 2]))
          throw DataError("Expected prior remove to be acked");  // 0xb5e
        seg->removes.back() = Stamp{op.seq, clientId, 0, 0};
        break;
      }
      default:
        throw DataError("unsupported ack op type");
    }
    addToLRUSet(seg, op.seq);
  }
  zamboniSegments();
}

// mergeTree.ts:2519-2536: the lengths of the not-removed segments before it.
int MergeTree::findRollbackPosition(const Seg* seg) const {
  int pos = 0;
  bool found = false;
  auto walk = [&](auto&& self, const Block* b) -> void {
    for (int i = 0; i < b->childCount && !found; i++) {
      const Node* n = b->children[i];
      if (!n->isLeaf) {
        self(self, static_cast<const Block*>(n));
        continue;
      }
      const Seg* s = static_cast<const Seg*>(n);
      if (s == seg) {
        found = true;
        return;
      }
      if (!s->removed()) pos += s->len();
    }
  };
  walk(walk, root_);
  return pos;
}

// mergeTree.ts:2388-2514 rollback (one op; GROUP members are rolled back last first by the caller).
void MergeTree::rollback(const fmt_mt_op& op) {
  if (pendingSegments_.empty()) throw DataError("Rollback op doesn't match last edit");
  SegmentGroup* g = pendingSegments_.back();
  if (g->type != op.type || (op.type == FMT_MT_ANNOTATE && !g->hasPrevious))
    throw DataError("Rollback op doesn't match last edit");
  pendingSegments_.pop_back();
  const Stamp rollbackStamp{kTreeMaintSeq, kNonCollabClient};
  if (op.type == FMT_MT_REMOVE) {
    for (Seg* seg : g->segments) {
      if (seg->groups.empty() || seg->groups.back() != g) throw DataError("Unexpected segmentGroup in segment");  // 0x3ee
      seg->groups.pop_back();
      if (!seg->removed() || seg->removes[0].kind != 0) throw DataError("Rollback segment removedClientId does not match local client");  // 0x39d
      // a peer's concurrent remove keeps the segment removed
      if (seg->removes[0].client == clientId) seg->removes.clear();  // removeRemovalInfo
    }
    return;
  }
  if (op.type != FMT_MT_INSERT && op.type != FMT_MT_ANNOTATE) throw DataError("Unsupported op type for rollback");
  size_t i = 0;
  for (Seg* seg : g->segments) {
    if (seg->groups.empty() || seg->groups.back() != g) throw DataError("Unexpected segmentGroup in segment");  // 0x3ef
    seg->groups.pop_back();
    const int start = findRollbackPosition(seg);
    if (op.type == FMT_MT_INSERT) {
      seg->ins = rollbackStamp;
      markRangeRemoved(start, start + seg->len(), localPerspective(), rollbackStamp);
    } else {
      const auto& props = g->previousProps.at(i);
      if (seg->removed()) {
        rollbackProperties(seg, props);
      } else {
        std::vector<PropChange> ch;
        for (const auto& [k, v] : props) ch.push_back(PropChange{k, v, -1});
        annotateRange(start, start + seg->len(), ch, localPerspective(), rollbackStamp, true);
      }
      i++;
    }
  }
}

// mergeTree.ts:2613-2712 normalizeAdjacentSegments over one run of adjacent removed / locally
// inserted segments: segments removed by others slide after the last segment the local client
// affected, locally removed ones past the local inserts made after their removal; the new order
// takes the run's slots (parent, index) in order.
void MergeTree::normalizeAdjacentSegments(std::vector<Seg*>& range) {
  std::vector<std::pair<Block*, int>> slots;
  for (Seg* s : range) slots.emplace_back(s->parent, s->index);
  std::list<Seg*> list(range.begin(), range.end());
  auto lastLocal = list.end();
  for (auto it = list.end(); it != list.begin();) {
    --it;
    if (!isRemovedAndAcked(*it)) {
      lastLocal = it;
      break;
    }
  }
  if (lastLocal == list.end()) return;
  auto slide = lastLocal;
  for (;;) {
    const bool hasNearer = slide != list.begin();
    const auto nearer = hasNearer ? std::prev(slide) : list.end();
    Seg* seg = *slide;
    if (isRemovedAndAcked(seg)) {
      list.erase(slide);
      list.insert(std::next(lastLocal), seg);
    } else if (seg->removed()) {
      auto cur = slide;
      for (auto scan = std::next(cur); scan != list.end() && !isRemovedAndAcked(*scan) && (*scan)->ins.localSeq > 0 &&
                                       stampGreater((*scan)->ins, seg->removes[0]);
           ++scan)
        cur = scan;
      if (cur != slide) {
        list.erase(slide);
        list.insert(std::next(cur), seg);
      }
    }
    if (!hasNearer) break;
    slide = nearer;
  }
  size_t k = 0;
  for (Seg* s : list) {
    assignChild(slots[k].first, s, slots[k].second);
    k++;
  }
}

// mergeTree.ts:2734-2766: runs of adjacent segments that are removed or locally inserted, normalized
// when a run holds both a local insert and a segment removed by an acked op.
void MergeTree::normalizeSegmentsOnRebase() {
  std::vector<Seg*> range;
  bool hasLocal = false, hasRemote = false;
  auto flush = [&]() {
    if (hasLocal && hasRemote && range.size() > 1) normalizeAdjacentSegments(range);
    range.clear();
    hasLocal = hasRemote = false;
  };
  std::vector<const Seg*> leaves;
  std::vector<int> blockOf;
  int nb = 0, depth = 0;
  collectLeaves(leaves, blockOf, &nb, &depth);
  for (const Seg* cs : leaves) {
    Seg* s = const_cast<Seg*>(cs);
    if (s->removed() || isLocal(s->ins)) {
      if (isRemovedAndAcked(s)) hasRemote = true;
      if (isLocal(s->ins)) hasLocal = true;
      range.push_back(s);
    } else {
      flush();
    }
  }
  flush();
}

void MergeTree::regeneratePending(std::vector<fmt_mt_op>* out, std::u16string* text) {
  if (pendingSegments_.empty()) return;
  std::vector<SegmentGroup*> rebase;
  rebase.swap(pendingSegments_);  // pendingRebase = pendingSegments.splice(first) (client.ts:1470-1477)
  if (!lastNormSet_ || currentSeq != lastNormRefSeq_ || localSeq != lastNormLocalSeq_) {
    normalizeSegmentsOnRebase();
    lastNormSet_ = true;
    lastNormRefSeq_ = currentSeq;
    lastNormLocalSeq_ = localSeq;
  }
  // document order of every leaf (the segments' ordinals)
  std::vector<const Seg*> leaves;
  std::vector<int> blockOf;
  int nb = 0, depth = 0;
  collectLeaves(leaves, blockOf, &nb, &depth);
  std::map<const Seg*, size_t> ordinal;
  for (size_t k = 0; k < leaves.size(); k++) ordinal[leaves[k]] = k;
  for (SegmentGroup* g : rebase) {  // resetPendingDeltaToOps (client.ts:963-1289), non-obliterate ops
    std::vector<Seg*> segs = g->segments;
    std::sort(segs.begin(), segs.end(), [&](const Seg* a, const Seg* b) { return ordinal.at(a) < ordinal.at(b); });
    const Perspective rp{false, currentSeq, clientId, g->localSeq};
    for (Seg* seg : segs) {
      auto it = std::find(seg->groups.begin(), seg->groups.end(), g);
      if (it == seg->groups.end()) throw DataError("Segment group not in segment pending queue");  // 0xb6c
      seg->groups.erase(it);
      const int pos = getPosition(seg, rp);  // findReconnectionPosition (client.ts:866-877)
      fmt_mt_op o;
      std::memset(&o, 0, sizeof o);
      o.seq = g->localSeq;
      o.ref_seq = currentSeq;
      o.client = 0;
      o.type = static_cast<uint8_t>(g->type);
      bool emit = false;
      if (g->type == FMT_MT_ANNOTATE) {
        if (!isRemovedAndAcked(seg)) {
          o.pos1 = pos;
          o.pos2 = pos + seg->len();
          o.payload = static_cast<uint32_t>(g->payload);
          emit = true;
        }
      } else if (g->type == FMT_MT_INSERT) {
        if (!isLocal(seg->ins)) throw DataError("Segment already has assigned sequence number");  // 0x037
        if (seg->removed() && !isLocal(seg->removes[0])) throw DataError("obliterated local insert (obliterate reconnect unsupported)");
        o.pos1 = pos;
        o.pos2 = g->pos2;  // the original op's seg props (client.ts:1246-1252)
        o.payload = static_cast<uint32_t>(text->size());
        const uint32_t len = static_cast<uint32_t>(seg->len());
        o.len = static_cast<uint16_t>(len & 0xFFFFu);
        o.flags = (len & FMT_MT_F_LEN_HI_MASK) | (seg->marker ? FMT_MT_F_MARKER : 0u);
        text->append(seg->text);
        emit = true;
      } else if (g->type == FMT_MT_REMOVE) {
        if (seg->removed() && isLocal(seg->removes[0])) {
          o.pos1 = pos;
          o.pos2 = pos + seg->len();
          emit = true;
        }
      } else {
        throw DataError("Invalid op type");
      }
      if (!emit) continue;
      groupPool_.push_back(std::make_unique<SegmentGroup>());
      SegmentGroup* ng = groupPool_.back().get();
      ng->localSeq = g->localSeq;
      ng->refSeq = currentSeq;
      ng->hasPrevious = g->hasPrevious;
      ng->previousProps = g->previousProps;
      ng->type = g->type;
      ng->payload = g->payload;
      ng->pos2 = g->pos2;
      ng->flags = g->flags;
      ng->inflightRef = g->inflightRef;
      seg->groups.push_back(ng);
      ng->segments.push_back(seg);
      pendingSegments_.push_back(ng);
      out->push_back(o);
    }
  }
}

void MergeTree::loadSnapshot(const std::vector<LoadedSeg>& header, const std::vector<LoadedSeg>& body,
                             int minSeqArg, int seqArg) {
  // specToSegment (snapshotLoader.ts:180-186): a legacy spec is inserted at {0, NonCollabClient};
  // TextSegment.fromJSONObject adds the spec's props in their key order.
  auto make = [&](const LoadedSeg& l) {
    Seg* s = makeSeg();
    s->text = l.text;
    s->marker = l.marker;
    s->ins = l.ins;
    s->removes = l.removes;
    if (l.hasProps) {
      s->props.defined = true;
      for (const auto& [key, value] : l.props) {
        auto it = std::find_if(s->props.kv.begin(), s->props.kv.end(),
                               [&](const auto& e) { return e.first == key; });
        if (value == 0) {
          if (it != s->props.kv.end()) s->props.kv.erase(it);
        } else if (it != s->props.kv.end()) {
          it->second = value;
        } else {
          s->props.kv.emplace_back(key, value);
        }
      }
    }
    if (s->marker) registerMarker(s);  // blockUpdate (mergeTree.ts:2833-2841): loaded markers are present
    return s;
  };
  // reloadFromSegments: bottom-up, MaxNodesInBlock - 1 = 7 children per block, layer by layer.
  std::vector<Node*> nodes;
  for (const LoadedSeg& l : header) nodes.push_back(make(l));
  if (nodes.empty()) {
    root_ = makeBlock(0);
  } else {
    constexpr int maxChildren = kMaxNodesInBlock - 1;
    for (;;) {
      std::vector<Node*> blocks;
      for (size_t i = 0; i < nodes.size();) {
        Block* b = makeBlock(0);
        for (int c = 0; c < maxChildren && i < nodes.size(); c++, i++) assignChild(b, nodes[i], b->childCount++);
        blocks.push_back(b);
      }
      if (blocks.size() == 1) {
        root_ = static_cast<Block*>(blocks[0]);
        break;
      }
      nodes.swap(blocks);
    }
  }
  root_->parent = nullptr;
  startCollaboration(0, minSeqArg, seqArg);  // loadHeader (snapshotLoader.ts:204-216)
  const Perspective p{false, 0, kNonCollabClient};
  // (the local length grows by each appended segment: every loaded segment is present, so it is
  // summed once rather than walked per append)
  int localLen = getLocalLength();
  for (const LoadedSeg& l : body) {
    Seg* s = make(l);
    const int len = s->len();
    insertSegments(localLen, s, p, Stamp{0, kNonCollabClient});
    localLen += len;
  }
}

void MergeTree::startCollaboration(int localClientId, int minSeqArg, int currentSeqArg) {
  clientId = localClientId;
  minSeq = minSeqArg;
  collaborating = true;
  currentSeq = currentSeqArg;
}

// client.ts:1291-1327 applyRemoteOp → applyInsertOp / applyRemoveRangeOp / applyAnnotateRangeOp
// with PriorPerspective(refSeq, clientId) and stamp {seq, clientId} (client.ts:581-611).
void MergeTree::applyRemote(const fmt_mt_op& opIn, const uint16_t* arena, const uint32_t* propsOff,
                            const uint32_t* propsKv) {
  const Perspective p{false, opIn.ref_seq, opIn.client};
  fmt_mt_op op = opIn;
  // getValidOpRange (client.ts:758-767): an undefined pos1/pos2 comes from relativePos1/2
  for (int k = 0; k < 2; k++) {
    if ((op.flags & (k == 0 ? FMT_MT_F_REL1 : FMT_MT_F_REL2)) == 0) continue;
    int32_t& pos = k == 0 ? op.pos1 : op.pos2;
    if (pos < 0 || static_cast<uint32_t>(pos) >= nRelpos) throw DataError("relative position index out of range");
    pos = posFromRelativePos(relpos[pos], p);
    if (pos < 0) throw DataError("relative position names no marker");
  }
  const Stamp stamp{op.seq, op.client};
  switch (op.type) {
    case FMT_MT_INSERT: {
      Seg* s = makeSeg();
      s->text.assign(reinterpret_cast<const char16_t*>(arena + op.payload), fmt_mt_op_len(&op));
      s->marker = (op.flags & FMT_MT_F_MARKER) != 0;  // Marker.make(refType, props)
      // seg {text, props}: TextSegment.make(text, props) → BaseSegment's `properties = clone(props)`
      // (textSegment.ts:41-52, mergeTreeNodes.ts:343-347; clone = extend({}, props): null values
      // dropped, properties.ts:68-95). pos2 = props-op id + 1 (0: a plain string segment).
      if (op.pos2 > 0) {
        const uint32_t id = static_cast<uint32_t>(op.pos2 - 1);
        s->props.defined = true;
        for (uint32_t i = propsOff[id]; i < propsOff[id + 1]; i++) {
          const uint16_t key = static_cast<uint16_t>(propsKv[i] >> 16), value = static_cast<uint16_t>(propsKv[i] & 0xffff);
          auto it = std::find_if(s->props.kv.begin(), s->props.kv.end(), [&](const auto& e) { return e.first == key; });
          if (value == 0) {
            if (it != s->props.kv.end()) s->props.kv.erase(it);
          } else if (it != s->props.kv.end()) {
            it->second = value;
          } else {
            s->props.kv.emplace_back(key, value);
          }
        }
      }
      if (s->marker) registerMarker(s);  // idToMarker.set (mergeTree.ts:1614-1620)
      if (op.flags & FMT_MT_F_LOADSEG) {
        // SnapshotLoader.loadBody's append (snapshotLoader.ts:287-309): insertSegments at
        // root.cachedLength from PriorPerspective(UniversalSequenceNumber, clientId) with stamp
        // {seq, clientId}; specToSegment's remove stamps stay on the segment (:105-175)
        const int client = op.client == FMT_MT_CLIENT_NONCOLLAB ? kNonCollabClient : static_cast<int>(op.client);
        if (snapInfo == nullptr || op.pos1 < 0 || static_cast<uint64_t>(op.pos1) >= nSnapInfo)
          throw DataError("loader segment without its merge info");
        const fmt_mt_snapshot_info& inf = snapInfo[op.pos1];
        for (uint32_t t = 0; t < inf.rm_count; t++) {
          const fmt_mt_stamp& st = snapStamps[inf.rm_first + t];
          s->removes.push_back(Stamp{st.seq, st.client, static_cast<int>(st.kind)});
        }
        insertSegments(getLocalLength(), s, Perspective{false, 0, client}, Stamp{op.seq, client},
                       (op.flags & FMT_MT_F_GROUP_CONT) == 0);
        break;
      }
      insertSegments(op.pos1, s, p, stamp);
      break;
    }
    case FMT_MT_REMOVE:
      markRangeRemoved(op.pos1, op.pos2, p, stamp);
      break;
    case FMT_MT_OBLITERATE:  // {pos1, Before} .. {pos2 - 1, After} (mergeTree.ts:2282-2286)
      obliterateRange(op.pos1, true, op.pos2 - 1, false, p, stamp);
      break;
    case FMT_MT_OBLITERATE_SIDED:  // client.ts:680-700
      obliterateRange(op.pos1, (op.flags & FMT_MT_F_START_BEFORE) != 0, op.pos2,
                      (op.flags & FMT_MT_F_END_BEFORE) != 0, p, stamp);
      break;
    case FMT_MT_ANNOTATE: {
      std::vector<PropChange> kv;
      for (uint32_t i = propsOff[op.payload]; i < propsOff[op.payload + 1]; i++) {
        const uint16_t key = static_cast<uint16_t>(propsKv[i] >> 16), value = static_cast<uint16_t>(propsKv[i] & 0xffff);
        if (value == FMT_MT_VALUE_ADJUST) {  // (key, adjust row in the next word)
          if (i + 1 >= propsOff[op.payload + 1]) throw DataError("adjust entry without its row");
          kv.push_back(PropChange{key, 0, static_cast<int32_t>(propsKv[++i])});
        } else {
          kv.push_back(PropChange{key, value, -1});
        }
      }
      annotateRange(op.pos1, op.pos2, kv, p, stamp);
      break;
    }
    default:
      throw DataError("unsupported op type");
  }
}

// ------------------------------------------------------------------------------------------------
// Zamboni (zamboni.ts:33-213)
// ------------------------------------------------------------------------------------------------
static bool canAppendText(const Seg* prev, const Seg* seg) {
  // textSegment.ts:76-83 (TextSegment.is(segment)); Marker.canAppend is false (mergeTreeNodes.ts:557-559)
  if (prev->marker || seg->marker) return false;
  if (!prev->text.empty() && prev->text.back() == u'\n') return false;
  return prev->len() <= kTextGranularity || seg->len() <= kTextGranularity;
}

void MergeTree::zamboniSegments() {
  if (!collaborating) return;
  for (int i = 0; i < kZamboniMax; i++) {
    if (heap_.count() == 0) break;
    // segmentToScour?.segment?.propertyManager?.updateMsn(minSeq) on the peeked entry (zamboni.ts:44)
    if (heap_.peek().seg->pm) updateMsn(*heap_.peek().seg->pm, minSeq);
    if (heap_.peek().maxSeq > minSeq) break;
    LruHeap::Entry e = heap_.get();
    Block* block = e.seg->parent;
    if (block != nullptr && block->needsScour != 0) {
      std::vector<Node*> hold;
      scourNode(block, hold);
      block->needsScour = 0;
      const int newCount = static_cast<int>(hold.size());
      if (newCount < block->childCount) {
        block->childCount = newCount;
        for (int j = 0; j < kMaxNodesInBlock; j++) block->children[j] = nullptr;
        for (int j = 0; j < newCount; j++) assignChild(block, hold[j], j);
        if (block->childCount < kMaxNodesInBlock / 2 && block->parent != nullptr)
          packParent(block->parent);
      }
    }
  }
}

void MergeTree::scourNode(Block* node, std::vector<Node*>& hold) {
  Seg* prev = nullptr;
  const Stamp minStamp{minSeq, kNonCollabClient};
  const Perspective lp = localPerspective();
  for (int k = 0; k < node->childCount; k++) {
    Node* child = node->children[k];
    if (!child->isLeaf || !static_cast<Seg*>(child)->groups.empty()) {  // pending local ops hold a leaf (zamboni.ts:148)
      hold.push_back(child);
      prev = nullptr;
      continue;
    }
    Seg* seg = static_cast<Seg*>(child);
    if (!seg->removed()) {
      if (stampLte(seg->ins, minStamp)) {
        const int l = leafLength(seg, lp);
        const bool positive = (l == kUndefinedLen ? 0 : l) > 0;
        if (prev != nullptr && canAppendText(prev, seg) && matchProperties(prev->props, seg->props) &&
            positive) {
          for (LRef* r : seg->refs) {  // LocalReferenceCollection.append (localReference.ts:233-251)
            r->seg = prev;
            r->offset += prev->len();
            prev->refs.push_back(r);
          }
          seg->refs.clear();
          prev->text += seg->text;  // BaseSegment.append + TextSegment.append
          seg->parent = nullptr;    // removeMergeNodeInfo
        } else {
          hold.push_back(seg);
          prev = positive ? seg : nullptr;
        }
      } else {
        hold.push_back(seg);
        prev = nullptr;
      }
    } else {
      if (stampLte(seg->removes[0], minStamp)) {
        if (seg->marker) unlinkMarker(seg);  // zamboni.ts:202-204
        seg->parent = nullptr;  // unlinked
      } else {
        hold.push_back(seg);
      }
      prev = nullptr;
    }
  }
}

void MergeTree::packParent(Block* parent) {
  std::vector<Node*> hold;
  for (int i = 0; i < parent->childCount; i++) {
    Block* child = static_cast<Block*>(parent->children[i]);
    scourNode(child, hold);
    child->parent = nullptr;
  }
  for (int j = 0; j < kMaxNodesInBlock; j++) parent->children[j] = nullptr;
  if (!hold.empty()) {
    const int total = static_cast<int>(hold.size());
    constexpr int half = kMaxNodesInBlock / 2;
    int childCount = std::min(kMaxNodesInBlock - 1, total / half);
    if (childCount < 1) childCount = 1;
    const int base = total / childCount;
    int remainder = total % childCount;
    int packed = 0;
    for (int b = 0; b < childCount; b++) {
      int n = base;
      if (remainder > 0) {
        n++;
        remainder--;
      }
      Block* pb = makeBlock(n);
      for (int j = 0; j < n; j++) assignChild(pb, hold[packed++], j);
      assignChild(parent, pb, b);
    }
    parent->childCount = childCount;
  } else {
    parent->childCount = 0;
  }
  if (parent->childCount < kMaxNodesInBlock / 2 && parent->parent != nullptr) {
    packParent(parent->parent);
  }
}

// ------------------------------------------------------------------------------------------------
// Remote-perspective length index (BlockIdx, see mergetree.hpp)
// ------------------------------------------------------------------------------------------------
namespace {
int rm1Of(const Seg* s) { return s->removed() ? s->removes[0].seq : 0x7fffffff; }
bool removedByClient(const Seg* s, int c) {
  for (const Stamp& r : s->removes)
    if (r.client == c) return true;
  return false;
}
void checkAcked(const Seg* s) {
  if (s->ins.seq == kUnassignedSeq) throw DataError("length index: unacknowledged insert");
  for (const Stamp& r : s->removes)
    if (r.seq == kUnassignedSeq) throw DataError("length index: unacknowledged remove");
}
// Whether leaf s can still change PriorPerspective(r, c) lengths for some r >= minSeq beyond its events.
bool clientRelevant(const Seg* s, int c, int minSeq) {
  if (s->ins.client == c && s->ins.seq > minSeq) return true;
  return s->removed() && rm1Of(s) > minSeq && removedByClient(s, c);
}
void addClientEntry(BlockIdx& ix, int client, Seg* s) {
  for (auto& e : ix.clients) {
    if (e.first != client) continue;
    for (Seg* t : e.second)
      if (t == s) return;
    e.second.push_back(s);
    return;
  }
  ix.clients.push_back({client, {s}});
}
}  // namespace

void MergeTree::idxMarkDirty(Block* b) {
  if (indexed_) b->idxDirty = true;
}

void MergeTree::idxAppendEvent(Block* b, int seq, int64_t delta) {
  BlockIdx& ix = *b->idx;
  if (seq <= minSeq) {
    ix.k0 += delta;
    return;
  }
  if (!ix.evSeq.empty() && seq < ix.evSeq.back()) {  // out of order: re-index from the children
    b->idxDirty = true;
    return;
  }
  ix.evSeq.push_back(seq);
  ix.evCum.push_back((ix.evCum.empty() ? 0 : ix.evCum.back()) + delta);
  // fold the prefix at or below minSeq into k0 once it is half the list
  if (ix.evSeq.size() >= 64 && ix.evSeq[ix.evSeq.size() / 2] <= minSeq) {
    const size_t k = static_cast<size_t>(std::upper_bound(ix.evSeq.begin(), ix.evSeq.end(), minSeq) - ix.evSeq.begin());
    const int64_t folded = ix.evCum[k - 1];
    ix.k0 += folded;
    ix.evSeq.erase(ix.evSeq.begin(), ix.evSeq.begin() + static_cast<long>(k));
    ix.evCum.erase(ix.evCum.begin(), ix.evCum.begin() + static_cast<long>(k));
    for (int64_t& c : ix.evCum) c -= folded;
  }
}

void MergeTree::idxAddClient(Block* b, int client, Seg* s) {
  if (client < 0) return;  // LocalClientId / NonCollabClient never query
  addClientEntry(*b->idx, client, s);
}

void MergeTree::idxLeafTerms(Seg* s, BlockIdx& ix) {
  checkAcked(s);
  const int64_t len = s->len();
  const int ins = s->ins.seq;
  if (ins <= minSeq) ix.k0 += len;
  else ix.evSeq.push_back(ins), ix.evCum.push_back(len);  // (seq, delta): sorted and summed by idxRebuild
  if (s->removed()) {
    const int m = std::max(ins, rm1Of(s));
    if (m <= minSeq) ix.k0 -= len;
    else ix.evSeq.push_back(m), ix.evCum.push_back(-len);
  }
  if (s->ins.client >= 0 && clientRelevant(s, s->ins.client, minSeq)) addClientEntry(ix, s->ins.client, s);
  for (const Stamp& r : s->removes)
    if (r.client >= 0 && clientRelevant(s, r.client, minSeq)) addClientEntry(ix, r.client, s);
}

void MergeTree::idxRebuild(Block* b) {
  auto ix = std::make_unique<BlockIdx>();
  for (int i = 0; i < b->childCount; i++) {
    Node* n = b->children[i];
    if (n->isLeaf) {
      idxLeafTerms(static_cast<Seg*>(n), *ix);
      continue;
    }
    Block* c = static_cast<Block*>(n);
    if (!c->idx || c->idxDirty) idxRebuild(c);
    const BlockIdx& ci = *c->idx;
    ix->k0 += ci.k0;
    for (size_t j = 0; j < ci.evSeq.size(); j++) {
      const int64_t d = ci.evCum[j] - (j ? ci.evCum[j - 1] : 0);
      if (ci.evSeq[j] <= minSeq) ix->k0 += d;
      else ix->evSeq.push_back(ci.evSeq[j]), ix->evCum.push_back(d);
    }
    for (const auto& e : ci.clients)
      for (Seg* t : e.second)
        if (clientRelevant(t, e.first, minSeq)) addClientEntry(*ix, e.first, t);
  }
  // (seq, delta) pairs → sorted by seq with prefix sums
  std::vector<std::pair<int, int64_t>> ev(ix->evSeq.size());
  for (size_t j = 0; j < ev.size(); j++) ev[j] = {ix->evSeq[j], ix->evCum[j]};
  std::stable_sort(ev.begin(), ev.end(), [](const auto& a, const auto& c) { return a.first < c.first; });
  int64_t cum = 0;
  for (size_t j = 0; j < ev.size(); j++) {
    cum += ev[j].second;
    ix->evSeq[j] = ev[j].first;
    ix->evCum[j] = cum;
  }
  b->idx = std::move(ix);
  b->idxDirty = false;
}

int64_t MergeTree::idxLength(Block* b, const Perspective& p) {
  if (!b->idx || b->idxDirty) idxRebuild(b);
  BlockIdx& ix = *b->idx;
  const int r = p.refSeq, c = p.client;
  const size_t k = static_cast<size_t>(std::upper_bound(ix.evSeq.begin(), ix.evSeq.end(), r) - ix.evSeq.begin());
  int64_t len = ix.k0 + (k ? ix.evCum[k - 1] : 0);
  for (auto& e : ix.clients) {
    if (e.first != c) continue;
    auto& v = e.second;
    size_t w = 0;
    for (size_t j = 0; j < v.size(); j++) {
      Seg* s = v[j];
      if (!clientRelevant(s, c, minSeq)) continue;  // dropped lazily
      v[w++] = s;
      const int ins = s->ins.seq, rm1 = rm1Of(s);
      const bool inR = removedByClient(s, c);
      if (inR && ins <= r && r < rm1) len -= s->len();
      if (!inR && s->ins.client == c && ins > r && rm1 > r) len += s->len();
    }
    v.resize(w);
    break;
  }
  return len;
}

void MergeTree::idxOnNewLeaf(Seg* s) {
  checkAcked(s);
  const int64_t len = s->len();
  for (Block* a = s->parent; a != nullptr; a = a->parent) {
    if (!a->idx || a->idxDirty) continue;  // re-indexed from its children on next use
    idxAppendEvent(a, s->ins.seq, len);
    if (s->removed()) idxAppendEvent(a, std::max(s->ins.seq, rm1Of(s)), -len);
    if (!a->idx || a->idxDirty) continue;
    if (clientRelevant(s, s->ins.client, minSeq)) idxAddClient(a, s->ins.client, s);
    for (const Stamp& r : s->removes)
      if (clientRelevant(s, r.client, minSeq)) idxAddClient(a, r.client, s);
  }
}

void MergeTree::idxOnSplit(Seg* left, Seg* right) {
  // the parts' lengths still sum to the original's: events stand; the right part needs the left
  // part's client entries
  for (Block* a = right->parent; a != nullptr; a = a->parent) {
    if (!a->idx || a->idxDirty) continue;
    if (clientRelevant(right, right->ins.client, minSeq)) idxAddClient(a, right->ins.client, right);
    for (const Stamp& r : right->removes)
      if (clientRelevant(right, r.client, minSeq)) idxAddClient(a, r.client, right);
  }
  (void)left;
}

void MergeTree::idxOnRemove(Seg* s, int client, bool wasRemoved) {
  checkAcked(s);
  for (Block* a = s->parent; a != nullptr; a = a->parent) {
    if (!a->idx || a->idxDirty) continue;
    if (!wasRemoved) idxAppendEvent(a, std::max(s->ins.seq, rm1Of(s)), -static_cast<int64_t>(s->len()));
    if (!a->idx || a->idxDirty) continue;
    if (clientRelevant(s, client, minSeq)) idxAddClient(a, client, s);
  }
}

// ------------------------------------------------------------------------------------------------
// Readouts
// ------------------------------------------------------------------------------------------------
std::u16string MergeTree::getText() const {
  std::u16string out;
  const Perspective lp = localPerspective();
  const int len = getLocalLength();
  nodeMap(lp, 0, len, [&](Seg* s) {
    if (!s->marker) out += s->text;  // getText collects TextSegments only (MergeTreeTextHelper.ts:60-87)
  });
  return out;
}

void MergeTree::collectLeaves(std::vector<const Seg*>& out, std::vector<int>& blockOfLeaf,
                              int* nLeafBlocks, int* depth) const {
  int blocks = 0;
  int maxDepth = 0;
  auto walk = [&](auto&& self, const Block* b, int d) -> void {
    maxDepth = std::max(maxDepth, d);
    bool leafBlock = false;
    for (int i = 0; i < b->childCount; i++) {
      const Node* n = b->children[i];
      if (n->isLeaf) {
        leafBlock = true;
        out.push_back(static_cast<const Seg*>(n));
        blockOfLeaf.push_back(blocks);
      } else {
        self(self, static_cast<const Block*>(n), d + 1);
      }
    }
    if (leafBlock) blocks++;
  };
  walk(walk, root_, 1);
  *nLeafBlocks = blocks;
  *depth = maxDepth;
}

// JSON.stringify of a number (ECMA-262 Number::toString): the shortest %.*e digits that read back
// as x, laid out in decimal for 1e-7 <= |x| < 1e21, else with an unpadded exponent; NaN / Infinity
// are null, -0 is 0. (The oracle's own restatement; csrc/jsnum.h is the product's.)
std::string jsNumberText(double x) {
  if (std::isnan(x) || std::isinf(x)) return "null";
  if (x == 0) return "0";
  if (x < 0) return "-" + jsNumberText(-x);
  char buf[64];
  for (int prec = 1; prec <= 17; prec++) {
    std::snprintf(buf, sizeof buf, "%.*e", prec - 1, x);
    if (std::strtod(buf, nullptr) == x) break;
  }
  std::string mant, exps(std::strchr(buf, 'e') + 1);
  for (const char* q = buf; *q != 'e'; q++)
    if (*q >= '0' && *q <= '9') mant.push_back(*q);
  while (mant.size() > 1 && mant.back() == '0') mant.pop_back();
  const int k = static_cast<int>(mant.size()), n = std::atoi(exps.c_str()) + 1;
  if (k <= n && n <= 21) return mant + std::string(n - k, '0');
  if (0 < n && n <= 21) return mant.substr(0, n) + "." + mant.substr(n);
  if (-6 < n && n <= 0) return "0." + std::string(-n, '0') + mant;
  return mant.substr(0, 1) + (k > 1 ? "." + mant.substr(1) : "") + "e" + (n - 1 >= 0 ? "+" : "-") +
         std::to_string(std::abs(n - 1));
}

// JSON object of a property map: array-index keys first ascending, then insertion order. Computed
// annotate-adjust values (ids from FMT_MT_VALUE_COMPUTED) are numbers of `numbers`.
static void emitProps(std::string& out, const PropMap& pm, const std::vector<std::string>& keys,
                      const std::vector<std::string>& values, const std::vector<double>& numbers) {
  std::vector<std::pair<uint64_t, size_t>> idx;
  std::vector<size_t> rest;
  for (size_t i = 0; i < pm.kv.size(); i++) {
    uint64_t v;
    if (isArrayIndexKey(keys.at(pm.kv[i].first), &v)) idx.emplace_back(v, i);
    else rest.push_back(i);
  }
  std::sort(idx.begin(), idx.end());
  out.push_back('{');
  bool first = true;
  auto one = [&](size_t i) {
    if (!first) out.push_back(',');
    first = false;
    jsonQuoteUtf8(out, keys.at(pm.kv[i].first));
    out.push_back(':');
    const uint16_t v = pm.kv[i].second;
    if (v >= FMT_MT_VALUE_COMPUTED && v - FMT_MT_VALUE_COMPUTED < numbers.size())
      out += jsNumberText(numbers[v - FMT_MT_VALUE_COMPUTED]);
    else
      out += values.at(v);
  };
  for (auto& e : idx) one(e.second);
  for (size_t i : rest) one(i);
  out.push_back('}');
}

Summary MergeTree::summarize(const std::vector<std::string>& keys,
                             const std::vector<std::string>& values, int chunkSize) {
  // extractSync: leaves present at PriorPerspective(minSeq, NonCollabClient), merged while
  // prev.canAppend(seg) && matchProperties (props for raw-only annotations = current props).
  struct Out {
    std::u16string text;
    PropMap props;
    bool marker;
  };
  std::vector<Out> segs;
  const Perspective mp{false, minSeq, kNonCollabClient};
  const int rootLen = nodeLength(root_, mp);
  const int total = rootLen == kUndefinedLen ? 0 : rootLen;
  nodeMap(mp, 0, total, [&](Seg* s) {
    if (!isPresent(s, mp)) return;
    // segment.propertyManager?.getAtSeq(segment.properties, minSeq) ?? segment.properties (:211-212)
    const PropMap props = s->pm ? getAtSeq(s, minSeq) : s->props;
    if (!segs.empty()) {
      Out& prev = segs.back();
      const bool endsNl = !prev.text.empty() && prev.text.back() == u'\n';
      const bool sizeOk = static_cast<int>(prev.text.size()) <= kTextGranularity ||
                          s->len() <= kTextGranularity;
      if (!prev.marker && !s->marker && !endsNl && sizeOk && matchProperties(prev.props, props)) {
        prev.text += s->text;
        return;
      }
    }
    segs.push_back({s->text, props, s->marker});
  });
  long long totalLen = 0;
  for (auto& o : segs) {
    totalLen += static_cast<long long>(o.text.size());
    if (o.props.defined && o.props.kv.empty()) o.props.defined = false;  // {} → undefined
  }

  auto chunk = [&](size_t startIndex, long long approx, bool header, size_t* count,
                   long long* chunkLen) {
    size_t n = 0;
    long long len = 0;
    while (len < approx && startIndex + n < segs.size()) {
      len += static_cast<long long>(segs[startIndex + n].text.size());
      n++;
    }
    std::string j = "{\"chunkStartSegmentIndex\":";
    jsonInt(j, static_cast<long long>(startIndex));
    j += ",\"chunkSegmentCount\":";
    jsonInt(j, static_cast<long long>(n));
    j += ",\"chunkLengthChars\":";
    jsonInt(j, len);
    j += ",\"totalLengthChars\":";
    jsonInt(j, totalLen);
    j += ",\"totalSegmentCount\":";
    jsonInt(j, static_cast<long long>(segs.size()));
    j += ",\"chunkSequenceNumber\":";
    jsonInt(j, minSeq);
    j += ",\"segmentTexts\":[";
    for (size_t i = 0; i < n; i++) {
      if (i) j.push_back(',');
      const Out& o = segs[startIndex + i];
      if (o.marker) {  // Marker.toJSONObject: {marker: {refType}} + props when defined
        j += "{\"marker\":{\"refType\":";
        jsonInt(j, static_cast<long long>(o.text[0]));
        j += "}";
        if (o.props.defined) {
          j += ",\"props\":";
          emitProps(j, o.props, keys, values, numbers);
        }
        j.push_back('}');
      } else if (o.props.defined) {
        j += "{\"text\":";
        jsonQuoteUtf16(j, o.text.data(), o.text.size());
        j += ",\"props\":";
        emitProps(j, o.props, keys, values, numbers);
        j.push_back('}');
      } else {
        jsonQuoteUtf16(j, o.text.data(), o.text.size());
      }
    }
    j.push_back(']');
    if (header) {
      // snapshotChunks.ts:182-204 buildHeaderMetadataForLegacyChunk
      j += ",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}";
      if (len < totalLen) j += ",{\"id\":\"body\"}";
      j += "],\"sequenceNumber\":";
      jsonInt(j, minSeq);
      j += ",\"totalLength\":";
      jsonInt(j, totalLen);
      j += ",\"totalSegmentCount\":";
      jsonInt(j, static_cast<long long>(segs.size()));
      j.push_back('}');
    }
    j.push_back('}');
    *count = n;
    *chunkLen = len;
    return j;
  };
  Summary s;
  size_t c1;
  long long l1;
  s.header = chunk(0, chunkSize, true, &c1, &l1);
  if (c1 < segs.size()) {
    size_t c2;
    long long l2;
    s.body = chunk(c1, totalLen, false, &c2, &l2);
  }
  return s;
}

}  // namespace orc
