// mt_engine.h — merge-tree observer replay for ONE document on ONE wavefront (gfx950 wave64).
//
// Reference semantics (packages/dds/merge-tree/src): Client.applyMsg → applyRemoteOp
// (client.ts:1291-1379) → MergeTree.insertSegments / markRangeRemoved / annotateRange
// (mergeTree.ts:1484-1517, 2292-2383, 2009-2081), the inserting walk (mergeTree.ts:1811-1987),
// zamboni (zamboni.ts:33-213) with its LRU heap (core-utils/src/heap.ts:54-182), and
// updateSeqNumbers / setMinSeq (client.ts:1381-1391, mergeTree.ts:1147-1166).
//
// MI355X data layout (what replaces the JS object tree):
//   * Leaves live in VGPRs, in document order: lane l holds leaves [8l, 8l+8), five 32-bit words
//     each (W0 len|block|props, W1 insert seq, W2 first-remove seq, W3 remove-client mask,
//     W4 leaf id|insert client). 40 VGPRs hold up to 512 leaves. A perspective's visible length
//     of every leaf, its prefix sums, and every "which leaf holds position p" question are then
//     lane-local arithmetic plus one wave scan / ballot: no tree walk and no partial-lengths index
//     (the reference's PartialSequenceLengths is only an index whose value must equal the sum of
//     leaf lengths, partialLengths.ts:1189-1240). Insert/delete of a leaf is a one-slot shift of
//     the register array (one cross-lane shuffle per word).
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

namespace fmt_mt {

constexpr int E = 8;                 // leaves per lane
constexpr int kCapLeaves = 64 * E;   // 512
constexpr int kCapChars = 2048;      // UTF-16 units per document (tombstones included)
constexpr int kMaxBlocks = 128;
constexpr int kHeapCap = 255;
constexpr int kPropCap = 32;
constexpr int kMaxClient = 31;       // remove-client set is a 32-bit mask
constexpr int kMaxNodes = 8;         // MaxNodesInBlock (mergeTreeNodes.ts:248)
constexpr int kGranularity = 256;    // TextSegmentGranularity (textSegment.ts:21)
constexpr uint32_t kNoBlk = 0xFF;
constexpr uint32_t kPropsUndef = 0xFF;
constexpr int32_t kNotRemoved = 0x7fffffff;

struct Blk {
  uint8_t count;
  uint8_t parent;
  uint8_t leaf;        // children are leaves
  int8_t needsScour;   // -1 undefined, 0 false, 1 true
  uint8_t child[kMaxNodes];
};

struct HeapEnt {
  int32_t maxSeq;
  uint32_t leafId;
};

struct PropSet {
  uint32_t n;
  uint32_t kv[FMT_MT_PROPS_MAX];
};

// Per-wave LDS state.
struct Scratch {
  uint16_t chars[kCapChars];
  Blk blk[kMaxBlocks];
  HeapEnt heap[kHeapCap + 1];  // 1-based
  PropSet props[kPropCap];
  uint8_t freeList[kMaxBlocks];
  uint32_t tmp[64];
};

// Leaf word fields.
FMT_DEV uint32_t fLen(uint32_t w0) { return w0 & 0xFFFFu; }
FMT_DEV uint32_t fBlk(uint32_t w0) { return (w0 >> 16) & 0xFFu; }
FMT_DEV uint32_t fProps(uint32_t w0) { return w0 >> 24; }
FMT_DEV uint32_t mkW0(uint32_t len, uint32_t blk, uint32_t props) { return len | (blk << 16) | (props << 24); }
FMT_DEV uint32_t fId(uint32_t w4) { return w4 & 0xFFFFFFu; }
FMT_DEV int32_t fClient(uint32_t w4) { return static_cast<int32_t>(static_cast<int8_t>(w4 >> 24)); }
FMT_DEV uint32_t mkW4(uint32_t id, int32_t client) { return (id & 0xFFFFFFu) | (static_cast<uint32_t>(client & 0xFF) << 24); }

struct LeafRec {
  uint32_t w[5];
};

struct DocInputs {
  const fmt_mt_op* ops;
  uint64_t begin, end;
  const uint16_t* text;
  uint32_t initOff, initLen;
  const uint32_t* propsOff;
  const uint32_t* propsKv;
  uint32_t nPropsOps;
};

struct DocOutputs {
  fmt_mt_doc_result* header;
  fmt_mt_leaf* leaves;    // kCapLeaves entries
  uint16_t* chars;        // kCapChars entries
  fmt_mt_propset* props;  // kPropCap entries
};

// Diagnostic build only (FMT_PROFILE=1): per-phase shader-clock totals, see stamp().
#ifndef FMT_PROFILE
#define FMT_PROFILE 0
#endif
enum ProfCat { kPfOpLoad, kPfScan, kPfSplit, kPfInsert, kPfRange, kPfLru, kPfZamboniOp, kPfWindow, kPfOutput, kPfCount };

class Doc {
 public:
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
  Lane<V8> W[5];  // W[f] element e = leaf lane*E + e
  Scratch* s;
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
  DocInputs in;

  // ------------------------------------------------------------------ leaf array primitives
  FMT_DEV Lane<uint32_t> selectE(const Lane<V8>& arr, int e) const {
    Lane<uint32_t> r;
    FOR_LANES(l) {
      V8 t = LANE(arr);
      launder(t);  // keep the dynamic index on a register value (v_movrels), never a scratch GEP
      LANE(r) = t[e];
    }
    return r;
  }

  FMT_DEV uint32_t readField(int j, int f) const { return readlane(selectE(W[f], j % E), j / E); }

  FMT_DEV LeafRec readLeaf(int j) const {
    LeafRec r;
    r.w[0] = readField(j, 0);
    r.w[1] = readField(j, 1);
    r.w[2] = readField(j, 2);
    r.w[3] = readField(j, 3);
    r.w[4] = readField(j, 4);
    return r;
  }

  FMT_DEV void writeField(int j, int f, uint32_t v) {
    const int lane = j / E, e = j % E;
    FOR_LANES(l) {
      if (l == lane) {
        V8 t = LANE(W[f]);
        launder(t);
        t[e] = v;
        LANE(W[f]) = t;
      }
    }
  }

  // One field of the leaf array shifted up by one slot from index k, `rv` written at k.
  FMT_DEV static void shiftUpField(Lane<V8>& w, int k, uint32_t rv) {
    const Lane<uint32_t> prev7 = shflUp1(selectLast(w));
    FOR_LANES(l) {
      V8 v = LANE(w);
#pragma unroll
      for (int e = E - 1; e >= 1; e--) {
        const int idx = l * E + e;
        v[e] = idx > k ? v[e - 1] : (idx == k ? rv : v[e]);
      }
      const int idx0 = l * E;
      v[0] = idx0 > k ? LANE(prev7) : (idx0 == k ? rv : v[0]);
      LANE(w) = v;
    }
  }

  // One field of the leaf array shifted down by one slot onto index k.
  FMT_DEV static void shiftDownField(Lane<V8>& w, int k) {
    const Lane<uint32_t> next0 = shflDown1(selectFirst(w));
    FOR_LANES(l) {
      V8 v = LANE(w);
#pragma unroll
      for (int e = 0; e < E - 1; e++) {
        const int idx = l * E + e;
        v[e] = idx >= k ? v[e + 1] : v[e];
      }
      const int idx7 = l * E + E - 1;
      v[E - 1] = idx7 >= k ? LANE(next0) : v[E - 1];
      LANE(w) = v;
    }
  }

  FMT_DEV static Lane<uint32_t> selectLast(const Lane<V8>& w) {
    Lane<uint32_t> r;
    FOR_LANES(l) { LANE(r) = LANE(w)[E - 1]; }
    return r;
  }

  FMT_DEV static Lane<uint32_t> selectFirst(const Lane<V8>& w) {
    Lane<uint32_t> r;
    FOR_LANES(l) { LANE(r) = LANE(w)[0]; }
    return r;
  }

  // Insert `rec` at index k, shifting leaves k.. up by one.
  FMT_DEV bool insertLeafAt(int k, const LeafRec& rec) {
    if (n >= kCapLeaves) return fail(FMT_E_CAPACITY);
    shiftUpField(W[0], k, rec.w[0]);
    shiftUpField(W[1], k, rec.w[1]);
    shiftUpField(W[2], k, rec.w[2]);
    shiftUpField(W[3], k, rec.w[3]);
    shiftUpField(W[4], k, rec.w[4]);
    n++;
    return true;
  }

  // Remove the leaf at index k, shifting leaves k+1.. down by one.
  FMT_DEV void deleteLeafAt(int k) {
    shiftDownField(W[0], k);
    shiftDownField(W[1], k);
    shiftDownField(W[2], k);
    shiftDownField(W[3], k);
    shiftDownField(W[4], k);
    n--;
  }

  // Exclusive prefix of per-leaf values (document order); returns the total.
  FMT_DEV uint32_t scanLeaves(const Lane<V8>& vals, Lane<V8>& excl) const {
    Lane<uint32_t> laneSum;
    FOR_LANES(l) {
      uint32_t t = 0;
#pragma unroll
      for (int e = 0; e < E; e++) t += LANE(vals)[e];
      LANE(laneSum) = t;
    }
    uint32_t total;
    const Lane<uint32_t> base = waveExclusiveSum(laneSum, &total);
    FOR_LANES(l) {
      uint32_t acc = LANE(base);
#pragma unroll
      for (int e = 0; e < E; e++) {
        LANE(excl)[e] = acc;
        acc += LANE(vals)[e];
      }
    }
    return total;
  }

  // Visible length of every leaf from PriorPerspective(refSeq, client) (perspective.ts:80-93).
  // Leaves removed at/below minSeq are never present for such a perspective (refSeq >= minSeq).
  FMT_DEV void visLengths(int refSeq, int client, Lane<V8>& vis) const {
    FOR_LANES(l) {
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int idx = l * E + e;
        const uint32_t w0 = LANE(W[0])[e];
        const int32_t ins = static_cast<int32_t>(LANE(W[1])[e]);
        const int32_t rm = static_cast<int32_t>(LANE(W[2])[e]);
        const uint32_t mask = LANE(W[3])[e];
        const int32_t ic = fClient(LANE(W[4])[e]);
        const bool present = idx < n && (ins <= refSeq || ic == client) &&
                             !(rm <= refSeq || ((mask >> client) & 1u));
        LANE(vis)[e] = present ? fLen(w0) : 0u;
      }
    }
  }

  // Char offset of every leaf (all leaves, tombstones included).
  FMT_DEV void charStarts(Lane<V8>& cst) const {
    Lane<V8> lens;
    FOR_LANES(l) {
#pragma unroll
      for (int e = 0; e < E; e++) LANE(lens)[e] = (l * E + e) < n ? fLen(LANE(W[0])[e]) : 0u;
    }
    scanLeaves(lens, cst);
  }

  FMT_DEV uint32_t charStartOf(int j) const {
    Lane<V8> cst;
    charStarts(cst);
    return j >= n ? static_cast<uint32_t>(nChars) : readlane(selectE(cst, j % E), j / E);
  }

  // First leaf index with block id b (leaf blocks are contiguous runs), or -1.
  FMT_DEV int firstLeafOf(uint32_t b) const {
    Lane<uint32_t> firstE;
    Lane<bool> has;
    FOR_LANES(l) {
      uint32_t fe = E;
#pragma unroll
      for (int e = E - 1; e >= 0; e--)
        if (l * E + e < n && fBlk(LANE(W[0])[e]) == b) fe = e;
      LANE(firstE) = fe;
      LANE(has) = fe < E;
    }
    const uint64_t m = ballot(has);
    if (m == 0) return -1;
    const int lane = ctz64(m);
    return lane * E + static_cast<int>(readlane(firstE, lane));
  }

  FMT_DEV int findLeafById(uint32_t id) const {
    Lane<uint32_t> hitE;
    Lane<bool> has;
    FOR_LANES(l) {
      uint32_t he = E;
#pragma unroll
      for (int e = 0; e < E; e++)
        if (l * E + e < n && fId(LANE(W[4])[e]) == id) he = e;
      LANE(hitE) = he;
      LANE(has) = he < E;
    }
    const uint64_t m = ballot(has);
    if (m == 0) return -1;
    const int lane = ctz64(m);
    return lane * E + static_cast<int>(readlane(hitE, lane));
  }

  // ------------------------------------------------------------------ chars (LDS, doc order)
  FMT_DEV void charsShiftUp(int from, int by) {  // chars[from..nChars) → chars[from+by..)
    const int count = nChars - from;
    for (int top = count - 1; top >= 0; top -= 64) {
      Lane<uint32_t> v;
      FOR_LANES(l) {
        const int t = top - l;
        LANE(v) = t >= 0 ? s->chars[from + t] : 0u;
      }
      waveSync();
      FOR_LANES(l) {
        const int t = top - l;
        if (t >= 0) s->chars[from + t + by] = static_cast<uint16_t>(LANE(v));
      }
      waveSync();
    }
  }

  FMT_DEV void charsShiftDown(int from, int by) {  // chars[from..nChars) → chars[from-by..)
    for (int base = from; base < nChars; base += 64) {
      Lane<uint32_t> v;
      FOR_LANES(l) {
        const int t = base + l;
        LANE(v) = t < nChars ? s->chars[t] : 0u;
      }
      waveSync();
      FOR_LANES(l) {
        const int t = base + l;
        if (t < nChars) s->chars[t - by] = static_cast<uint16_t>(LANE(v));
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
    Blk& b = s->blk[id];
    b.count = 0;
    b.parent = kNoBlk;
    b.leaf = leafType;
    b.needsScour = -1;
    waveSync();
    return id;
  }

  FMT_DEV void freeBlk(int id) {
    s->freeList[nFree++] = static_cast<uint8_t>(id);
    waveSync();
  }

  // Re-tag leaves [first, first+count) with block id b.
  FMT_DEV void tagLeaves(int first, int count, uint32_t b) {
    FOR_LANES(l) {
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int idx = l * E + e;
        if (idx >= first && idx < first + count) {
          const uint32_t w0 = LANE(W[0])[e];
          LANE(W[0])[e] = mkW0(fLen(w0), b, fProps(w0));
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
          s->blk[nb].child[i] = static_cast<uint8_t>(c);
          s->blk[c].parent = static_cast<uint8_t>(nb);
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
        s->blk[r].child[0] = static_cast<uint8_t>(b);
        s->blk[r].child[1] = static_cast<uint8_t>(nb);
        s->blk[b].parent = static_cast<uint8_t>(r);
        s->blk[nb].parent = static_cast<uint8_t>(r);
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
        s->blk[p].child[i] = static_cast<uint8_t>(c);
      }
      s->blk[p].child[idx + 1] = static_cast<uint8_t>(nb);
      s->blk[nb].parent = static_cast<uint8_t>(p);
      s->blk[p].count = static_cast<uint8_t>(pc + 1);
      waveSync();
      cnt = pc + 1;
      b = p;
    }
  }

  // ------------------------------------------------------------------ LRU heap (heap.ts)
  FMT_DEV void heapSwap(int a, int b) {
    const HeapEnt x = s->heap[a], y = s->heap[b];
    waveSync();
    s->heap[a] = y;
    s->heap[b] = x;
    waveSync();
  }

  FMT_DEV int heapSeq(int k) const { return uni(s->heap[k].maxSeq); }

  FMT_DEV void heapAdd(int maxSeq, uint32_t leafId) {
    if (heapN >= kHeapCap) {
      fail(FMT_E_CAPACITY);
      return;
    }
    heapN++;
    s->heap[heapN].maxSeq = maxSeq;
    s->heap[heapN].leafId = leafId;
    waveSync();
    int k = heapN;
    while (k > 1 && heapSeq(k >> 1) - heapSeq(k) > 0) {
      heapSwap(k, k >> 1);
      k >>= 1;
    }
  }

  FMT_DEV HeapEnt heapGet() {
    heapSwap(1, heapN);
    HeapEnt x;
    x.maxSeq = uni(s->heap[heapN].maxSeq);
    x.leafId = uni(s->heap[heapN].leafId);
    heapN--;
    int k = 1;
    while ((k << 1) <= heapN) {
      int j = k << 1;
      if (j < heapN && heapSeq(j) - heapSeq(j + 1) > 0) j++;
      if (heapSeq(k) - heapSeq(j) <= 0) break;
      heapSwap(k, j);
      k = j;
    }
    return x;
  }

  // ------------------------------------------------------------------ prop sets
  FMT_DEV bool propsMatch(uint32_t a, uint32_t b) const {  // properties.ts:32-61
    if (a == b) return true;
    const uint32_t na = a == kPropsUndef ? 0u : uni(s->props[a].n);
    const uint32_t nb = b == kPropsUndef ? 0u : uni(s->props[b].n);
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
      const uint32_t kv = uni(s->props[a].kv[i]);
      bool found = false;
      for (uint32_t k = 0; k < nb; k++) {
        const uint32_t kv2 = uni(s->props[b].kv[k]);
        if ((kv2 >> 16) == (kv >> 16)) {
          if (kv2 != kv) return false;
          found = true;
        }
      }
      if (!found) return false;
    }
    return true;
  }

  // `seg.properties ??= {}` then raw LWW per key, null deletes (segmentPropertiesManager.ts:188-238).
  FMT_DEV uint32_t applyProps(uint32_t old, uint32_t opId) {
    V4 kv;
    uint32_t cnt = 0;
    if (old != kPropsUndef) {
      cnt = uni(s->props[old].n);
      for (uint32_t i = 0; i < FMT_MT_PROPS_MAX; i++) kv[i] = i < cnt ? uni(s->props[old].kv[i]) : 0u;
    } else {
      for (uint32_t i = 0; i < FMT_MT_PROPS_MAX; i++) kv[i] = 0;
    }
    const uint32_t a = uni(in.propsOff[opId]), b = uni(in.propsOff[opId + 1]);
    for (uint32_t t = a; t < b; t++) {
      const uint32_t e = uni(in.propsKv[t]);
      const uint32_t key = e >> 16;
      uint32_t pos = cnt;
      for (uint32_t i = 0; i < FMT_MT_PROPS_MAX; i++)
        if (i < cnt && (kv[i] >> 16) == key) pos = i;
      if ((e & 0xFFFFu) == 0) {  // null: delete the key
        if (pos < cnt) {
          for (uint32_t i = 0; i + 1 < FMT_MT_PROPS_MAX; i++)
            if (i >= pos && i + 1 < cnt) kv[i] = kv[i + 1];
          cnt--;
        }
      } else if (pos < cnt) {
        for (uint32_t i = 0; i < FMT_MT_PROPS_MAX; i++)
          if (i == pos) kv[i] = e;
      } else {
        if (cnt >= FMT_MT_PROPS_MAX) {
          fail(FMT_E_CAPACITY);
          return 0;
        }
        for (uint32_t i = 0; i < FMT_MT_PROPS_MAX; i++)
          if (i == cnt) kv[i] = e;
        cnt++;
      }
    }
    for (int p = 0; p < nProps; p++) {
      if (uni(s->props[p].n) != cnt) continue;
      bool same = true;
      for (uint32_t i = 0; i < FMT_MT_PROPS_MAX; i++)
        if (i < cnt) same = same && uni(s->props[p].kv[i]) == kv[i];
      if (same) return static_cast<uint32_t>(p);
    }
    if (nProps >= kPropCap) {
      fail(FMT_E_CAPACITY);
      return 0;
    }
    s->props[nProps].n = cnt;
    for (uint32_t i = 0; i < FMT_MT_PROPS_MAX; i++) s->props[nProps].kv[i] = kv[i];
    waveSync();
    return static_cast<uint32_t>(nProps++);
  }

  // ------------------------------------------------------------------ ops
  // addToLRUSet for every hit leaf in document order: only the first hit of each block can add
  // (the first one sets needsScour, mergeTree.ts:812-822).
  FMT_DEV void lruForHits(const Lane<uint32_t>& hits, int seq) {
    // exclusive max-scan of (index << 8 | block) over hit leaves gives each leaf's previous hit
    Lane<int32_t> laneLast;
    FOR_LANES(l) {
      int32_t last = -1;
#pragma unroll
      for (int e = 0; e < E; e++)
        if ((LANE(hits) >> e) & 1u) last = ((l * E + e) << 8) | static_cast<int32_t>(fBlk(LANE(W[0])[e]));
      LANE(laneLast) = last;
    }
    const Lane<int32_t> before = waveExclusiveMax(laneLast, -1);
    Lane<uint32_t> cand;
    Lane<bool> has;
    FOR_LANES(l) {
      int32_t prev = LANE(before);
      uint32_t c = 0;
#pragma unroll
      for (int e = 0; e < E; e++) {
        if ((LANE(hits) >> e) & 1u) {
          const int32_t b = static_cast<int32_t>(fBlk(LANE(W[0])[e]));
          if (prev < 0 || (prev & 0xFF) != b) c |= 1u << e;
          prev = ((l * E + e) << 8) | b;
        }
      }
      LANE(cand) = c;
      LANE(has) = c != 0;
    }
    uint64_t m = ballot(has);
    while (m) {
      const int lane = ctz64(m);
      uint32_t c = readlane(cand, lane);
      while (c) {
        const int e = ctz32(c);
        c &= c - 1;
        const int j = lane * E + e;
        const int b = static_cast<int>(fBlk(readField(j, 0)));
        if (uni(static_cast<int>(s->blk[b].needsScour)) != 1 && seq > curSeq) {
          s->blk[b].needsScour = 1;
          waveSync();
          heapAdd(seq, fId(readField(j, 4)));
          if (status != FMT_OK) return;
        }
      }
      m &= m - 1;
    }
  }

  // One member op of a remote message (client.ts:1291-1327). The phases share one view scan:
  //   phase < nb : ensureIntervalBoundary at pos1 (and pos2) — mergeTree.ts:1798-1808: split the
  //                unique leaf that strictly contains the position in the op's view;
  //   phase == nb: insert (mergeTree.ts:1484-1750) or collect the nodeMap range (mergeTree.ts:
  //                2961-3020) for remove / annotate.
  FMT_DEV void applyOp(const fmt_mt_op& op) {
    const int refSeq = op.ref_seq, client = op.client, seq = op.seq;
    const bool isInsert = op.type == FMT_MT_INSERT;
    const int nb = isInsert ? 1 : 2;
    Lane<uint32_t> hits;
    FOR_LANES(l) { LANE(hits) = 0u; }
    for (int phase = 0;; phase++) {
      Lane<V8> vis, st;
      visLengths(refSeq, client, vis);
      const uint32_t total = scanLeaves(vis, st);
      stamp(kPfScan);
      int insIdx = -1, blk = 0;
      LeafRec rec;
      if (phase < nb) {
        const int pos = phase == 0 ? op.pos1 : op.pos2;
        Lane<uint32_t> hitE;
        Lane<bool> has;
        FOR_LANES(l) {
          uint32_t he = E;
#pragma unroll
          for (int e = 0; e < E; e++) {
            const int sp = static_cast<int>(LANE(st)[e]);
            if (sp < pos && pos < sp + static_cast<int>(LANE(vis)[e])) he = e;
          }
          LANE(hitE) = he;
          LANE(has) = he < E;
        }
        const uint64_t m = ballot(has);
        if (m != 0) {
          const int lane = ctz64(m);
          const int e = static_cast<int>(readlane(hitE, lane));
          const int j = lane * E + e;
          const int offset = pos - static_cast<int>(readlane(selectE(st, e), lane));
          const uint32_t w0 = readField(j, 0), w4 = readField(j, 4);
          rec.w[0] = mkW0(fLen(w0) - static_cast<uint32_t>(offset), fBlk(w0), fProps(w0));
          rec.w[1] = readField(j, 1);
          rec.w[2] = readField(j, 2);
          rec.w[3] = readField(j, 3);
          rec.w[4] = mkW4(nextId++, fClient(w4));
          writeField(j, 0, mkW0(static_cast<uint32_t>(offset), fBlk(w0), fProps(w0)));
          insIdx = j + 1;
          blk = static_cast<int>(fBlk(w0));
        }
      } else if (isInsert) {
        const int pos = op.pos1, len = op.len;
        if (len > 0) {
          // anchor: the first leaf whose view prefix equals pos, leaves removed at/below minSeq
          // skipped except the very last leaf (mergeTree.ts:1862-1875)
          Lane<uint32_t> anchorE;
          Lane<bool> has;
          FOR_LANES(l) {
            uint32_t ae = E;
#pragma unroll
            for (int e = E - 1; e >= 0; e--) {
              const int idx = l * E + e;
              const bool undefinedLen = static_cast<int32_t>(LANE(W[2])[e]) <= minSeq;
              const bool skipped = undefinedLen && idx != n - 1;
              if (idx < n && !skipped && static_cast<int>(LANE(st)[e]) == pos) ae = e;
            }
            LANE(anchorE) = ae;
            LANE(has) = ae < E;
          }
          const uint64_t m = ballot(has);
          if (m != 0) {
            const int lane = ctz64(m);
            insIdx = lane * E + static_cast<int>(readlane(anchorE, lane));
            blk = static_cast<int>(fBlk(readField(insIdx, 0)));
          } else {
            if (pos != static_cast<int>(total)) {  // "MergeTree insert failed" (mergeTree.ts:1629)
              fail(FMT_E_DATA);
              return;
            }
            insIdx = n;
            blk = n > 0 ? static_cast<int>(fBlk(readField(n - 1, 0))) : root;
          }
          if (nChars + len > kCapChars) {
            fail(FMT_E_CAPACITY);
            return;
          }
          const int cpos = static_cast<int>(charStartOf(insIdx));
          charsShiftUp(cpos, len);
          const uint16_t* src = in.text + op.payload;
          FOR_LANES(l) {
            for (int t = l; t < len; t += 64) s->chars[cpos + t] = src[t];
          }
          waveSync();
          nChars += len;
          rec.w[0] = mkW0(static_cast<uint32_t>(len), static_cast<uint32_t>(blk), kPropsUndef);
          rec.w[1] = static_cast<uint32_t>(seq);
          rec.w[2] = static_cast<uint32_t>(kNotRemoved);
          rec.w[3] = 0;
          rec.w[4] = mkW4(nextId++, client);
          if (uni(static_cast<int>(s->blk[blk].count)) == 0) {
            s->blk[blk].leaf = 1;  // an empty root becomes a leaf block
            waveSync();
          }
        }
      } else {
        const int start = op.pos1, end = op.pos2;
        FOR_LANES(l) {
          uint32_t h = 0;
#pragma unroll
          for (int e = 0; e < E; e++) {
            const int sp = static_cast<int>(LANE(st)[e]);
            if (LANE(vis)[e] > 0 && sp >= start && sp < end) h |= 1u << e;
          }
          LANE(hits) = h;
        }
        break;
      }
      if (insIdx >= 0) {
        if (!insertLeafAt(insIdx, rec)) return;
        childAdded(blk);
        if (status != FMT_OK) return;
      }
      stamp(phase < nb ? kPfSplit : kPfInsert);
      if (phase >= nb) {
        if (insIdx >= 0) {
          const int lane = insIdx / E, e = insIdx % E;
          FOR_LANES(l) { LANE(hits) = l == lane ? (1u << e) : 0u; }
        }
        break;
      }
    }
    if (op.type == FMT_MT_REMOVE) {
      // markRangeRemoved (mergeTree.ts:2292-2383): first remove stays the lowest seq
      FOR_LANES(l) {
#pragma unroll
        for (int e = 0; e < E; e++) {
          if ((LANE(hits) >> e) & 1u) {
            const int32_t rm = static_cast<int32_t>(LANE(W[2])[e]);
            LANE(W[2])[e] = static_cast<uint32_t>(rm < seq ? rm : seq);
            LANE(W[3])[e] |= 1u << client;
          }
        }
      }
    } else if (op.type == FMT_MT_ANNOTATE) {
      // annotateRange (mergeTree.ts:2009-2081): one prop-set transition per distinct old set
      Lane<uint32_t> todo = hits;
      for (;;) {
        Lane<bool> has;
        FOR_LANES(l) { LANE(has) = LANE(todo) != 0; }
        const uint64_t m = ballot(has);
        if (m == 0) break;
        const int lane = ctz64(m);
        const int e = ctz32(readlane(todo, lane));
        const uint32_t old = fProps(readField(lane * E + e, 0));
        const uint32_t nw = applyProps(old, op.payload);
        if (status != FMT_OK) return;
        FOR_LANES(l) {
#pragma unroll
          for (int k = 0; k < E; k++) {
            if (((LANE(todo) >> k) & 1u) && fProps(LANE(W[0])[k]) == old) {
              const uint32_t w0 = LANE(W[0])[k];
              LANE(W[0])[k] = mkW0(fLen(w0), fBlk(w0), nw);
              LANE(todo) &= ~(1u << k);
            }
          }
        }
      }
    }
    stamp(kPfRange);
    lruForHits(hits, seq);
    stamp(kPfLru);
  }

  // ------------------------------------------------------------------ zamboni (zamboni.ts)
  // scourNode over leaf block b: drops tombstones removed at/below minSeq and appends acked,
  // same-props, appendable leaves onto the previous kept leaf. Returns the new child count.
  FMT_DEV int scourLeafBlock(int b) {
    const int cnt = uni(static_cast<int>(s->blk[b].count));
    if (cnt == 0) return 0;
    const int first = firstLeafOf(static_cast<uint32_t>(b));
    Lane<V8> cst;
    charStarts(cst);
    // serial decisions over <= 7 leaves: keep, merge into the previous kept leaf, or drop
    uint32_t mergeMask = 0, dropMask = 0;
    int prev = -1;
    uint32_t prevLen = 0, prevProps = 0, prevBlk = 0;
    bool prevNl = false;
    int kept = 0;
    for (int k = 0; k < cnt; k++) {
      const int j = first + k;
      const uint32_t w0 = readField(j, 0);
      const uint32_t len = fLen(w0);
      const int32_t ins = static_cast<int32_t>(readField(j, 1));
      const int32_t rm = static_cast<int32_t>(readField(j, 2));
      if (rm == kNotRemoved) {
        if (ins <= minSeq) {
          const uint32_t cs = readlane(selectE(cst, j % E), j / E);
          const bool lastNl = len > 0 && uni(static_cast<uint32_t>(s->chars[cs + len - 1])) == 10u;
          const bool canAppend = prev >= 0 && !prevNl &&
                                 (prevLen <= static_cast<uint32_t>(kGranularity) ||
                                  len <= static_cast<uint32_t>(kGranularity)) &&
                                 propsMatch(prevProps, fProps(w0)) && len > 0;
          if (canAppend) {
            mergeMask |= 1u << k;
            prevLen += len;
            prevNl = lastNl;
            // the head keeps its index until the deletions below, so its length can be set now
            writeField(prev, 0, mkW0(prevLen, prevBlk, prevProps));
          } else {
            prev = len > 0 ? j : -1;
            prevLen = len;
            prevProps = fProps(w0);
            prevBlk = fBlk(w0);
            prevNl = lastNl;
            kept++;
          }
        } else {
          prev = -1;
          kept++;
        }
      } else {
        if (rm <= minSeq) {
          dropMask |= 1u << k;
        } else {
          kept++;
        }
        prev = -1;
      }
    }
    // remove merged / dropped leaves from the highest index down (lower indices stay valid)
    for (int k = cnt - 1; k >= 0; k--) {
      if ((((mergeMask | dropMask) >> k) & 1u) == 0) continue;
      const int j = first + k;
      if ((dropMask >> k) & 1u) {
        const uint32_t len = fLen(readField(j, 0));
        const int cs = static_cast<int>(readlane(selectE(cst, j % E), j / E));
        charsShiftDown(cs + static_cast<int>(len), static_cast<int>(len));
        nChars -= static_cast<int>(len);
      }
      deleteLeafAt(j);
    }
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
        s->blk[id].parent = static_cast<uint8_t>(p);
        if (leafLevel) {
          tagLeaves(firstLeaf + consumed, cnt, static_cast<uint32_t>(id));
        } else {
          for (int k = 0; k < cnt; k++) {
            const int g = uni(static_cast<int>(s->tmp[consumed + k]));
            s->blk[id].child[k] = static_cast<uint8_t>(g);
            s->blk[g].parent = static_cast<uint8_t>(id);
          }
        }
        s->blk[p].child[q] = static_cast<uint8_t>(id);
        waveSync();
        consumed += cnt;
      }
      s->blk[p].count = static_cast<uint8_t>(nb);
    } else {
      s->blk[p].count = 0;
      if (p == root) s->blk[p].leaf = 1;
    }
    waveSync();
  }

  // zamboni.ts:33-80, with packParent (zamboni.ts:83-139) folded in so that every block scour —
  // the popped block's own and each sibling's during packParent — goes through one call site.
  FMT_DEV void zamboni() {
    for (int i = 0; i < 2; i++) {
      if (heapN == 0) break;
      if (heapSeq(1) > minSeq) break;
      const HeapEnt ent = heapGet();
      const int j = findLeafById(ent.leafId);
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
    FOR_LANES(l) {
      V8 z;
#pragma unroll
      for (int e = 0; e < E; e++) z[e] = 0u;
      LANE(W[0]) = z;
      LANE(W[1]) = z;
      LANE(W[2]) = z;
      LANE(W[3]) = z;
      LANE(W[4]) = z;
    }
    FOR_LANES(l) {
      for (int i = l; i < kMaxBlocks; i += 64) s->freeList[i] = static_cast<uint8_t>(kMaxBlocks - 1 - i);
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
    if (len > kCapChars || len > 0xFFFF) {
      fail(FMT_E_CAPACITY);
      return;
    }
    const uint16_t* src = in.text + in.initOff;
    FOR_LANES(l) {
      for (int t = l; t < len; t += 64) s->chars[t] = src[t];
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
      }
    }
    n = 1;
    s->blk[root].count = 1;
    waveSync();
  }

  FMT_DEV void replay() {
    stamp(kPfOutput);
    for (uint64_t i = in.begin; i < in.end; i++) {
      fmt_mt_op op = in.ops[i];
      op.seq = uni(op.seq);
      op.ref_seq = uni(op.ref_seq);
      op.min_seq = uni(op.min_seq);
      op.pos1 = uni(op.pos1);
      op.pos2 = uni(op.pos2);
      op.payload = uni(op.payload);
      const uint32_t lenClientType = uni(static_cast<uint32_t>(op.len) | (static_cast<uint32_t>(op.client) << 16) |
                                         (static_cast<uint32_t>(op.type) << 24));
      op.len = static_cast<uint16_t>(lenClientType & 0xFFFF);
      op.client = static_cast<uint8_t>((lenClientType >> 16) & 0xFF);
      op.type = static_cast<uint8_t>(lenClientType >> 24);
      stamp(kPfOpLoad);
      if (op.client > kMaxClient || op.type > FMT_MT_ANNOTATE) fail(FMT_E_UNSUPPORTED);
      else if (op.type == FMT_MT_ANNOTATE && op.payload >= in.nPropsOps) fail(FMT_E_DATA);
      else applyOp(op);
      const bool lastMember = i + 1 == in.end || (uni(in.ops[i + 1].flags) & FMT_MT_F_GROUP_CONT) == 0;
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
          if (op.min_seq <= minSeq) break;
          minSeq = op.min_seq;
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
    // char offsets and leaf-block ordinals
    Lane<V8> cst;
    charStarts(cst);
    Lane<V8> startFlag, ord;
    const Lane<uint32_t> prevBlk7 = shflUp1(selectE(W[0], E - 1));
    FOR_LANES(l) {
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int idx = l * E + e;
        const uint32_t b = fBlk(LANE(W[0])[e]);
        const uint32_t pb = e == 0 ? fBlk(LANE(prevBlk7)) : fBlk(LANE(W[0])[e - 1]);
        LANE(startFlag)[e] = idx < n && (idx == 0 || b != pb) ? 1u : 0u;
      }
    }
    const uint32_t nLeafBlocks = scanLeaves(startFlag, ord);
    uint32_t visible = 0;
    {
      Lane<V8> vlen, tmp;
      FOR_LANES(l) {
#pragma unroll
        for (int e = 0; e < E; e++) {
          const int idx = l * E + e;
          const bool live = idx < n && static_cast<int32_t>(LANE(W[2])[e]) == kNotRemoved;
          LANE(vlen)[e] = live ? fLen(LANE(W[0])[e]) : 0u;
        }
      }
      visible = scanLeaves(vlen, tmp);
    }
    FOR_LANES(l) {
#pragma unroll
      for (int e = 0; e < E; e++) {
        const int idx = l * E + e;
        if (idx < n) {
          fmt_mt_leaf L;
          const uint32_t w0 = LANE(W[0])[e];
          L.ins_seq = static_cast<int32_t>(LANE(W[1])[e]);
          L.rm_seq = static_cast<int32_t>(LANE(W[2])[e]);
          L.rm_clients = LANE(W[3])[e];
          L.char_off = LANE(cst)[e];
          L.len = static_cast<uint16_t>(fLen(w0));
          L.ins_client = static_cast<int16_t>(fClient(LANE(W[4])[e]));
          L.props = fProps(w0) == kPropsUndef ? 0xFFFFu : static_cast<uint16_t>(fProps(w0));
          L.block = static_cast<uint16_t>(LANE(ord)[e] + LANE(startFlag)[e] - 1u);
          L.pad = 0;
          out.leaves[idx] = L;
        }
      }
    }
    FOR_LANES(l) {
      for (int t = l; t < nChars; t += 64) out.chars[t] = s->chars[t];
      for (int p = l; p < nProps; p += 64) {
        fmt_mt_propset ps;
        ps.n = s->props[p].n;
#pragma unroll
        for (int k = 0; k < FMT_MT_PROPS_MAX; k++) ps.kv[k] = s->props[p].kv[k];
        out.props[p] = ps;
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
        h.pad[0] = 0;
        h.pad[1] = 0;
        *out.header = h;
      }
    }
  }

  FMT_DEV void run(const DocInputs& inputs, const DocOutputs& out) {
#if FMT_PROFILE && FMT_GPU
    profT = __builtin_amdgcn_s_memtime();
#endif
    in = inputs;
    init();
    loadInitial();
    if (status == FMT_OK) replay();
    writeOutputs(out);
    stamp(kPfOutput);
  }
};

}  // namespace fmt_mt
