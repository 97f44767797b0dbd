// adjust.h — annotate-adjust value folding shared by the merge-tree tiers (mt_engine.h) and the
// huge-document engine (huge_engine.h): the batch's adjust tables in device memory and
// computePropertyValue (segmentPropertiesManager.ts:54-78) over them.
#pragma once

#include "../../include/fmt.h"
#include "wave.h"

namespace fmt_mt {

// legacyProps entry (every leaf of the document) when the getAtSeq view of an annotate-adjust document
// did not fit its prop-set table: the replay state stands, its legacy summary reports FMT_E_CAPACITY
constexpr uint16_t kLegacyUnavailable = 0xFFFEu;

// Annotate-adjust tables of a batch (device memory): the rows, the number of each host value id
// (NaN: not a number), the host's numbers ascending with their value ids, and per document a slab
// of computed numbers (numOffsets) with its count (numCount, kept in memory across tiers).
struct AdjustTables {
  const fmt_mt_adjust* adjusts;
  uint32_t nAdjusts;
  uint32_t nValues;
  const double* valueNum;
  const double* numSorted;
  const uint32_t* numSortedId;
  uint32_t nNumSorted;
  uint32_t pad;
  // document-local value ids (fmt_mt_batch.doc_value_base): per document its value base (nDocs + 1),
  // and its own host numbers numSorted[numSortedOffs[doc] .. numSortedOffs[doc + 1]) with local ids;
  // nullptr: batch-global ids, one sorted list
  const uint32_t* valueBase;
  const uint32_t* numSortedOffs;
  double* nums;
  const uint64_t* numOffsets;  // nDocs + 1
  uint32_t* numCount;          // nDocs
  // per document: its leaves' PropertiesManager records (Doc::pm*), 4 words each, at pmOffsets[doc]
  uint32_t* pm;
  const uint64_t* pmOffsets;   // nDocs + 1, in records
};

// ------------------------------------------------------------------ annotate-adjust
// computePropertyValue for one adjust change (segmentPropertiesManager.ts:54-78): the current value's
// number (typeof "number", else 0) + delta, then max clamps, else min, in IEEE double. A change's
// current value is always the running fold of the key's changes in seq order (every remote change
// folds into properties[key] when it applies, :199-235), so the replay state needs no per-segment
// change lists. Returns the result's value id (0: null, the key is deleted) or a kAdjFail* code.
// Compiled only into the Doc<..., Adj = true> variants (batches with adjusts): inlined into the op
// loop it costs the register allocation of every other variant (measured: ~1000 VGPR spills).
constexpr uint32_t kAdjFailData = 0xFFFFFFFFu, kAdjFailCap = 0xFFFFFFFEu;

FMT_DEV double adjNumberOf(const AdjustTables* A, uint32_t doc, uint32_t id) {  // NaN: not a number
  if (id >= FMT_MT_VALUE_COMPUTED) {
    const uint32_t k = id - FMT_MT_VALUE_COMPUTED;
    const uint32_t cnt = uni(loadCoherent(A->numCount + doc));
    return k < cnt ? uniD(loadCoherentD(A->nums + A->numOffsets[doc] + k)) : __builtin_nan("");
  }
  if (A->valueBase != nullptr) {
    const uint32_t b0 = uni(A->valueBase[doc]), cnt = uni(A->valueBase[doc + 1]) - b0;
    return id >= 1 && id <= cnt ? uniD(A->valueNum[b0 + id]) : __builtin_nan("");
  }
  return id < A->nValues ? uniD(A->valueNum[id]) : __builtin_nan("");
}

// The value id of a number: the host's id of an equal number (binary search of its sorted numbers),
// else the document table's entry (lane-parallel search), else a new entry. -0 is +0 (=== equal, and
// JSON.stringify writes both as 0).
FMT_DEV uint32_t adjNumberId(const AdjustTables* A, uint32_t doc, double x) {
  if (x == 0.0) x = 0.0;
  const int ns = static_cast<int>(A->numSortedOffs != nullptr ? uni(A->numSortedOffs[doc + 1]) : uni(A->nNumSorted));
  int lo = A->numSortedOffs != nullptr ? static_cast<int>(uni(A->numSortedOffs[doc])) : 0, hi = ns;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (uniD(A->numSorted[mid]) < x) lo = mid + 1;
    else hi = mid;
  }
  if (lo < ns && uniD(A->numSorted[lo]) == x) return uni(A->numSortedId[lo]);
  double* nums = A->nums + A->numOffsets[doc];
  const uint32_t cap = static_cast<uint32_t>(A->numOffsets[doc + 1] - A->numOffsets[doc]);
  const uint32_t cnt = uni(loadCoherent(A->numCount + doc));
  for (uint32_t base = 0; base < cnt; base += 64) {
    Lane<bool> eq;
    FOR_LANES(l) { LANE(eq) = base + l < cnt && loadCoherentD(nums + base + l) == x; }
    const uint64_t m = ballot(eq);
    if (m != 0) return FMT_MT_VALUE_COMPUTED + base + static_cast<uint32_t>(ctz64(m));
  }
  if (cnt >= cap) return kAdjFailCap;
  FOR_LANES(l) {
    if (l == 0) {
      storeGlobal(nums + cnt, x);
      storeGlobal(A->numCount + doc, cnt + 1);
    }
  }
  return FMT_MT_VALUE_COMPUTED + cnt;
}

FMT_DEV uint32_t adjustFold(const AdjustTables* A, uint32_t doc, uint32_t cur, uint32_t row) {
  if (A == nullptr || row >= A->nAdjusts) return kAdjFailData;
  const fmt_mt_adjust* R = A->adjusts + row;
  const double delta = uniD(R->delta), mn = uniD(R->min), mx = uniD(R->max);
  const uint32_t fl = uni(R->flags);
  const double c = adjNumberOf(A, doc, cur);
  const double adjusted = (c == c ? c : 0.0) + delta;
  // `adjusted > adjust.max` with a null max compares against 0 and assigns null
  if ((fl & FMT_MT_ADJ_MAX) != 0 && adjusted > ((fl & FMT_MT_ADJ_MAX_NULL) ? 0.0 : mx))
    return (fl & FMT_MT_ADJ_MAX_NULL) ? 0u : adjNumberId(A, doc, mx);
  if ((fl & FMT_MT_ADJ_MIN) != 0 && adjusted < ((fl & FMT_MT_ADJ_MIN_NULL) ? 0.0 : mn))
    return (fl & FMT_MT_ADJ_MIN_NULL) ? 0u : adjNumberId(A, doc, mn);
  return adjNumberId(A, doc, adjusted);
}

}  // namespace fmt_mt
