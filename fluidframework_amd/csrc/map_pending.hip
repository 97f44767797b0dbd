// map_pending.hip — the local-client pending state of SharedMap (fmt.h fmt_map_pending_run): per
// document, MapKernel.pendingData (mapKernel.ts:132-139) rebuilt from the document's local events
// and merged with the sequenced entries of the last sparse run into the optimistic view.
//
// One thread per document. pendingData is an ordered list of entries — a set "lifetime" (its
// pending sets, oldest first), a delete, a clear — created by submissions (set :402-447, delete
// :453-490, clear :495-538); an ack removes the oldest unacknowledged submission (the local branches
// of the handlers :706-853), a rollback the newest (:633-700). Every list lives in the per-event
// scratch records below (linked lists indexed by event number), so a document costs O(its events)
// of HBM; the walks are O(pending) per op — pending lists are short (a reconnecting client's unsent
// ops), and the work is a dependent pointer chase per document, not a bandwidth problem.
#include "kernels.h"

namespace fmt_kernels {

namespace {

constexpr uint32_t kNil = 0xFFFFFFFFu;
enum : uint32_t { kLifetime = 0, kDelete = 1, kClear = 2 };

// Scratch record of event i (only submissions use one).
struct PendRec {
  uint32_t type;            // entry type of a submission that created an entry (kLifetime/kDelete/kClear)
  uint32_t ePrev, eNext;    // pendingData order (entries: the submission that created them)
  uint32_t ksPrev, ksNext;  // a set submission: its lifetime's keySets, oldest first
  uint32_t lHead, lTail;    // a lifetime entry: first / last pending set
  uint32_t life;            // a set submission: its lifetime entry
  uint32_t uPrev, uNext;    // unacknowledged submissions, oldest first
};

__device__ inline uint32_t kindOf(uint32_t kv) { return kv >> FMT_MAP_KIND_SHIFT; }

__global__ void __launch_bounds__(256) mapPendingKernel(const fmt_map_local_op* __restrict__ ev, const uint64_t* __restrict__ evOffs,
                                                        const fmt_map_entry* __restrict__ seqEnt, const uint64_t* __restrict__ seqOffs,
                                                        const uint32_t* __restrict__ seqCounts, uint32_t nDocs, PendRec* rec,
                                                        const uint64_t* __restrict__ outBase, fmt_map_entry* out, uint32_t* outCounts,
                                                        int32_t* outStatus) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= nDocs) return;
  const uint64_t e0 = evOffs[d], e1 = evOffs[d + 1];
  if (e1 - e0 > FMT_MAP_PENDING_MAX_EVENTS) {  // one lane's dependent list walks: bounded per document
    outCounts[d] = 0;
    outStatus[d] = FMT_E_CAPACITY;
    return;
  }
  uint32_t eHead = kNil, eTail = kNil, uHead = kNil, uTail = kNil;
  bool bad = false;
  auto keyOf = [&](uint32_t i) { return ev[i].key; };
  auto appendEntry = [&](uint32_t i, uint32_t type) {
    rec[i].type = type;
    rec[i].ePrev = eTail;
    rec[i].eNext = kNil;
    if (eTail != kNil) rec[eTail].eNext = i;
    else eHead = i;
    eTail = i;
  };
  auto unlinkEntry = [&](uint32_t i) {
    const uint32_t p = rec[i].ePrev, n = rec[i].eNext;
    if (p != kNil) rec[p].eNext = n;
    else eHead = n;
    if (n != kNil) rec[n].ePrev = p;
    else eTail = p;
  };
  for (uint64_t j = e0; j < e1 && !bad; j++) {
    const uint32_t i = static_cast<uint32_t>(j);
    const fmt_map_local_op o = ev[i];
    const uint32_t kind = kindOf(o.kind_value);
    if (o.event == FMT_MAP_EV_SUBMIT) {
      rec[i].uPrev = uTail;
      rec[i].uNext = kNil;
      if (uTail != kNil) rec[uTail].uNext = i;
      else uHead = i;
      uTail = i;
      if (kind == FMT_MAP_SET) {
        // findLast(entry => clear || entry.key === key) (:427-430); a new lifetime unless it is one
        uint32_t e = eTail;
        while (e != kNil && rec[e].type != kClear && keyOf(e) != o.key) e = rec[e].ePrev;
        if (e == kNil || rec[e].type != kLifetime) {
          e = i;
          appendEntry(i, kLifetime);
          rec[i].lHead = rec[i].lTail = kNil;
        }
        rec[i].life = e;
        rec[i].ksPrev = rec[e].lTail;
        rec[i].ksNext = kNil;
        if (rec[e].lTail != kNil) rec[rec[e].lTail].ksNext = i;
        else rec[e].lHead = i;
        rec[e].lTail = i;
      } else {
        appendEntry(i, kind == FMT_MAP_DELETE ? kDelete : kClear);
      }
      continue;
    }
    // ACK: the oldest unacknowledged submission; ROLLBACK: the newest
    const bool ack = o.event == FMT_MAP_EV_ACK;
    const uint32_t s = ack ? uHead : uTail;
    if (o.event > FMT_MAP_EV_ROLLBACK || s == kNil || ev[s].kind_value != o.kind_value ||
        (kind != FMT_MAP_CLEAR && ev[s].key != o.key)) {
      bad = true;
      break;
    }
    const uint32_t up = rec[s].uPrev, un = rec[s].uNext;
    if (up != kNil) rec[up].uNext = un;
    else uHead = un;
    if (un != kNil) rec[un].uPrev = up;
    else uTail = up;
    if (kind == FMT_MAP_SET) {  // keySets.shift() (ack, :829-833) / keySets.pop() (rollback, :680)
      const uint32_t e = rec[s].life;
      if ((ack ? rec[e].lHead : rec[e].lTail) != s) {
        bad = true;
        break;
      }
      const uint32_t p = rec[s].ksPrev, n = rec[s].ksNext;
      if (p != kNil) rec[p].ksNext = n;
      else rec[e].lHead = n;
      if (n != kNil) rec[n].ksPrev = p;
      else rec[e].lTail = p;
      if (rec[e].lHead == kNil) unlinkEntry(e);  // an emptied lifetime leaves pendingData
    } else {
      unlinkEntry(s);
    }
  }
  uint32_t n = 0;
  if (!bad) {
    fmt_map_entry* o = out + outBase[d];
    const fmt_map_entry* se = seqEnt + seqOffs[d];
    const uint32_t ns = seqCounts[d];
    bool anyClear = false;
    for (uint32_t e = eHead; e != kNil; e = rec[e].eNext) anyClear = anyClear || rec[e].type == kClear;
    // 1. sequenced keys not optimistically deleted or cleared, with their optimistic value (:184-202)
    for (uint32_t q = 0; q < ns && !anyClear; q++) {
      const fmt_map_entry x = se[q];
      bool deleted = false;
      uint32_t latest = kNil;
      for (uint32_t e = eHead; e != kNil; e = rec[e].eNext) {
        if (keyOf(e) != x.key) continue;
        deleted = deleted || rec[e].type == kDelete;
        latest = e;
      }
      if (deleted) continue;
      const uint32_t v = latest == kNil ? x.value : (ev[rec[latest].lTail].kind_value & FMT_MAP_VALUE_MASK);
      o[n++] = {x.key, v, x.birth_seq};
    }
    // 2. pending lifetimes not deleted or cleared after they began (:204-235)
    for (uint32_t e = eHead; e != kNil; e = rec[e].eNext) {
      if (rec[e].type != kLifetime) continue;
      const uint32_t key = keyOf(e);
      bool later = false, earlier = false;
      for (uint32_t f = rec[e].eNext; f != kNil && !later; f = rec[f].eNext)
        later = rec[f].type == kClear || (rec[f].type == kDelete && keyOf(f) == key);
      if (later) continue;
      for (uint32_t f = rec[e].ePrev; f != kNil && !earlier; f = rec[f].ePrev)
        earlier = rec[f].type == kClear || (rec[f].type == kDelete && keyOf(f) == key);
      bool inSeq = false;
      for (uint32_t q = 0; q < ns && !inSeq; q++) inSeq = se[q].key == key;
      if (inSeq && !earlier) continue;  // (iterated with the sequenced keys)
      o[n++] = {key, ev[rec[e].lTail].kind_value & FMT_MAP_VALUE_MASK,
                FMT_MAP_PENDING_BIRTH | static_cast<uint32_t>(e - e0)};
    }
  }
  outCounts[d] = n;
  outStatus[d] = bad ? FMT_E_DATA : FMT_OK;
}

}  // namespace

size_t mapPendingScratchBytes(uint64_t nEvents) { return static_cast<size_t>(nEvents) * sizeof(PendRec); }

hipError_t launchMapPending(const fmt_map_local_op* events, const uint64_t* evOffs, const fmt_map_entry* seqEntries,
                            const uint64_t* seqOffs, const uint32_t* seqCounts, uint32_t nDocs, void* scratch,
                            const uint64_t* outBase, fmt_map_entry* out, uint32_t* outCounts, int32_t* outStatus,
                            hipStream_t stream) {
  if (nDocs == 0) return hipSuccess;
  hipLaunchKernelGGL(mapPendingKernel, dim3((nDocs + 255) / 256), dim3(256), 0, stream, events, evOffs, seqEntries,
                     seqOffs, seqCounts, nDocs, static_cast<PendRec*>(scratch), outBase, out, outCounts, outStatus);
  return hipGetLastError();
}

}  // namespace fmt_kernels
