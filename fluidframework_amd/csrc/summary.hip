// summary.hip — bulk legacy SharedString summaries: SnapshotLegacy.extractSync's segment merge
// (merge-tree/src/snapshotlegacy.ts:195-262) for every document of a replay, on the device.
//
// One wave per document (4 per workgroup, grid-stride). The document's leaves are read 64 at a time:
// a leaf is in the summary iff it is present at PriorPerspective(minSeq, NonCollabClient) (inserted
// at/below minSeq, not removed at/below it). Present leaves are appended onto the previous run while
// prev.canAppend(seg) && matchProperties: both TextSegments, the run not ending in '\n', the run or
// the leaf at most TextSegmentGranularity long (textSegment.ts:76-83), and props equal as maps
// (undefined ≡ {}: match classes computed per prop set first). The decisions are a serial scan over
// the present leaves (wave-uniform); the text of the present leaves is copied lane-parallel into one
// compact run text. Output per document: runs {len, head's prop set, marker flag} and the text, in
// spans reserved with one atomic per document; the host formats the JSON (snapshotChunks.ts:85-204).
#include <hip/hip_runtime.h>

#include "../../include/fmt.h"
#include "kernels.h"
#include "adjust.h"

namespace fmt_kernels {

constexpr int kSumWaves = 4;
constexpr int kSumMaxProps = 4096;  // prop sets per document (the huge tier's table)

__device__ __forceinline__ void sumSync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t sumUni(uint32_t x) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(x))); }

__device__ __forceinline__ uint32_t sumLane(uint32_t v, int lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), lane));
}

// Entry k of the prop set whose first record is p (fmt.h: wide sets take consecutive records).
__device__ __forceinline__ uint32_t sumKv(const fmt_mt_propset* T, uint32_t p, uint32_t k) {
  return T[p + k / FMT_MT_PROPS_MAX].kv[k % FMT_MT_PROPS_MAX];
}

// Sets p and q (first records, np records in all) hold the same (key, value) pairs, any order.
__device__ __forceinline__ bool sumSameSet(const fmt_mt_propset* T, uint32_t p, uint32_t q, uint32_t np) {
  const uint32_t n = T[p].n;
  if (n != T[q].n || n == FMT_MT_PROPS_CONT || n > FMT_MT_PROPS_KEYS_MAX) return false;
  if (p + (n ? (n - 1) / FMT_MT_PROPS_MAX : 0) >= np || q + (n ? (n - 1) / FMT_MT_PROPS_MAX : 0) >= np) return false;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t x = sumKv(T, p, i);
    bool found = false;
    for (uint32_t j = 0; j < n; j++) found = found || sumKv(T, q, j) == x;
    if (!found) return false;
  }
  return true;
}

__global__ __launch_bounds__(64 * kSumWaves) void summaryRunsKernel(const fmt_mt_doc_result* __restrict__ hdrs,
                                                              const SumView* __restrict__ views, uint32_t nDocs,
                                                              SumRun* __restrict__ runs, uint16_t* __restrict__ text,
                                                              unsigned long long* __restrict__ cursors,
                                                              SumDocOut* __restrict__ docOut) {
  __shared__ uint16_t clsAll[kSumWaves][kSumMaxProps];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  uint16_t* cls = clsAll[wave];
  for (uint32_t d = blockIdx.x * kSumWaves + wave; d < nDocs; d += gridDim.x * kSumWaves) {
    const fmt_mt_doc_result h = hdrs[d];
    SumDocOut od{};
    od.status = static_cast<uint32_t>(h.status);
    const SumView V = views[d];
    if (h.status != FMT_OK || (V.cls == nullptr && h.n_props > static_cast<uint32_t>(kSumMaxProps))) {
      if (h.status == FMT_OK) od.status = static_cast<uint32_t>(FMT_E_CAPACITY);
      if (lane == 0) docOut[d] = od;
      continue;
    }
    const uint32_t n = h.n_leaves, np = h.n_props;
    const int32_t minSeq = h.min_seq;
    // match classes: the first prop set with the same content (empty sets: undefined's class)
    for (uint32_t p = lane; p < np && V.cls == nullptr; p += 64) {  // (huge documents: the engine's classes)
      const uint32_t an = V.props[p].n;
      uint16_t c = an == 0 ? 0xFFFFu : static_cast<uint16_t>(p);
      if (an != 0 && an != FMT_MT_PROPS_CONT)  // (continuation records: no leaf names them)
        for (uint32_t q = 0; q < p; q++)
          if (sumSameSet(V.props, q, p, np)) {
            c = static_cast<uint16_t>(q);
            break;
          }
      cls[p] = c;
    }
    // present leaves and their units: the spans reserved for this document
    uint32_t nPresent = 0, nUnits = 0;
    bool unavailable = false;  // the engine could not intern this document's getAtSeq view
    for (uint32_t b = 0; b < n; b += 64) {
      const uint32_t i = b + lane;
      bool pres = false;
      uint32_t len = 0;
      if (i < n) {
        const fmt_mt_leaf L = V.leaves[i];
        pres = L.ins_seq <= minSeq && !(L.rm_seq <= minSeq);
        len = pres ? L.len : 0u;
        if (V.legacyProps != nullptr && V.legacyProps[i] == fmt_mt::kLegacyUnavailable) unavailable = true;
      }
      nPresent += static_cast<uint32_t>(__popcll(__ballot(pres)));
      for (int off = 32; off > 0; off >>= 1) len += static_cast<uint32_t>(__shfl_xor(static_cast<int>(len), off));
      nUnits += len;
    }
    if (__ballot(unavailable) != 0) {
      od.status = static_cast<uint32_t>(FMT_E_CAPACITY);
      if (lane == 0) docOut[d] = od;
      continue;
    }
    unsigned long long runBase = 0, textBase = 0;
    if (lane == 0) {
      runBase = atomicAdd(&cursors[0], static_cast<unsigned long long>(nPresent));
      textBase = atomicAdd(&cursors[1], static_cast<unsigned long long>(nUnits));
    }
    runBase = __shfl(runBase, 0);
    textBase = __shfl(textBase, 0);
    sumSync();
    // serial merge decisions over the present leaves, text copied chunk by chunk
    uint32_t nRuns = 0, runLen = 0, runProps = 0xFFFFu, runFlags = 0, runCls = 0xFFFFu, runLast = 0;
    bool have = false, runMarker = false;
    uint64_t tpos = 0;
    for (uint32_t b = 0; b < n; b += 64) {
      const uint32_t i = b + lane;
      bool pres = false;
      uint32_t len = 0, props = 0xFFFFu, last = 0, off = 0, marker = 0;
      if (i < n) {
        const fmt_mt_leaf L = V.leaves[i];
        pres = L.ins_seq <= minSeq && !(L.rm_seq <= minSeq);
        if (pres) {
          len = L.len;
          props = V.legacyProps != nullptr ? V.legacyProps[i] : L.props;  // getAtSeq(minSeq) (adjust batches)
          off = L.char_off;
          marker = (L.pad & FMT_MT_LEAF_MARKER) != 0 ? 1u : 0u;
          last = len > 0 ? V.chars[off + len - 1] : 0u;
        }
      }
      // text: present leaves' units to text[textBase + tpos + prefix]
      uint32_t ex = len;  // exclusive prefix of len over lanes
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = static_cast<uint32_t>(__shfl_up(static_cast<int>(ex), o));
        if (lane >= o) ex += t;
      }
      const uint32_t chunkUnits = sumUni(static_cast<uint32_t>(__shfl(static_cast<int>(ex), 63)));
      ex -= len;
      for (uint32_t u0 = 0; u0 < chunkUnits; u0 += 64) {
        const uint32_t t = u0 + lane;
        // source leaf of unit t: the last lane whose start <= t (binary search by shuffles)
        int pos = 0;
        for (int step = 32; step >= 1; step >>= 1) {
          const uint32_t s = static_cast<uint32_t>(__shfl(static_cast<int>(ex), pos + step));
          if (s <= t) pos += step;
        }
        const uint32_t st = static_cast<uint32_t>(__shfl(static_cast<int>(ex), pos));
        const uint32_t so = static_cast<uint32_t>(__shfl(static_cast<int>(off), pos));
        if (t < chunkUnits) text[textBase + tpos + t] = V.chars[so + (t - st)];
      }
      tpos += chunkUnits;
      uint64_t m = __ballot(pres);
      while (m) {
        const int k = __ffsll(static_cast<long long>(m)) - 1;
        m &= m - 1;
        const uint32_t l = sumLane(len, k), p = sumLane(props, k), lc = sumLane(last, k);
        const bool mk = sumLane(marker, k) != 0;
        const uint32_t c = p == 0xFFFFu ? 0xFFFFu : V.cls != nullptr ? (V.cls[p] & 0xFFFFu) : static_cast<uint32_t>(cls[p]);
        const bool append = have && !runMarker && !mk && runLast != 10u &&
                            (runLen <= 256u || l <= 256u) && runCls == c;
        if (append) {
          runLen += l;
          runLast = lc;
        } else {
          if (have && lane == 0) runs[runBase + nRuns] = SumRun{runLen, static_cast<uint16_t>(runProps), static_cast<uint16_t>(runFlags)};
          nRuns += have ? 1u : 0u;
          have = true;
          runLen = l;
          runProps = p;
          runCls = c;
          runLast = lc;
          runMarker = mk;
          runFlags = mk ? 1u : 0u;
        }
      }
    }
    if (have) {
      if (lane == 0) runs[runBase + nRuns] = SumRun{runLen, static_cast<uint16_t>(runProps), static_cast<uint16_t>(runFlags)};
      nRuns++;
    }
    od.run_off = runBase;
    od.text_off = textBase;
    od.n_runs = nRuns;
    od.n_units = nUnits;
    if (lane == 0) docOut[d] = od;
    sumSync();
  }
}

hipError_t launchSummaryRuns(const fmt_mt_doc_result* hdrs, const SumView* views, uint32_t nDocs, SumRun* runs,
                             uint16_t* text, unsigned long long* cursors, SumDocOut* docOut, int numCUs,
                             hipStream_t stream) {
  const uint32_t wanted = (nDocs + kSumWaves - 1) / kSumWaves;
  const uint32_t cap = static_cast<uint32_t>(numCUs) * 4u;
  const uint32_t grid = wanted < cap ? (wanted > 0 ? wanted : 1) : cap;
  hipLaunchKernelGGL(summaryRunsKernel, dim3(grid), dim3(64 * kSumWaves), 0, stream, hdrs, views, nDocs, runs, text,
                     cursors, docOut);
  return hipGetLastError();
}

}  // namespace fmt_kernels
