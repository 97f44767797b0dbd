// runtime.cpp — the C ABI of include/fmt.h over HIP (host side of libfmt.so).
//
// Owns the device, the stream, device buffers and HIP events. Inputs cross host→HBM once per batch
// in fmt_*_load (the only PCIe traffic); fmt_*_run only launches kernels on resident data, so a
// caller can time run() alone ("inputs already resident in HBM"). No exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "../../include/fmt.h"
#include "huge_engine.h"
#include "jsnum.h"
#include "mt_engine.h"  // fmt_mt::AdjustTables
#include "kernels.h"

namespace {

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  hipError_t reserve(size_t n) {
    if (n <= cap && p != nullptr) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t bytes = (n > 0 ? n : 1) * sizeof(T);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), bytes);
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Large host <-> device copies through pinned staging. The caller's arrays are pageable (numpy, JS
// ArrayBuffers), which the DMA engines reach only through the runtime's own small bounce buffer
// (measured: 4.3 GB/s H2D for T1's 7.3 GB, 0.18 GB/s for the catch-up fetch). Here kStageWorkers
// host threads each own two pinned chunks and a stream, and move every kStageWorkers-th chunk of
// the copy: one chunk's host memcpy overlaps the DMA of the chunk before it.
constexpr size_t kStageChunk = 8u << 20;
constexpr int kStageWorkers = 8;
constexpr size_t kStageMin = 16u << 20;  // smaller copies go straight through hipMemcpy

// Pinned host memory the ctx keeps across calls (hipHostMalloc'd, grown on demand): DMA lands in it
// directly, no staging copy.
template <class T>
struct PinnedBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    void* q = nullptr;
    const hipError_t e = hipHostMalloc(&q, (n ? n : 1) * sizeof(T), hipHostMallocDefault);
    if (e != hipSuccess) return e;
    p = static_cast<T*>(q);
    cap = n;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  ~PinnedBuf() { release(); }
};

struct Stager {
  bool ready = false;
  void* buf[kStageWorkers][2] = {};
  hipStream_t st[kStageWorkers] = {};
  hipEvent_t ev[kStageWorkers][2] = {};
  void release() {
    for (int w = 0; w < kStageWorkers; w++) {
      for (int k = 0; k < 2; k++) {
        if (buf[w][k]) (void)hipHostFree(buf[w][k]);
        if (ev[w][k]) (void)hipEventDestroy(ev[w][k]);
        buf[w][k] = nullptr;
        ev[w][k] = nullptr;
      }
      if (st[w]) (void)hipStreamDestroy(st[w]);
      st[w] = nullptr;
    }
    ready = false;
  }
};

}  // namespace

struct fmt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool ownStream = false;
  int numCUs = 256;
  std::string arch;
  std::string err;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the run's (first) launch
  hipEvent_t ev2 = nullptr, ev3 = nullptr;  // around a second launch (large-tier replay), if any
  hipEvent_t evS0 = nullptr, evS1 = nullptr;  // around the bulk summary kernel (fmt_mt_summarize_legacy)
  bool timed = false, timed2 = false;
  fmt_stats stats{};

  // SharedMap
  DevBuf<fmt_map_op> mapOps;
  DevBuf<uint64_t> mapOffs;
  DevBuf<fmt_map_slot> mapOut;
  DevBuf<uint32_t> mapScratch;  // kill / first tables of the HBM-table path (large key pools)
  DevBuf<int> errWord;
  uint64_t mapNOps = 0;
  uint32_t mapDocs = 0, mapKeyBound = 0;
  bool mapLoaded = false;
  // SharedMap, sparse path: entries at each document's op offset, live counts, packed copy
  DevBuf<fmt_map_entry> mapEntries, mapPacked;
  DevBuf<uint32_t> mapCounts;
  DevBuf<uint64_t> mapPackedOff;
  bool mapSparse = false;
  bool mapSparseRan = false;
  std::vector<uint64_t> mapOffsHost;  // the staged batch's doc_op_offsets
  // SharedMap local-client pending state (fmt_map_pending_run): events, per-event scratch, the
  // optimistic entries at mapPendBase[d] = op offset + event offset of the document
  DevBuf<fmt_map_local_op> mapEv;
  DevBuf<uint64_t> mapEvOffs, mapPendBase;
  DevBuf<uint8_t> mapPendScratch;
  DevBuf<fmt_map_entry> mapPendOut;
  DevBuf<uint32_t> mapPendCounts;
  DevBuf<int32_t> mapPendStatus;
  bool mapPendRan = false;

  // merge-tree
  DevBuf<fmt_mt_op> mtOps;
  DevBuf<uint64_t> mtOffs;
  DevBuf<uint16_t> mtText;
  DevBuf<uint32_t> mtInit, mtPropsOff, mtPropsKv;
  DevBuf<fmt_mt_doc_result> mtHdr;
  DevBuf<fmt_mt_leaf> mtLeaves;
  DevBuf<uint16_t> mtChars;
  DevBuf<fmt_mt_propset> mtProps;
  DevBuf<uint32_t> mtEsc;                    // small-tier overflow list: [0] = count, then doc ids
  DevBuf<uint32_t> mtEsc2;                   // compact-tier overflow list (no remove order), same layout
  DevBuf<uint32_t> mtEsc3;                   // the same list, longest remaining streams first
  DevBuf<uint32_t> mtCkpt;                   // per-document compact → small tier checkpoints
  DevBuf<uint32_t> mtHugeCk;                 // per large-tier slot: its large → huge checkpoint record (huge_ckpt.h)
  bool mtCkptOk = false;                     // allocated for this batch (else tiers replay overflow from op 0)
  DevBuf<uint32_t> mtSched;                  // per-tier document counters (dynamic dealing to waves)
  DevBuf<fmt_mt_leaf> mtBigLeaves;           // large-tier result slabs, one per escalated doc
  DevBuf<uint16_t> mtBigChars;
  DevBuf<fmt_mt_propset> mtBigProps;
  std::vector<int32_t> mtBigSlot;            // doc -> large-tier slab, or -1
  DevBuf<fmt_mt_snapshot_doc> mtSnap;       // per-doc summary loads (f3)
  DevBuf<fmt_mt_snapshot_seg> mtSnapSegs;
  DevBuf<fmt_mt_relpos> mtRelpos;            // relative positions (FMT_MT_F_REL1/REL2 ops)
  DevBuf<fmt_mt_snapshot_info> mtSnapInfo;   // SnapshotV1 merge info of loaded segments
  DevBuf<fmt_mt_stamp> mtSnapStamps;
  bool mtHasSnapInfo = false;
  uint64_t mtNSnapSegs = 0;
  uint32_t mtNRelpos = 0, mtMarkerKey = FMT_MT_NO_MARKER;
  bool mtHasSnap = false;
  bool mtObliterate = false;                 // batch holds obliterates: launch the Doc<true> kernel
  DevBuf<uint64_t> mtCuOffs;                 // per-doc catch-up slab offsets (n_docs + 1)
  DevBuf<fmt_mt_catchup_range> mtCatchup;    // catch-up range slabs
  std::vector<uint64_t> mtCuOffsHost;
  bool mtHasCatchup = false;
  DevBuf<uint64_t> mtRmOffs;                 // per-doc remove-order slab offsets (n_docs + 1)
  DevBuf<fmt_mt_remove_order> mtRmOrder;     // remove-order slabs (FMT_MT_F_RMORDER ops)
  std::vector<uint64_t> mtRmOffsHost;
  bool mtHasRmOrder = false;
  // huge documents (T3, huge_engine.h): one wave each, state in per-document HBM buffers
  struct HugeDocBufs {
    std::vector<void*> allocs;
    fmt_huge::HugeState state{};
    fmt_huge::HugeInputs in{};
    fmt_kernels::HugeOut out{};
    std::vector<uint32_t> shape;             // host copy of in.shape (kept until the load completes)
  };
  std::vector<HugeDocBufs> huge;             // per huge document
  std::vector<int32_t> mtHugeSlot;           // doc -> index in huge, or -1
  // documents that outgrow the large tier replay again, from their start, in the huge tier when
  // they hold nothing it does not (mtHugeOk: no SnapshotV1 body segments with merge info,
  // FMT_MT_F_LOADSEG); their starts
  std::vector<uint8_t> mtHugeOk;
  std::vector<uint32_t> mtLoadSegs;          // per document: its FMT_MT_F_LOADSEG ops (V1 body segments)
  std::vector<uint8_t> mtSegProps;           // per document: a loaded segment has properties
  std::vector<uint64_t> mtDocChars;          // per document: start units + inserted units (its most text)
  std::vector<fmt_mt_snapshot_seg> mtStartSeg;  // per document: its initial text as one segment (len 0: none)
  uint32_t mtHugeLoaded = 0;                 // huge documents routed at load (the rest were escalated)
  // documents refused at load (a feature the huge tier lacks, or no device memory for its state):
  // their headers are written at load and no tier runs them; the rest of the batch is unaffected
  std::vector<uint32_t> mtRefused;
  bool mtUseList = false;                    // the small tiers run mtSmallList (huge or refused docs)
  uint32_t mtGrown = 0;                      // documents the last run escalated into the huge tier
  uint32_t mtNPropsOps = 0;
  std::vector<uint64_t> mtOffsHost;          // host copies of doc_op_offsets and the snapshot docs
  std::vector<fmt_mt_snapshot_doc> mtSnapHost;
  DevBuf<fmt_mt_snapshot_seg> mtStartSegDev;
  DevBuf<fmt_huge::HugeState> hugeStates2;
  DevBuf<fmt_huge::HugeInputs> hugeInputs2;
  DevBuf<fmt_kernels::HugeOut> hugeOuts2;
  // bulk legacy summaries (fmt_mt_summarize_legacy): device runs / text, host blobs
  DevBuf<fmt_kernels::SumView> sumViews;
  DevBuf<fmt_kernels::SumRun> sumRuns;
  DevBuf<uint16_t> sumText;
  DevBuf<unsigned long long> sumCursors;
  DevBuf<fmt_kernels::SumDocOut> sumDocs;
  DevBuf<uint64_t> digests;                   // fmt_mt_state_digest output
  Stager stage;                               // pinned staging of large host <-> device copies
  DevBuf<fmt_kernels::GatherSpan> spans;      // packing before a D2H copy
  DevBuf<uint32_t> packed;
  std::vector<std::string> sumBlobs;          // per document: header, then body
  std::vector<uint32_t> sumSplit;             // per document: header length in sumBlobs[d]
  std::vector<int32_t> sumStatus;
  PinnedBuf<fmt_kernels::SumDocOut> sumHostDocs;  // host copies of the device runs / text / prop sets
  PinnedBuf<fmt_kernels::SumRun> sumHostRuns;
  PinnedBuf<uint16_t> sumHostText;
  PinnedBuf<fmt_mt_propset> sumHostProps;
  // annotate-adjust: rows, numbers of host value ids, host numbers sorted for number → id lookups,
  // per-document computed-number slabs and their counts
  DevBuf<fmt_mt_adjust> mtAdjusts;
  DevBuf<double> mtValueNum, mtNumSorted, mtNums;
  DevBuf<uint32_t> mtNumSortedId, mtNumCount;
  DevBuf<uint32_t> mtValueBase, mtNumSortedOffs;  // document-local value ids (doc_value_base)
  std::vector<uint32_t> mtValueBaseHost;         // empty: batch-global value ids
  DevBuf<uint64_t> mtNumOffs;
  DevBuf<fmt_mt::AdjustTables> mtAdjTab;      // the pointers above, for the kernels
  std::vector<uint64_t> mtNumOffsHost;
  DevBuf<uint32_t> mtPm;                      // PropertiesManager records (4 words each) per document
  DevBuf<uint64_t> mtPmOffs;
  std::vector<uint64_t> mtPmOffsHost;
  DevBuf<uint16_t> mtLegacy, mtBigLegacy;     // per leaf: the getAtSeq(minSeq) prop set (small / large slabs)
  bool mtHasAdjust = false;
  uint32_t mtNAdjusts = 0, mtNValues = 0, mtNNumSorted = 0;
  DevBuf<uint32_t> mtSmallList;              // the other documents (small tier), when huge ones exist
  // f4 (local-client records): every document replays in the compact tier's Loc variant first, the ones
  // it cannot hold in the small tier's, then the large tier's (round 6; mergetree_local.hip); its pending
  // groups, group records, PropertiesManager records, regenerated ops / text and normalization
  // scratch live in per-document slabs (mt_engine.h LocalTables)
  bool mtLocal = false;
  bool mtHiClients = false;  // some op or merge-info stamp names a short client id 64..253 (huge tier only)
  DevBuf<uint32_t> mtLocGroups, mtLocRecs, mtLocPm, mtLocScratch, mtLocRegenCount;
  DevBuf<uint64_t> mtLocOffs;                // 6 offset arrays of n + 1: groups, recs, pm, regen, text, scratch
  DevBuf<fmt_mt_op> mtLocRegen;
  DevBuf<uint16_t> mtLocRegenText;
  DevBuf<fmt_mt::LocalTables> mtLocTab;
  std::vector<uint64_t> mtLocRegenOffsHost, mtLocRegenTextOffsHost;
  uint32_t mtNSmall = 0;
  DevBuf<fmt_huge::HugeState> hugeStates;
  DevBuf<fmt_huge::HugeInputs> hugeInputs;
  DevBuf<fmt_kernels::HugeOut> hugeOuts;
  uint64_t mtNOps = 0, mtTextLen = 0, mtInsertChars = 0, mtInitChars = 0;
  uint32_t mtDocs = 0, mtNProps = 0;
  bool mtHasInit = false, mtLoaded = false;
};

namespace {

int setErr(fmt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hipErr(fmt_ctx* c, hipError_t e, const char* what) {
  return setErr(c, FMT_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define FMT_HIP(ctx, expr)                                 \
  do {                                                     \
    hipError_t e_ = (expr);                                \
    if (e_ != hipSuccess) return hipErr((ctx), e_, #expr); \
  } while (0)

// Host threads for the runtime's own passes over a batch (validation, per-document sizing).
unsigned hostWorkers() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

// fn(begin, end, worker) over hostWorkers() contiguous shares of [0, n) (one share below 2^16 items).
template <class F>
void parallelChunks(uint64_t n, F&& fn) {
  const unsigned T = n < (1u << 16) ? 1u : hostWorkers();
  if (T == 1) {
    fn(0, n, 0u);
    return;
  }
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < T; t++) pool.emplace_back([&, t] { fn(n * t / T, n * (t + 1) / T, t); });
  for (auto& th : pool) th.join();
}

hipError_t stageInit(fmt_ctx* c) {
  Stager& S = c->stage;
  if (S.ready) return hipSuccess;
  for (int w = 0; w < kStageWorkers; w++) {
    for (int k = 0; k < 2; k++) {
      hipError_t e = hipHostMalloc(&S.buf[w][k], kStageChunk, hipHostMallocDefault);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&S.ev[w][k], hipEventDisableTiming);
      if (e != hipSuccess) {
        S.release();
        return e;
      }
    }
    const hipError_t e = hipStreamCreateWithFlags(&S.st[w], hipStreamNonBlocking);
    if (e != hipSuccess) {
      S.release();
      return e;
    }
  }
  S.ready = true;
  return hipSuccess;
}

// Copies `bytes` between pageable host memory and the device, synchronously with respect to the
// ctx stream (it waits for the work already queued there first). toDevice: dst is device memory.
hipError_t stagedCopy(fmt_ctx* c, void* dst, const void* src, size_t bytes, bool toDevice) {
  if (bytes == 0) return hipSuccess;
  hipError_t e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return e;
  if (bytes < kStageMin || stageInit(c) != hipSuccess)  // (no pinned memory: the runtime's own path)
    return hipMemcpy(dst, src, bytes, toDevice ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost);
  const size_t nChunks = (bytes + kStageChunk - 1) / kStageChunk;
  const int workers = static_cast<int>(std::min<size_t>(kStageWorkers, nChunks));
  std::vector<hipError_t> errs(workers, hipSuccess);
  std::vector<std::thread> pool;
  for (int w = 0; w < workers; w++)
    pool.emplace_back([&, w] {
      Stager& S = c->stage;
      hipError_t err = hipSetDevice(c->device);
      auto span = [&](size_t k) { return std::min(kStageChunk, bytes - k * kStageChunk); };
      if (toDevice) {
        int slot = 0;
        for (size_t k = w; k < nChunks && err == hipSuccess; k += workers, slot ^= 1) {
          err = hipEventSynchronize(S.ev[w][slot]);  // the DMA that last read this chunk is done
          if (err != hipSuccess) break;
          std::memcpy(S.buf[w][slot], static_cast<const char*>(src) + k * kStageChunk, span(k));
          err = hipMemcpyAsync(static_cast<char*>(dst) + k * kStageChunk, S.buf[w][slot], span(k), hipMemcpyHostToDevice,
                               S.st[w]);
          if (err == hipSuccess) err = hipEventRecord(S.ev[w][slot], S.st[w]);
        }
      } else {
        // two chunks in flight: issue both, then drain one and refill it while the other lands
        auto issue = [&](size_t k, int slot) {
          hipError_t r = hipMemcpyAsync(S.buf[w][slot], static_cast<const char*>(src) + k * kStageChunk, span(k),
                                        hipMemcpyDeviceToHost, S.st[w]);
          return r == hipSuccess ? hipEventRecord(S.ev[w][slot], S.st[w]) : r;
        };
        size_t k0 = w, k1 = w + workers;
        if (k0 < nChunks) err = issue(k0, 0);
        if (err == hipSuccess && k1 < nChunks) err = issue(k1, 1);
        int slot = 0;
        for (size_t k = k0; k < nChunks && err == hipSuccess; k += workers, slot ^= 1) {
          err = hipEventSynchronize(S.ev[w][slot]);
          if (err != hipSuccess) break;
          std::memcpy(static_cast<char*>(dst) + k * kStageChunk, S.buf[w][slot], span(k));
          if (k + 2 * workers < nChunks) err = issue(k + 2 * workers, slot);
        }
      }
      const hipError_t e2 = hipStreamSynchronize(S.st[w]);
      errs[w] = err != hipSuccess ? err : e2;
    });
  for (auto& t : pool) t.join();
  for (hipError_t x : errs)
    if (x != hipSuccess) return x;
  return hipSuccess;
}

}  // namespace

extern "C" {

int fmt_open(const fmt_config* cfg, fmt_ctx** out) {
  if (out == nullptr) return FMT_E_USAGE;
  *out = nullptr;
  auto* c = new (std::nothrow) fmt_ctx();
  if (c == nullptr) return FMT_E_DEVICE;
  *out = c;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return setErr(c, FMT_E_DEVICE, "no HIP device visible");
  c->device = cfg ? cfg->device : 0;
  if (c->device < 0 || c->device >= n) return setErr(c, FMT_E_USAGE, "device ordinal out of range");
  FMT_HIP(c, hipSetDevice(c->device));
  hipDeviceProp_t prop;
  FMT_HIP(c, hipGetDeviceProperties(&prop, c->device));
  c->arch = prop.gcnArchName;
  c->numCUs = prop.multiProcessorCount;
  if (c->arch.rfind("gfx950", 0) != 0)
    return setErr(c, FMT_E_DEVICE, "libfmt is built for gfx950 only; device is " + c->arch);
  if (cfg && cfg->stream) {
    c->stream = static_cast<hipStream_t>(cfg->stream);
  } else {
    FMT_HIP(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->ownStream = true;
  }
  FMT_HIP(c, hipEventCreate(&c->ev0));
  FMT_HIP(c, hipEventCreate(&c->ev1));
  FMT_HIP(c, hipEventCreate(&c->ev2));
  FMT_HIP(c, hipEventCreate(&c->ev3));
  FMT_HIP(c, hipEventCreate(&c->evS0));
  FMT_HIP(c, hipEventCreate(&c->evS1));
  FMT_HIP(c, c->errWord.reserve(1));
  return FMT_OK;
}

void fmt_close(fmt_ctx* c) {
  if (c == nullptr) return;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  c->mapOps.release();
  c->mapOffs.release();
  c->mapOut.release();
  c->mapScratch.release();
  c->mapEntries.release();
  c->mapPacked.release();
  c->mapEv.release();
  c->mapEvOffs.release();
  c->mapPendBase.release();
  c->mapPendScratch.release();
  c->mapPendOut.release();
  c->mapPendCounts.release();
  c->mapPendStatus.release();
  c->mapCounts.release();
  c->mapPackedOff.release();
  c->errWord.release();
  c->mtOps.release();
  c->mtOffs.release();
  c->mtText.release();
  c->mtInit.release();
  c->mtPropsOff.release();
  c->mtPropsKv.release();
  c->mtHdr.release();
  c->mtLeaves.release();
  c->mtChars.release();
  c->mtProps.release();
  c->mtEsc.release();
  c->mtEsc2.release();
  c->mtEsc3.release();
  c->mtSched.release();
  c->mtCkpt.release();
  c->mtHugeCk.release();
  c->mtBigLeaves.release();
  c->mtBigChars.release();
  c->mtBigProps.release();
  c->mtSnap.release();
  c->mtSnapSegs.release();
  c->mtRelpos.release();
  c->mtSnapInfo.release();
  c->mtSnapStamps.release();
  c->mtCuOffs.release();
  c->mtCatchup.release();
  c->mtRmOffs.release();
  c->mtRmOrder.release();
  for (auto& h : c->huge)
    for (void* p : h.allocs) (void)hipFree(p);
  c->huge.clear();
  c->mtSmallList.release();
  c->hugeStates.release();
  c->hugeInputs.release();
  c->hugeOuts.release();
  c->stage.release();
  c->mtPm.release();
  c->mtPmOffs.release();
  c->mtLegacy.release();
  c->mtBigLegacy.release();
  for (auto* q : {&c->mtLocGroups, &c->mtLocRecs, &c->mtLocPm, &c->mtLocScratch, &c->mtLocRegenCount}) q->release();
  c->mtLocOffs.release();
  c->mtLocRegen.release();
  c->mtLocRegenText.release();
  c->mtLocTab.release();
  c->spans.release();
  c->packed.release();
  c->digests.release();
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev2) (void)hipEventDestroy(c->ev2);
  if (c->ev3) (void)hipEventDestroy(c->ev3);
  if (c->evS0) (void)hipEventDestroy(c->evS0);
  if (c->evS1) (void)hipEventDestroy(c->evS1);
  if (c->ownStream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* fmt_last_error(const fmt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int fmt_sync(fmt_ctx* c) {
  if (c == nullptr) return FMT_E_USAGE;
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  return FMT_OK;
}

int fmt_get_stats(const fmt_ctx* cc, fmt_stats* out) {
  auto* c = const_cast<fmt_ctx*>(cc);
  if (c == nullptr || out == nullptr) return FMT_E_USAGE;
  if (c->timed) {
    FMT_HIP(c, hipEventSynchronize(c->ev1));
    float ms = 0;
    FMT_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (c->timed2) {
      float ms2 = 0;
      FMT_HIP(c, hipEventSynchronize(c->ev3));
      FMT_HIP(c, hipEventElapsedTime(&ms2, c->ev2, c->ev3));
      ms += ms2;
    }
    c->stats.kernel_ms = ms;
    c->stats.total_ms = ms;
  }
  *out = c->stats;
  return FMT_OK;
}

int fmt_device_info(fmt_ctx* c, char* buf, size_t cap) {
  if (c == nullptr || buf == nullptr || cap == 0) return FMT_E_USAGE;
  std::snprintf(buf, cap, "%s device=%d CUs=%d", c->arch.c_str(), c->device, c->numCUs);
  return FMT_OK;
}

// ------------------------------------------------------------------------------ SharedMap
static int mapValidate(fmt_ctx* c, const fmt_map_op* ops, uint64_t nOps, const uint64_t* offs, uint32_t nDocs,
                       uint32_t keyBound) {
  if (c == nullptr || (nOps > 0 && ops == nullptr) || offs == nullptr || keyBound == 0)
    return setErr(c, FMT_E_USAGE, "fmt_map_load: bad arguments");
  if (offs[0] != 0 || offs[nDocs] != nOps) return setErr(c, FMT_E_USAGE, "doc_op_offsets do not cover ops");
  for (uint32_t d = 0; d < nDocs; d++) {
    if (offs[d + 1] < offs[d]) return setErr(c, FMT_E_USAGE, "doc_op_offsets not monotone");
    for (uint64_t i = offs[d] + 1; i < offs[d + 1]; i++) {
      if (ops[i].seq <= ops[i - 1].seq) {
        char m[128];
        std::snprintf(m, sizeof m, "doc %u: seq %u after %u (ops must be in increasing seq order)", d,
                      ops[i].seq, ops[i - 1].seq);
        return setErr(c, FMT_E_DATA, m);
      }
    }
  }
  return FMT_OK;
}

static int mapStage(fmt_ctx* c, const fmt_map_op* ops, uint64_t nOps, const uint64_t* offs, uint32_t nDocs,
                    uint32_t keyBound, bool sparse) {
  FMT_HIP(c, hipSetDevice(c->device));
  FMT_HIP(c, c->mapOps.reserve(nOps));
  FMT_HIP(c, c->mapOffs.reserve(nDocs + 1ull));
  if (sparse) {
    FMT_HIP(c, c->mapEntries.reserve(nOps));
    FMT_HIP(c, c->mapCounts.reserve(nDocs));
  } else {
    FMT_HIP(c, c->mapOut.reserve(static_cast<size_t>(nDocs) * keyBound));
  }
  if (nOps) FMT_HIP(c, stagedCopy(c, c->mapOps.p, ops, nOps * sizeof(fmt_map_op), true));
  FMT_HIP(c, hipMemcpyAsync(c->mapOffs.p, offs, (nDocs + 1ull) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  c->mapNOps = nOps;
  c->mapDocs = nDocs;
  c->mapKeyBound = keyBound;
  c->mapLoaded = true;
  c->mapSparse = sparse;
  c->mapSparseRan = false;
  c->mapPendRan = false;
  c->mapOffsHost.assign(offs, offs + nDocs + 1ull);
  return FMT_OK;
}

int fmt_map_load(fmt_ctx* c, const fmt_map_op* ops, uint64_t nOps, const uint64_t* offs, uint32_t nDocs,
                 uint32_t keyBound) {
  const int rc = mapValidate(c, ops, nOps, offs, nDocs, keyBound);
  return rc != FMT_OK ? rc : mapStage(c, ops, nOps, offs, nDocs, keyBound, false);
}

int fmt_map_load_sparse(fmt_ctx* c, const fmt_map_op* ops, uint64_t nOps, const uint64_t* offs, uint32_t nDocs,
                        uint32_t keyBound) {
  const int rc = mapValidate(c, ops, nOps, offs, nDocs, keyBound);
  return rc != FMT_OK ? rc : mapStage(c, ops, nOps, offs, nDocs, keyBound, true);
}

int fmt_map_run_sparse(fmt_ctx* c) {
  if (c == nullptr || !c->mapLoaded || !c->mapSparse) return setErr(c, FMT_E_USAGE, "fmt_map_run_sparse before fmt_map_load_sparse");
  FMT_HIP(c, hipSetDevice(c->device));
  FMT_HIP(c, hipMemsetAsync(c->errWord.p, 0, sizeof(int), c->stream));
  FMT_HIP(c, hipEventRecord(c->ev0, c->stream));
  FMT_HIP(c, fmt_kernels::launchMapSparse(c->mapOps.p, c->mapOffs.p, c->mapDocs, c->mapKeyBound, c->mapEntries.p,
                                          c->mapCounts.p, c->errWord.p, c->numCUs, c->stream));
  FMT_HIP(c, hipEventRecord(c->ev1, c->stream));
  c->timed = true;
  c->timed2 = false;
  c->stats = fmt_stats{};
  c->stats.ops = c->mapNOps;
  c->stats.docs = c->mapDocs;
  c->stats.bytes_read = c->mapNOps * sizeof(fmt_map_op) + (c->mapDocs + 1ull) * sizeof(uint64_t);
  c->stats.bytes_written = static_cast<uint64_t>(c->mapDocs) * sizeof(uint32_t);  // + entries, at fetch
  c->stats.launches = 1;
  c->mapSparseRan = true;
  c->mapPendRan = false;
  return FMT_OK;
}

int fmt_map_fetch_sparse(fmt_ctx* c, uint32_t* counts, fmt_map_entry* entries, uint64_t capEntries, uint64_t* nEntries) {
  if (c == nullptr || counts == nullptr || !c->mapLoaded || !c->mapSparse)
    return setErr(c, FMT_E_USAGE, "fmt_map_fetch_sparse: nothing loaded");
  FMT_HIP(c, hipSetDevice(c->device));
  int errWord = 0;
  FMT_HIP(c, hipMemcpyAsync(&errWord, c->errWord.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipMemcpyAsync(counts, c->mapCounts.p, c->mapDocs * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  std::vector<uint64_t> packedOff(c->mapDocs + 1ull, 0);
  for (uint32_t d = 0; d < c->mapDocs; d++) packedOff[d + 1] = packedOff[d] + counts[d];
  const uint64_t n = packedOff[c->mapDocs];
  if (nEntries) *nEntries = n;
  c->stats.bytes_written = static_cast<uint64_t>(c->mapDocs) * sizeof(uint32_t) + n * sizeof(fmt_map_entry);
  if (entries != nullptr) {
    if (capEntries < n) return setErr(c, FMT_E_USAGE, "fmt_map_fetch_sparse: cap_entries below the live entries");
    FMT_HIP(c, c->mapPackedOff.reserve(c->mapDocs + 1ull));
    FMT_HIP(c, c->mapPacked.reserve(n));
    FMT_HIP(c, hipMemcpyAsync(c->mapPackedOff.p, packedOff.data(), (c->mapDocs + 1ull) * sizeof(uint64_t),
                              hipMemcpyHostToDevice, c->stream));
    FMT_HIP(c, fmt_kernels::launchMapSparsePack(c->mapEntries.p, c->mapOffs.p, c->mapCounts.p, c->mapPackedOff.p,
                                                c->mapDocs, c->mapPacked.p, c->stream));
    FMT_HIP(c, hipMemcpyAsync(entries, c->mapPacked.p, n * sizeof(fmt_map_entry), hipMemcpyDeviceToHost, c->stream));
    FMT_HIP(c, hipStreamSynchronize(c->stream));
  }
  if (errWord & 1) return setErr(c, FMT_E_DATA, "an op referenced a key id >= key_bound");
  if (errWord & 2) return setErr(c, FMT_E_CAPACITY, "a document exceeded the sparse path's keys or ops per document");
  return FMT_OK;
}

int fmt_map_pending_run(fmt_ctx* c, const fmt_map_local_op* events, uint64_t nEvents, const uint64_t* evOffs) {
  if (c == nullptr || !c->mapLoaded || !c->mapSparse || !c->mapSparseRan)
    return setErr(c, FMT_E_USAGE, "fmt_map_pending_run needs a sparse map run (fmt_map_run_sparse) first");
  if ((nEvents > 0 && events == nullptr) || evOffs == nullptr)
    return setErr(c, FMT_E_USAGE, "fmt_map_pending_run: null events or offsets");
  if (nEvents >= 0xFFFFFFFFull) return setErr(c, FMT_E_USAGE, "fmt_map_pending_run: too many events");
  const uint32_t n = c->mapDocs;
  if (evOffs[0] != 0 || evOffs[n] != nEvents) return setErr(c, FMT_E_USAGE, "doc_event_offsets must span [0, n_events)");
  std::vector<uint64_t> base(n);
  for (uint32_t d = 0; d < n; d++) {
    if (evOffs[d + 1] < evOffs[d]) return setErr(c, FMT_E_USAGE, "doc_event_offsets is not ascending");
    for (uint64_t i = evOffs[d]; i < evOffs[d + 1]; i++) {
      const fmt_map_local_op& e = events[i];
      const uint32_t kind = e.kind_value >> FMT_MAP_KIND_SHIFT;
      if (e.doc != d || e.event > FMT_MAP_EV_ROLLBACK || kind > FMT_MAP_CLEAR ||
          (kind != FMT_MAP_CLEAR && e.key >= c->mapKeyBound))
        return setErr(c, FMT_E_DATA, "a local event with a bad document, event, kind or key id");
    }
    base[d] = c->mapOffsHost[d] + evOffs[d];  // room for the sequenced entries plus one per event
  }
  FMT_HIP(c, hipSetDevice(c->device));
  FMT_HIP(c, c->mapEv.reserve(nEvents));
  FMT_HIP(c, c->mapEvOffs.reserve(n + 1ull));
  FMT_HIP(c, c->mapPendBase.reserve(n));
  FMT_HIP(c, c->mapPendScratch.reserve(fmt_kernels::mapPendingScratchBytes(nEvents)));
  FMT_HIP(c, c->mapPendOut.reserve(c->mapNOps + nEvents));
  FMT_HIP(c, c->mapPendCounts.reserve(n));
  FMT_HIP(c, c->mapPendStatus.reserve(n));
  if (nEvents) FMT_HIP(c, stagedCopy(c, c->mapEv.p, events, nEvents * sizeof(fmt_map_local_op), true));
  FMT_HIP(c, hipMemcpyAsync(c->mapEvOffs.p, evOffs, (n + 1ull) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  FMT_HIP(c, hipMemcpyAsync(c->mapPendBase.p, base.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  FMT_HIP(c, hipEventRecord(c->ev0, c->stream));
  FMT_HIP(c, fmt_kernels::launchMapPending(c->mapEv.p, c->mapEvOffs.p, c->mapEntries.p, c->mapOffs.p, c->mapCounts.p, n,
                                           c->mapPendScratch.p, c->mapPendBase.p, c->mapPendOut.p, c->mapPendCounts.p,
                                           c->mapPendStatus.p, c->stream));
  FMT_HIP(c, hipEventRecord(c->ev1, c->stream));
  // (the host arrays above are read by the copies before the call returns: synchronize)
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  c->timed = true;
  c->timed2 = false;
  c->stats = fmt_stats{};
  c->stats.ops = nEvents;
  c->stats.docs = n;
  c->stats.bytes_read = nEvents * sizeof(fmt_map_local_op) + c->mapNOps * sizeof(fmt_map_entry);
  c->stats.launches = 1;
  c->mapPendRan = true;
  return FMT_OK;
}

int fmt_map_pending_fetch(fmt_ctx* c, uint32_t* counts, int32_t* status, fmt_map_entry* entries, uint64_t capEntries,
                          uint64_t* nEntries) {
  if (c == nullptr || counts == nullptr || !c->mapPendRan)
    return setErr(c, FMT_E_USAGE, "fmt_map_pending_fetch before fmt_map_pending_run");
  const uint32_t n = c->mapDocs;
  FMT_HIP(c, hipSetDevice(c->device));
  FMT_HIP(c, hipMemcpyAsync(counts, c->mapPendCounts.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  if (status) FMT_HIP(c, hipMemcpyAsync(status, c->mapPendStatus.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  std::vector<uint64_t> packedOff(n + 1ull, 0);
  for (uint32_t d = 0; d < n; d++) packedOff[d + 1] = packedOff[d] + counts[d];
  const uint64_t total = packedOff[n];
  if (nEntries) *nEntries = total;
  if (entries != nullptr) {
    if (capEntries < total) return setErr(c, FMT_E_USAGE, "fmt_map_pending_fetch: cap_entries below the entries");
    FMT_HIP(c, c->mapPackedOff.reserve(n + 1ull));
    FMT_HIP(c, c->mapPacked.reserve(total));
    FMT_HIP(c, hipMemcpyAsync(c->mapPackedOff.p, packedOff.data(), (n + 1ull) * sizeof(uint64_t), hipMemcpyHostToDevice,
                              c->stream));
    FMT_HIP(c, fmt_kernels::launchMapSparsePack(c->mapPendOut.p, c->mapPendBase.p, c->mapPendCounts.p, c->mapPackedOff.p,
                                                n, c->mapPacked.p, c->stream));
    FMT_HIP(c, hipMemcpyAsync(entries, c->mapPacked.p, total * sizeof(fmt_map_entry), hipMemcpyDeviceToHost, c->stream));
    FMT_HIP(c, hipStreamSynchronize(c->stream));
  }
  return FMT_OK;
}

static int runMap(fmt_ctx* c, const fmt_map_op* ops, const uint64_t* offs, uint32_t nDocs, uint32_t keyBound,
                  uint64_t nOps, fmt_map_slot* out) {
  FMT_HIP(c, hipSetDevice(c->device));
  uint32_t* scratch = nullptr;
  if (fmt_kernels::mapLwwNeedsScratch(keyBound)) {  // key pool beyond the LDS table: HBM tables
    FMT_HIP(c, c->mapScratch.reserve(static_cast<size_t>(nDocs) * keyBound * 2));
    scratch = c->mapScratch.p;
  }
  FMT_HIP(c, hipMemsetAsync(c->errWord.p, 0, sizeof(int), c->stream));
  FMT_HIP(c, hipEventRecord(c->ev0, c->stream));
  FMT_HIP(c, fmt_kernels::launchMapLww(ops, offs, nDocs, keyBound, out, c->errWord.p, c->numCUs, c->stream, scratch));
  FMT_HIP(c, hipEventRecord(c->ev1, c->stream));
  c->timed = true;
  c->timed2 = false;
  c->stats = fmt_stats{};
  c->stats.ops = nOps;
  c->stats.docs = nDocs;
  const uint64_t nSlots = static_cast<uint64_t>(nDocs) * keyBound;
  c->stats.bytes_read = nOps * sizeof(fmt_map_op) + (nDocs + 1ull) * sizeof(uint64_t);
  c->stats.bytes_written = nSlots * sizeof(fmt_map_slot);
  c->stats.launches = 1;
  if (scratch != nullptr) {
    // HBM-table path: three table fills (8 B slot + 4 B kill + 4 B first per slot) and the finish
    // pass (reads slot + first, writes the slot) on top of the op stream and the kernel's atomics
    c->stats.bytes_written += nSlots * 16;
    c->stats.bytes_read += nSlots * 12;
    c->stats.launches = 5;
  }
  return FMT_OK;
}

int fmt_map_run(fmt_ctx* c) {
  if (c == nullptr || !c->mapLoaded || c->mapSparse) return setErr(c, FMT_E_USAGE, "fmt_map_run before fmt_map_load");
  return runMap(c, c->mapOps.p, c->mapOffs.p, c->mapDocs, c->mapKeyBound, c->mapNOps, c->mapOut.p);
}

int fmt_map_fetch(fmt_ctx* c, fmt_map_slot* out) {
  if (c == nullptr || out == nullptr || !c->mapLoaded || c->mapSparse)
    return setErr(c, FMT_E_USAGE, "fmt_map_fetch: nothing loaded");
  int errWord = 0;
  FMT_HIP(c, hipMemcpyAsync(&errWord, c->errWord.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipMemcpyAsync(out, c->mapOut.p, static_cast<size_t>(c->mapDocs) * c->mapKeyBound * sizeof(fmt_map_slot),
                            hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  if (errWord) return setErr(c, FMT_E_DATA, "an op referenced a key id >= key_bound");
  return FMT_OK;
}

int fmt_map_replay_device(fmt_ctx* c, const fmt_map_op* dOps, const uint64_t* dOffs, uint32_t nDocs,
                          uint32_t keyBound, fmt_map_slot* dOut) {
  if (c == nullptr || dOffs == nullptr || dOut == nullptr || keyBound == 0)
    return setErr(c, FMT_E_USAGE, "fmt_map_replay_device: bad arguments");
  // the HBM-table path runs 64-bit atomics on the output slots viewed as u64
  if (fmt_kernels::mapLwwNeedsScratch(keyBound) && (reinterpret_cast<uintptr_t>(dOut) & 7u) != 0)
    return setErr(c, FMT_E_USAGE, "fmt_map_replay_device: d_out must be 8-byte aligned for key_bound > 2560");
  return runMap(c, dOps, dOffs, nDocs, keyBound, 0, dOut);
}

int fmt_map_check(fmt_ctx* c) {
  if (c == nullptr) return FMT_E_USAGE;
  int errWord = 0;
  FMT_HIP(c, hipMemcpyAsync(&errWord, c->errWord.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  if (errWord) return setErr(c, FMT_E_DATA, "an op referenced a key id >= key_bound");
  return FMT_OK;
}

// ------------------------------------------------------------------------------ merge-tree
int fmt_mt_capacity(uint32_t* maxLeaves, uint32_t* maxChars, uint32_t* maxProps) {
  // A document is replayed in the large tier when it overflows the small one, so the limits are
  // the large tier's (the small tier's prop-set table is one larger: report the larger).
  const fmt_kernels::MtCaps big = fmt_kernels::mergeTreeCaps(true), small = fmt_kernels::mergeTreeCaps(false);
  if (maxLeaves) *maxLeaves = big.leaves;
  if (maxChars) *maxChars = big.chars;
  if (maxProps) *maxProps = big.props > small.props ? big.props : small.props;
  return FMT_OK;
}

// One huge-tier document (huge_engine.h): its HBM state sized from its op count and start, inputs
// (ops [o0, o1) of the staged batch, nSegs start segments at segsDev) and output buffers; header d.
// textPerOp bounds the merge area (zamboni appends build their text there).
static int setupHugeDoc(fmt_ctx* c, uint64_t textLen, uint32_t nPropsOps, uint32_t d, uint64_t o0,
                        uint64_t o1, const fmt_mt_snapshot_seg* segsDev, uint64_t nHeader, uint64_t nBody, int32_t minSeq,
                        int32_t seq, int32_t initClient, uint64_t textPerOp, uint64_t docChars) {
  const uint64_t nOps = o1 - o0, N = nHeader + nBody;
  c->mtHugeSlot[d] = static_cast<int32_t>(c->huge.size());
  c->huge.emplace_back();
  auto& H = c->huge.back();
  auto alloc = [&](size_t bytes, void** out) -> hipError_t {
    hipError_t e = hipMalloc(out, bytes ? bytes : 1);
    if (e == hipSuccess) H.allocs.push_back(*out);
    return e;
  };
  // a document whose state does not fit in device memory fails alone (FMT_E_CAPACITY): what it
  // allocated is released and it leaves the huge tier
  auto drop = [&](hipError_t e) -> int {
    for (void* q : H.allocs) (void)hipFree(q);
    c->huge.pop_back();
    c->mtHugeSlot[d] = -1;
    if (e == hipErrorOutOfMemory) {
      (void)hipGetLastError();
      return FMT_E_CAPACITY;
    }
    return hipErr(c, e, "setupHugeDoc");
  };
  fmt_huge::HugeState& S = H.state;
  uint64_t shapeBlocks = 0;
  if (nBody > 0) {
    fmt_huge::loadShape(nHeader, nBody, H.shape);
    for (uint32_t l = 0; l < H.shape[0]; l++) shapeBlocks += H.shape[1 + l];
  }
  const uint64_t blockCap = shapeBlocks + 2 * (N / 7 + 1) + 2 * nOps + 1024;
  if (blockCap > 0xFFFFFFF0ull || N + 3 * nOps + 16 > 0xFFFFFFF0ull) return drop(hipErrorOutOfMemory);
  S.blockCap = static_cast<uint32_t>(blockCap);
  S.idCap = static_cast<uint32_t>(N + 3 * nOps + 16);
  S.winCap = S.idCap;  // every leaf can be in the window (a wide remove puts many there)
  // the merge area: two halves (huge_engine.h compactText), each able to hold the document's whole
  // text twice over (its live merged text plus one run as long as the document)
  const uint64_t merge = std::max<uint64_t>(textPerOp * nOps + 65536, 4 * docChars + 131072);
  const uint64_t textCap = std::min<uint64_t>(textLen + merge, 0xFFFFFFF0ull);
  if (textCap <= textLen) return drop(hipErrorOutOfMemory);  // (offsets are 32-bit)
  const size_t nl = static_cast<size_t>(S.blockCap) * 8, nb = S.blockCap;
  void* p;
  hipError_t e;
#define FMT_ALLOC(field, T, count)                                      \
  if ((e = alloc((count) * sizeof(T), &p)) != hipSuccess) return drop(e); \
  S.field = static_cast<T*>(p);
  FMT_ALLOC(lLen, uint32_t, nl) FMT_ALLOC(lIns, int32_t, nl) FMT_ALLOC(lRm, int32_t, nl)
  FMT_ALLOC(lMlo, uint32_t, nl) FMT_ALLOC(lMhi, uint32_t, nl) FMT_ALLOC(lId, uint32_t, nl)
  FMT_ALLOC(lText, uint32_t, nl) FMT_ALLOC(lMeta, uint32_t, nl)
  FMT_ALLOC(bCount, uint32_t, nb) FMT_ALLOC(bParent, uint32_t, nb) FMT_ALLOC(bLeaf, uint32_t, nb)
  FMT_ALLOC(bScour, int32_t, nb) FMT_ALLOC(bChild, uint32_t, nb * 8) FMT_ALLOC(bGroup, uint32_t, nb)
  FMT_ALLOC(bSlot, uint32_t, nb) FMT_ALLOC(freeBlk, uint32_t, nb)
  FMT_ALLOC(gSlotBlk, uint32_t, static_cast<size_t>(fmt_huge::kGroupCap) * fmt_huge::kSlotCap)
  FMT_ALLOC(gSlotStable, int32_t, static_cast<size_t>(fmt_huge::kGroupCap) * fmt_huge::kSlotCap)
  FMT_ALLOC(leafBlk, uint32_t, S.idCap) FMT_ALLOC(winIdx, uint32_t, S.idCap)
  FMT_ALLOC(wRec, uint32_t, static_cast<size_t>(S.winCap) * 4) FMT_ALLOC(wMask, uint32_t, static_cast<size_t>(S.winCap) * 2)
  FMT_ALLOC(wBlk, uint32_t, S.winCap)
  FMT_ALLOC(wLeaf, uint32_t, S.winCap)
  // the merge area only; the batch text is read in place (huge_engine.h HugeState::base)
  FMT_ALLOC(text, uint16_t, textCap - textLen)
  FMT_ALLOC(props, uint32_t, static_cast<size_t>(fmt_huge::kPropCap) * fmt_huge::kPropWords)
  FMT_ALLOC(pClass, uint32_t, fmt_huge::kPropCap)
  FMT_ALLOC(pHead, uint32_t, 2ull * fmt_huge::kPropHash)
  FMT_ALLOC(pNext, uint32_t, 2ull * fmt_huge::kPropCap)
  S.text -= textLen;
  S.base = c->mtText.p;
  S.textLen = textLen;
  S.textCap = textCap;
  fmt_huge::HugeInputs& I = H.in;
  I.ops = c->mtOps.p;
  I.begin = o0;
  I.end = o1;
  I.propsOff = c->mtPropsOff.p;
  I.propsKv = c->mtPropsKv.p;
  I.nPropsOps = nPropsOps;
  I.segs = segsDev;
  I.nSegs = static_cast<uint32_t>(N);
  I.segProps = c->mtSegProps.empty() ? 0u : c->mtSegProps[d];
  // SnapshotV1 merge info of a summary-loaded document's segments (header chunk)
  I.info = nullptr;
  I.stamps = c->mtHasSnapInfo ? c->mtSnapStamps.p : nullptr;
  if (c->mtHasSnapInfo && c->mtSnapHost.size() > d && c->mtSnapHost[d].loaded) I.info = c->mtSnapInfo.p + c->mtSnapHost[d].first_seg;
  // V1 body-chunk segments with merge info (FMT_MT_F_LOADSEG ops) name rows of the batch's table
  I.infoAll = c->mtHasSnapInfo ? c->mtSnapInfo.p : nullptr;
  I.nInfoAll = c->mtHasSnapInfo ? c->mtNSnapSegs : 0;
  // catch-up ranges go to the document's slab, as in the other tiers
  I.catchup = nullptr;
  I.catchupCap = 0;
  S.cuIds = nullptr;
  if (c->mtHasCatchup && c->mtCuOffsHost[d + 1] > c->mtCuOffsHost[d]) {
    I.catchup = c->mtCatchup.p + c->mtCuOffsHost[d];
    I.catchupCap = static_cast<uint32_t>(std::min<uint64_t>(c->mtCuOffsHost[d + 1] - c->mtCuOffsHost[d], 0xFFFFFFFFull));
    if ((e = alloc(static_cast<size_t>(S.idCap) * sizeof(uint32_t), &p)) != hipSuccess) return drop(e);
    S.cuIds = static_cast<uint32_t*>(p);
  }
  // relative positions: the batch's table, and the document's marker list
  I.relpos = c->mtNRelpos ? c->mtRelpos.p : nullptr;
  I.nRelpos = c->mtNRelpos;
  I.markerKey = c->mtMarkerKey;
  // annotate-adjust: the batch's tables (computed numbers, PropertiesManager records), the leaf id ->
  // output index map of the getAtSeq output
  I.adj = c->mtHasAdjust ? c->mtAdjTab.p : nullptr;
  I.doc = d;
  S.outIdx = nullptr;
  if (c->mtHasAdjust) {
    if ((e = alloc(static_cast<size_t>(S.idCap) * sizeof(uint32_t), &p)) != hipSuccess) return drop(e);
    S.outIdx = static_cast<uint32_t*>(p);
  }
  S.mkIds = nullptr;
  S.mkCap = 0;
  if (c->mtNRelpos) {
    if ((e = alloc(static_cast<size_t>(S.idCap) * sizeof(uint32_t), &p)) != hipSuccess) return drop(e);
    S.mkIds = static_cast<uint32_t*>(p);
    S.mkCap = S.idCap;
  }
  // remove-order entries (SnapshotV1) go to the document's slab too
  I.rmOrder = nullptr;
  I.rmOrderCap = 0;
  S.rmIds = nullptr;
  if (c->mtHasRmOrder && c->mtRmOffsHost[d + 1] > c->mtRmOffsHost[d]) {
    I.rmOrder = c->mtRmOrder.p + c->mtRmOffsHost[d];
    I.rmOrderCap = static_cast<uint32_t>(std::min<uint64_t>(c->mtRmOffsHost[d + 1] - c->mtRmOffsHost[d], 0xFFFFFFFFull));
    if ((e = alloc(static_cast<size_t>(S.idCap) * sizeof(uint32_t), &p)) != hipSuccess) return drop(e);
    S.rmIds = static_cast<uint32_t*>(p);
  }
  I.shape = nullptr;
  if (!H.shape.empty()) {
    if ((e = alloc(H.shape.size() * sizeof(uint32_t), &p)) != hipSuccess) return drop(e);
    FMT_HIP(c, hipMemcpyAsync(p, H.shape.data(), H.shape.size() * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    I.shape = static_cast<const uint32_t*>(p);
  }
  I.snapMinSeq = minSeq;
  I.snapSeq = seq;
  I.initClient = initClient;
  fmt_kernels::HugeOut& O = H.out;
  O.header = c->mtHdr.p + d;
  O.capLeaves = N + 3 * nOps + 8;
  O.capChars = docChars + 8;  // (every unit the document can hold: its start plus its inserts)
  if ((e = alloc(O.capLeaves * sizeof(fmt_mt_leaf), &p)) != hipSuccess) return drop(e);
  O.leaves = static_cast<fmt_mt_leaf*>(p);
  if ((e = alloc(O.capChars * sizeof(uint16_t), &p)) != hipSuccess) return drop(e);
  O.chars = static_cast<uint16_t*>(p);
  if ((e = alloc(fmt_huge::kPropCap * sizeof(fmt_mt_propset), &p)) != hipSuccess) return drop(e);
  O.props = static_cast<fmt_mt_propset*>(p);
  O.cls = S.pClass;
  O.legacy = nullptr;  // annotate-adjust batches: per leaf the getAtSeq(minSeq) prop set
  if (c->mtHasAdjust) {
    if ((e = alloc(O.capLeaves * sizeof(uint16_t), &p)) != hipSuccess) return drop(e);
    O.legacy = static_cast<uint16_t*>(p);
  }
  if ((e = alloc(fmt_huge::HugeDoc::kProf * sizeof(unsigned long long), &p)) != hipSuccess) return drop(e);
  O.prof = static_cast<unsigned long long*>(p);
  // live obliterates: at most one per op of the document is alive at once (HBM; batches with obliterates)
  S.obRec = S.obUsed = S.obSeq = S.obStart = nullptr;
  S.obCap = 0;
  if (c->mtObliterate && nOps > 0) {
    if (nOps > 0x0FFFFFFFull) return drop(hipErrorOutOfMemory);
    S.obCap = static_cast<uint32_t>(std::max<uint64_t>(nOps, fmt_ckpt::kObSlots));  // (a checkpoint keeps its slot ids)
    if ((e = alloc(9ull * S.obCap * sizeof(uint32_t), &p)) != hipSuccess) return drop(e);
    S.obRec = static_cast<uint32_t*>(p);
    S.obUsed = S.obRec + 6ull * S.obCap;
    S.obSeq = S.obUsed + S.obCap;
    S.obStart = S.obSeq + S.obCap;
  }
  // remove clients 64..253: the per-leaf-id side table (zeroed, kHiWords words per id) and its per-leaf
  // output (kHiOutWords 64-bit words per leaf: ids 64..127, 128..191, 192..253)
  S.hiMask = nullptr;
  O.leavesHi = nullptr;
  if (c->mtHiClients) {
    constexpr size_t kW = fmt_huge::kHiWords;
    if ((e = alloc(kW * S.idCap * sizeof(uint32_t), &p)) != hipSuccess) return drop(e);
    FMT_HIP(c, hipMemsetAsync(p, 0, kW * S.idCap * sizeof(uint32_t), c->stream));
    S.hiMask = static_cast<uint32_t*>(p);
    if ((e = alloc(O.capLeaves * fmt_huge::kHiOutWords * sizeof(uint64_t), &p)) != hipSuccess) return drop(e);
    O.leavesHi = static_cast<uint64_t*>(p);
  }
  return FMT_OK;
}

int fmt_mt_load(fmt_ctx* c, const fmt_mt_batch* b) {
  if (c == nullptr || b == nullptr || b->doc_op_offsets == nullptr || (b->n_ops && b->ops == nullptr))
    return setErr(c, FMT_E_USAGE, "fmt_mt_load: bad arguments");
  const uint32_t n = b->n_docs;
  if (b->doc_op_offsets[0] != 0 || b->doc_op_offsets[n] != b->n_ops)
    return setErr(c, FMT_E_USAGE, "doc_op_offsets do not cover ops");
  // one pass over the op records on host threads: counts, and the first invalid record
  struct OpScan {
    uint64_t insertChars = 0, catchupOps = 0, rmOrderOps = 0;
    bool obliterates = false, local = false, hiClients = false;
    uint64_t errAt = ~0ull;
    int errCode = FMT_OK;
    const char* err = nullptr;
  };
  std::vector<OpScan> scans(hostWorkers());
  parallelChunks(b->n_ops, [&](uint64_t lo, uint64_t hi, unsigned t) {
    OpScan& S = scans[t];
    auto bad = [&](uint64_t i, int code, const char* what) {
      S.errAt = i;
      S.errCode = code;
      S.err = what;
    };
    for (uint64_t i = lo; i < hi; i++) {
      const fmt_mt_op& op = b->ops[i];
      if (op.flags & FMT_MT_F_CATCHUP) S.catchupOps++;
      if (op.flags & FMT_MT_F_RMORDER) S.rmOrderOps++;
      if (op.flags & FMT_MT_F_LOCAL_ANY) S.local = true;
      if (op.client > 63 && op.client != FMT_MT_CLIENT_NONCOLLAB) S.hiClients = true;
      if (op.flags & FMT_MT_F_LOADSEG) {  // a SnapshotV1 body segment: its merge info row in range
        if (op.type != FMT_MT_INSERT || b->snapshot_info == nullptr || op.pos1 < 0 ||
            static_cast<uint64_t>(op.pos1) >= b->n_snapshot_segs ||
            b->snapshot_info[op.pos1].rm_first + static_cast<uint64_t>(b->snapshot_info[op.pos1].rm_count) > b->n_snapshot_stamps) {
          bad(i, FMT_E_DATA, "a loader segment (FMT_MT_F_LOADSEG) without a valid merge-info row");
          return;
        }
      }
      if (op.type == FMT_MT_INSERT) {
        if (static_cast<uint64_t>(op.payload) + fmt_mt_op_len(&op) > b->text_len) {
          bad(i, FMT_E_DATA, "insert payload outside the text arena");
          return;
        }
        S.insertChars += fmt_mt_op_len(&op);
      } else if (op.type == FMT_MT_ANNOTATE) {
        if (op.payload >= b->n_props_ops) {
          bad(i, FMT_E_DATA, "annotate props op id out of range");
          return;
        }
      } else if (op.type == FMT_MT_OBLITERATE || op.type == FMT_MT_OBLITERATE_SIDED) {
        S.obliterates = true;
      } else if (op.type != FMT_MT_REMOVE) {
        bad(i, FMT_E_UNSUPPORTED, "op type not supported by this engine build");
        return;
      }
    }
  });
  uint64_t insertChars = 0, catchupOps = 0, rmOrderOps = 0;
  bool obliterates = false, local = false, hiClients = false;
  const OpScan* firstBad = nullptr;
  for (const OpScan& S : scans) {
    insertChars += S.insertChars;
    catchupOps += S.catchupOps;
    rmOrderOps += S.rmOrderOps;
    obliterates = obliterates || S.obliterates;
    local = local || S.local;
    hiClients = hiClients || S.hiClients;
    if (S.err != nullptr && (firstBad == nullptr || S.errAt < firstBad->errAt)) firstBad = &S;
  }
  if (firstBad != nullptr) return setErr(c, firstBad->errCode, firstBad->err);
  // f4 batches run the Loc variants (annotate-adjust and remote ops with relative positions too since
  // round 6): features they do not combine with are refused
  if (local && (obliterates || catchupOps || rmOrderOps || b->snapshot_info != nullptr))
    return setErr(c, FMT_E_UNSUPPORTED,
                  "local-client records (FMT_MT_F_LOCAL_ANY) do not combine with obliterate, catch-up, remove order "
                  "or SnapshotV1 merge info");
  if (b->snapshots) {
    for (uint32_t d = 0; d < n; d++) {
      const fmt_mt_snapshot_doc& sd = b->snapshots[d];
      if (!sd.loaded) continue;
      if (b->snapshot_segs == nullptr || sd.first_seg + sd.n_header + sd.n_body > b->n_snapshot_segs)
        return setErr(c, FMT_E_USAGE, "snapshot segments out of range");
      for (uint64_t k = sd.first_seg; k < sd.first_seg + sd.n_header + sd.n_body; k++) {
        const fmt_mt_snapshot_seg& sg = b->snapshot_segs[k];
        const uint32_t len = sg.len & ~FMT_MT_SEG_MARKER;
        if ((sg.len & FMT_MT_SEG_MARKER) != 0 && len != 1)
          return setErr(c, FMT_E_DATA, "a marker segment has length 1");
        if (static_cast<uint64_t>(sg.text) + len > b->text_len)
          return setErr(c, FMT_E_DATA, "snapshot segment text outside the text arena");
        if (sg.props != FMT_MT_NO_PROPS && sg.props >= b->n_props_ops)
          return setErr(c, FMT_E_DATA, "snapshot segment props op id out of range");
        insertChars += len;
      }
    }
  }
  uint64_t initChars = 0;
  if (b->doc_init) {
    for (uint32_t d = 0; d < n; d++) {
      if (static_cast<uint64_t>(b->doc_init[2 * d]) + b->doc_init[2 * d + 1] > b->text_len)
        return setErr(c, FMT_E_DATA, "initial text outside the text arena");
      initChars += b->doc_init[2 * d + 1];
    }
  }
  // Annotate-adjust entries (FMT_MT_VALUE_ADJUST + row index) in the props ops: validated here; per
  // document they size its computed-number slab and decide whether its legacy summary is exact.
  const uint32_t nKvAll = b->props_off ? b->props_off[b->n_props_ops] : 0;
  std::vector<uint32_t> adjCount(b->n_props_ops, 0);  // adjust entries per props op
  bool anyAdjust = false;
  for (uint32_t op = 0; b->props_off && op < b->n_props_ops; op++) {
    const uint32_t a = b->props_off[op], e = b->props_off[op + 1];
    if (a > e || e > nKvAll) return setErr(c, FMT_E_USAGE, "props_off is not ascending");
    for (uint32_t t = a; t < e; t++) {
      const uint32_t v = b->props_kv[t] & 0xFFFFu;
      if (v == FMT_MT_VALUE_ADJUST) {
        if (t + 1 >= e || b->adjusts == nullptr || b->props_kv[t + 1] >= b->n_adjusts)
          return setErr(c, FMT_E_DATA, "annotate-adjust entry without a valid adjust row");
        adjCount[op]++;
        anyAdjust = true;
        t++;
      }
    }
  }
  if (b->doc_value_base != nullptr) {
    for (uint32_t d = 0; d < n; d++)
      if (b->doc_value_base[d + 1] < b->doc_value_base[d])
        return setErr(c, FMT_E_USAGE, "doc_value_base is not ascending");
    if (b->value_num != nullptr && b->doc_value_base[n] >= b->n_values)
      return setErr(c, FMT_E_USAGE, "doc_value_base reaches past value_num");
    c->mtValueBaseHost.assign(b->doc_value_base, b->doc_value_base + n + 1);
  } else {
    c->mtValueBaseHost.clear();
  }
  if (anyAdjust) {
    if (b->value_num == nullptr && b->n_values > 0) return setErr(c, FMT_E_USAGE, "adjusts need value_num");
    for (uint32_t t = 0; t < nKvAll; t++) {
      const uint32_t v = b->props_kv[t] & 0xFFFFu;
      if (v == FMT_MT_VALUE_ADJUST) {
        t++;
      } else if (v >= FMT_MT_VALUE_COMPUTED) {
        return setErr(c, FMT_E_USAGE, "host value ids must stay below FMT_MT_VALUE_COMPUTED in a batch with adjusts");
      }
    }
  }
  const fmt_kernels::MtCaps caps = fmt_kernels::mergeTreeCaps(false);
  FMT_HIP(c, hipSetDevice(c->device));
  FMT_HIP(c, c->mtOps.reserve(b->n_ops));
  FMT_HIP(c, c->mtOffs.reserve(n + 1ull));
  FMT_HIP(c, c->mtText.reserve(b->text_len));
  FMT_HIP(c, c->mtInit.reserve(2ull * n));
  FMT_HIP(c, c->mtPropsOff.reserve(b->n_props_ops + 1ull));
  const uint32_t nKv = b->props_off ? b->props_off[b->n_props_ops] : 0;
  FMT_HIP(c, c->mtPropsKv.reserve(nKv));
  FMT_HIP(c, c->mtHdr.reserve(n));
  FMT_HIP(c, c->mtLeaves.reserve(static_cast<size_t>(n) * caps.leaves));
  FMT_HIP(c, c->mtChars.reserve(static_cast<size_t>(n) * caps.chars));
  FMT_HIP(c, c->mtProps.reserve(static_cast<size_t>(n) * caps.props));
  FMT_HIP(c, c->mtEsc.reserve(n + 1ull));
  FMT_HIP(c, c->mtEsc2.reserve(n + 1ull));
  FMT_HIP(c, c->mtEsc3.reserve(n + 1ull));
  FMT_HIP(c, c->mtSched.reserve(4));
  c->mtBigSlot.assign(n, -1);
  // Catch-up slabs: kCatchupPerOp ranges per flagged op plus kCatchupPerDoc per document that has
  // any; a document that needs more reports FMT_E_CAPACITY.
  c->mtHasCatchup = catchupOps > 0;
  if (c->mtHasCatchup) {
    constexpr uint64_t kCatchupPerOp = 16, kCatchupPerDoc = 16;
    c->mtCuOffsHost.assign(n + 1ull, 0);
    for (uint32_t d = 0; d < n; d++) {
      uint64_t f = 0;
      for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++)
        f += (b->ops[i].flags & FMT_MT_F_CATCHUP) ? 1 : 0;
      c->mtCuOffsHost[d + 1] = c->mtCuOffsHost[d] + (f ? f * kCatchupPerOp + kCatchupPerDoc : 0);
    }
    FMT_HIP(c, c->mtCuOffs.reserve(n + 1ull));
    FMT_HIP(c, c->mtCatchup.reserve(c->mtCuOffsHost[n]));
  }
  // Remove-order slabs: kRmPerOp entries per flagged remove plus kRmPerDoc per document that has
  // any (split copies included); a document that needs more reports FMT_E_CAPACITY.
  c->mtHasRmOrder = rmOrderOps > 0;
  if (c->mtHasRmOrder) {
    constexpr uint64_t kRmPerOp = 64, kRmPerDoc = 256;
    c->mtRmOffsHost.assign(n + 1ull, 0);
    for (uint32_t d = 0; d < n; d++) {
      uint64_t f = 0;
      for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++)
        f += (b->ops[i].flags & FMT_MT_F_RMORDER) ? 1 : 0;
      c->mtRmOffsHost[d + 1] = c->mtRmOffsHost[d] + (f ? f * kRmPerOp + kRmPerDoc : 0);
    }
    FMT_HIP(c, c->mtRmOffs.reserve(n + 1ull));
    FMT_HIP(c, c->mtRmOrder.reserve(c->mtRmOffsHost[n]));
  }
  auto cp = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
    return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream) : hipSuccess;
  };
  // Computed-number slabs: 64 per adjust entry of the document's annotates + 64 (at most 0x7fff, the
  // computed id range: one adjust over a range can compute a new number per leaf it hits); a document
  // that computes more distinct numbers reports FMT_E_CAPACITY. PropertiesManager record slabs
  // (mt_engine.h Doc::pm*): 32 per change of the document's annotates + 256 records.
  c->mtHasAdjust = anyAdjust;
  if (anyAdjust) {
    c->mtNumOffsHost.assign(n + 1ull, 0);
    c->mtPmOffsHost.assign(n + 1ull, 0);
    for (uint32_t d = 0; d < n; d++) {
      uint64_t f = 0, g = 0;
      for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++) {
        const fmt_mt_op& op = b->ops[i];
        if (op.type != FMT_MT_ANNOTATE) continue;
        f += adjCount[op.payload];
        g += b->props_off[op.payload + 1] - b->props_off[op.payload];
      }
      c->mtNumOffsHost[d + 1] = c->mtNumOffsHost[d] + (f ? std::min<uint64_t>(64 * f + 64, 0x7FFF) : 0);
      c->mtPmOffsHost[d + 1] = c->mtPmOffsHost[d] + (g ? std::min<uint64_t>(32 * g + 256, 1u << 20) : 0);
    }
    // the host's numbers, ascending, each with the first value id that holds it: one list for the
    // batch, or per document with its local ids (doc_value_base)
    std::vector<double> sv;
    std::vector<uint32_t> si, so;
    auto sortNumbers = [&](uint32_t lo, uint32_t hi, uint32_t base) {
      std::vector<std::pair<double, uint32_t>> nums;
      for (uint32_t i = lo; b->value_num && i < hi; i++)
        if (b->value_num[base + i] == b->value_num[base + i])
          nums.emplace_back(b->value_num[base + i] == 0.0 ? 0.0 : b->value_num[base + i], i);
      std::stable_sort(nums.begin(), nums.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      const size_t first = sv.size();
      for (const auto& [x, i] : nums) {
        if (sv.size() > first && sv.back() == x) continue;  // (one text per number: the first id)
        sv.push_back(x);
        si.push_back(i);
      }
    };
    if (b->doc_value_base != nullptr) {
      so.assign(1, 0);
      for (uint32_t d = 0; d < n; d++) {
        sortNumbers(1, b->doc_value_base[d + 1] - b->doc_value_base[d] + 1, b->doc_value_base[d]);
        so.push_back(static_cast<uint32_t>(sv.size()));
      }
    } else {
      sortNumbers(0, b->n_values, 0);
    }
    c->mtNAdjusts = b->n_adjusts;
    c->mtNValues = b->value_num ? b->n_values : 0u;
    c->mtNNumSorted = static_cast<uint32_t>(sv.size());
    FMT_HIP(c, c->mtAdjusts.reserve(b->n_adjusts));
    FMT_HIP(c, c->mtValueNum.reserve(c->mtNValues));
    FMT_HIP(c, c->mtNumSorted.reserve(sv.size()));
    FMT_HIP(c, c->mtNumSortedId.reserve(si.size()));
    FMT_HIP(c, c->mtNumOffs.reserve(n + 1ull));
    FMT_HIP(c, c->mtNums.reserve(c->mtNumOffsHost[n]));
    FMT_HIP(c, c->mtNumCount.reserve(n));
    FMT_HIP(c, c->mtPmOffs.reserve(n + 1ull));
    FMT_HIP(c, c->mtPm.reserve(4 * c->mtPmOffsHost[n]));
    FMT_HIP(c, c->mtLegacy.reserve(static_cast<size_t>(n) * caps.leaves));
    FMT_HIP(c, cp(c->mtPmOffs.p, c->mtPmOffsHost.data(), (n + 1ull) * sizeof(uint64_t)));
    FMT_HIP(c, cp(c->mtAdjusts.p, b->adjusts, b->n_adjusts * sizeof(fmt_mt_adjust)));
    FMT_HIP(c, cp(c->mtValueNum.p, b->value_num, c->mtNValues * sizeof(double)));
    FMT_HIP(c, cp(c->mtNumSorted.p, sv.data(), sv.size() * sizeof(double)));
    FMT_HIP(c, cp(c->mtNumSortedId.p, si.data(), si.size() * sizeof(uint32_t)));
    if (b->doc_value_base != nullptr) {
      FMT_HIP(c, c->mtValueBase.reserve(n + 1ull));
      FMT_HIP(c, c->mtNumSortedOffs.reserve(n + 1ull));
      FMT_HIP(c, cp(c->mtValueBase.p, b->doc_value_base, (n + 1ull) * sizeof(uint32_t)));
      FMT_HIP(c, cp(c->mtNumSortedOffs.p, so.data(), (n + 1ull) * sizeof(uint32_t)));
    }
    FMT_HIP(c, cp(c->mtNumOffs.p, c->mtNumOffsHost.data(), (n + 1ull) * sizeof(uint64_t)));
    FMT_HIP(c, hipMemsetAsync(c->mtNumCount.p, 0, n * sizeof(uint32_t), c->stream));
    fmt_mt::AdjustTables T{};
    T.adjusts = c->mtAdjusts.p;
    T.nAdjusts = b->n_adjusts;
    T.nValues = c->mtNValues;
    T.valueNum = c->mtValueNum.p;
    T.numSorted = c->mtNumSorted.p;
    T.numSortedId = c->mtNumSortedId.p;
    T.valueBase = b->doc_value_base != nullptr ? c->mtValueBase.p : nullptr;
    T.numSortedOffs = b->doc_value_base != nullptr ? c->mtNumSortedOffs.p : nullptr;
    T.nNumSorted = c->mtNNumSorted;
    T.nums = c->mtNums.p;
    T.numOffsets = c->mtNumOffs.p;
    T.numCount = c->mtNumCount.p;
    T.pm = c->mtPm.p;
    T.pmOffsets = c->mtPmOffs.p;
    FMT_HIP(c, c->mtAdjTab.reserve(1));
    FMT_HIP(c, cp(c->mtAdjTab.p, &T, sizeof T));
    FMT_HIP(c, hipStreamSynchronize(c->stream));  // (sv / si / T are about to go out of scope)
  }
  c->mtLocal = local;
  c->mtHiClients = hiClients;
  if (local) {
    // Per-document slabs, sized from the document's local records (a document that needs more reports
    // FMT_E_CAPACITY): 4 + 2 pending groups per submission (a reconnect replaces a group by one per
    // segment), 32 group records per submission (hits and split copies; deleted ones compact away),
    // 64 PropertiesManager records per key of a local annotate (annotate-adjust batches: + 32 per key
    // of any annotate, whose remote changes stay listed until minSeq passes them), regenerated ops /
    // text per reconnect, and normalization scratch for a document that reconnects.
    const fmt_kernels::MtCaps big = fmt_kernels::mergeTreeCaps(true);
    std::vector<uint64_t> offs(6 * (n + 1ull), 0);
    for (uint32_t d = 0; d < n; d++) {
      uint64_t sub = 0, keys = 0, regens = 0, text = 0;
      for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++) {
        const fmt_mt_op& op = b->ops[i];
        if (op.flags & FMT_MT_F_REGEN) regens++;
        if (anyAdjust && op.type == FMT_MT_ANNOTATE && !(op.flags & (FMT_MT_F_LOCAL | FMT_MT_F_ROLLBACK)))
          keys += (b->props_off[op.payload + 1] - b->props_off[op.payload] + 1) / 2;
        if (!(op.flags & FMT_MT_F_LOCAL)) continue;
        sub++;
        if (op.type == FMT_MT_INSERT) text += fmt_mt_op_len(&op);
        if (op.type == FMT_MT_ANNOTATE) keys += b->props_off[op.payload + 1] - b->props_off[op.payload];
      }
      const uint64_t cap[6] = {sub ? std::min<uint64_t>(6 * sub + 64 + (regens ? big.leaves : 0), 1u << 22) : 0,
                               sub ? std::min<uint64_t>(32 * sub + 1024, 1u << 24) : 0,
                               keys ? std::min<uint64_t>(64 * keys + 512, 1u << 22) : 0,
                               regens ? std::min<uint64_t>(regens * std::min<uint64_t>(8 * sub + 64, big.leaves), 1u << 22) : 0,
                               regens ? std::min<uint64_t>(regens * std::min<uint64_t>(text, big.chars) + 64, 1u << 26) : 0,
                               regens ? 15ull * big.leaves + big.chars / 2 + 64 : 0};
      for (int k = 0; k < 6; k++) offs[k * (n + 1ull) + d + 1] = offs[k * (n + 1ull) + d] + cap[k];
    }
    auto total = [&](int k) { return offs[k * (n + 1ull) + n]; };
    FMT_HIP(c, c->mtLocOffs.reserve(6 * (n + 1ull)));
    FMT_HIP(c, c->mtLocGroups.reserve(8 * total(0)));
    FMT_HIP(c, c->mtLocRecs.reserve(2 * total(1)));
    FMT_HIP(c, c->mtLocPm.reserve(4 * total(2)));
    FMT_HIP(c, c->mtLocRegen.reserve(total(3)));
    FMT_HIP(c, c->mtLocRegenText.reserve(total(4)));
    FMT_HIP(c, c->mtLocScratch.reserve(total(5)));
    FMT_HIP(c, c->mtLocRegenCount.reserve(2ull * n));
    FMT_HIP(c, c->mtLocTab.reserve(1));
    FMT_HIP(c, cp(c->mtLocOffs.p, offs.data(), offs.size() * sizeof(uint64_t)));
    FMT_HIP(c, hipMemsetAsync(c->mtLocRegenCount.p, 0, 2ull * n * sizeof(uint32_t), c->stream));
    const uint64_t* O = c->mtLocOffs.p;
    fmt_mt::LocalTables T{c->mtLocGroups.p, O, c->mtLocRecs.p, O + (n + 1ull), c->mtLocPm.p, O + 2 * (n + 1ull),
                          c->mtLocRegen.p, O + 3 * (n + 1ull), c->mtLocRegenText.p, O + 4 * (n + 1ull),
                          c->mtLocRegenCount.p, c->mtLocScratch.p, O + 5 * (n + 1ull)};
    FMT_HIP(c, cp(c->mtLocTab.p, &T, sizeof T));
    c->mtLocRegenOffsHost.assign(offs.begin() + 3 * (n + 1ull), offs.begin() + 4 * (n + 1ull));
    c->mtLocRegenTextOffsHost.assign(offs.begin() + 4 * (n + 1ull), offs.begin() + 5 * (n + 1ull));
    FMT_HIP(c, hipStreamSynchronize(c->stream));  // (offs / T are about to go out of scope)
  }
  FMT_HIP(c, stagedCopy(c, c->mtOps.p, b->ops, b->n_ops * sizeof(fmt_mt_op), true));
  FMT_HIP(c, cp(c->mtOffs.p, b->doc_op_offsets, (n + 1ull) * sizeof(uint64_t)));
  FMT_HIP(c, stagedCopy(c, c->mtText.p, b->text, b->text_len * sizeof(uint16_t), true));
  if (b->doc_init) FMT_HIP(c, cp(c->mtInit.p, b->doc_init, 2ull * n * sizeof(uint32_t)));
  c->mtHasSnap = b->snapshots != nullptr;
  if (c->mtHasSnap) {
    FMT_HIP(c, c->mtSnap.reserve(n));
    FMT_HIP(c, c->mtSnapSegs.reserve(b->n_snapshot_segs));
    FMT_HIP(c, cp(c->mtSnap.p, b->snapshots, n * sizeof(fmt_mt_snapshot_doc)));
    FMT_HIP(c, stagedCopy(c, c->mtSnapSegs.p, b->snapshot_segs, b->n_snapshot_segs * sizeof(fmt_mt_snapshot_seg), true));
  }
  c->mtHasSnapInfo = c->mtHasSnap && b->snapshot_info != nullptr;
  c->mtNSnapSegs = b->n_snapshot_segs;
  if (c->mtHasSnapInfo) {
    FMT_HIP(c, c->mtSnapInfo.reserve(b->n_snapshot_segs));
    FMT_HIP(c, c->mtSnapStamps.reserve(b->n_snapshot_stamps));
    FMT_HIP(c, cp(c->mtSnapInfo.p, b->snapshot_info, b->n_snapshot_segs * sizeof(fmt_mt_snapshot_info)));
    FMT_HIP(c, cp(c->mtSnapStamps.p, b->snapshot_stamps, b->n_snapshot_stamps * sizeof(fmt_mt_stamp)));
    for (uint64_t k = 0; k < b->n_snapshot_stamps && !c->mtHiClients; k++) c->mtHiClients = b->snapshot_stamps[k].client > 63;
    for (uint64_t k = 0; k < b->n_snapshot_segs && !c->mtHiClients; k++) c->mtHiClients = b->snapshot_info[k].ins_client > 63;
  }
  c->mtNRelpos = b->relpos ? b->n_relpos : 0u;
  c->mtMarkerKey = b->marker_id_key;
  if (c->mtNRelpos) {
    FMT_HIP(c, c->mtRelpos.reserve(c->mtNRelpos));
    FMT_HIP(c, cp(c->mtRelpos.p, b->relpos, c->mtNRelpos * sizeof(fmt_mt_relpos)));
  }
  if (c->mtHasCatchup) FMT_HIP(c, cp(c->mtCuOffs.p, c->mtCuOffsHost.data(), (n + 1ull) * sizeof(uint64_t)));
  if (c->mtHasRmOrder) FMT_HIP(c, cp(c->mtRmOffs.p, c->mtRmOffsHost.data(), (n + 1ull) * sizeof(uint64_t)));
  if (b->props_off) {
    FMT_HIP(c, cp(c->mtPropsOff.p, b->props_off, (b->n_props_ops + 1ull) * sizeof(uint32_t)));
    FMT_HIP(c, cp(c->mtPropsKv.p, b->props_kv, nKv * sizeof(uint32_t)));
  } else {
    FMT_HIP(c, hipMemsetAsync(c->mtPropsOff.p, 0, sizeof(uint32_t), c->stream));
  }
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  c->mtNOps = b->n_ops;
  c->mtDocs = n;
  c->mtTextLen = b->text_len;
  c->mtNPropsOps = b->n_props_ops;
  c->mtOffsHost.assign(b->doc_op_offsets, b->doc_op_offsets + n + 1);
  if (b->snapshots) c->mtSnapHost.assign(b->snapshots, b->snapshots + n);
  else c->mtSnapHost.clear();
  c->mtNProps = b->n_props_ops;
  c->mtHasInit = b->doc_init != nullptr;
  c->mtObliterate = obliterates;
  // A batch without remove-order recording starts in the compact tier; a document about to outgrow
  // it stops at a checkpoint (≈17 KiB per document) that the small tier resumes from.
  c->mtCkptOk = false;
  if (!c->mtHasRmOrder) {
    // (a batch too large for the checkpoints still replays: overflowing documents then restart in
    // the next tier from their first op, as batches with obliterates do)
    c->mtCkptOk = c->mtCkpt.reserve(static_cast<size_t>(n) * (fmt_kernels::mergeTreeCheckpointBytes() / sizeof(uint32_t))) ==
                  hipSuccess;
    if (!c->mtCkptOk) (void)hipGetLastError();
  }
  c->mtInsertChars = insertChars;
  c->mtInitChars = initChars;
  // Huge documents: a summary-loaded document with more segments or text than the large tier holds
  // is replayed by the huge-document engine (huge_engine.h: one wave, state in HBM). It loads from
  // one header chunk; catch-up / remove-order recording stays with the other tiers.
  for (auto& h : c->huge)
    for (void* p : h.allocs) (void)hipFree(p);
  c->huge.clear();
  c->mtHugeSlot.assign(n, -1);
  c->mtHugeOk.assign(n, 1);
  c->mtLoadSegs.assign(n, 0);
  c->mtSegProps.assign(n, 0);
  c->mtDocChars.assign(n, 0);
  c->mtStartSeg.assign(n, fmt_mt_snapshot_seg{0, 0, FMT_MT_NO_PROPS});
  parallelChunks(n, [&](uint64_t d0, uint64_t d1, unsigned) {
  for (uint64_t d = d0; d < d1; d++) {
    uint8_t ok = 1;  // (the huge tier replays every feature a document of the other tiers may hold)
    uint64_t chars = 0;
    uint32_t loadSegs = 0;
    for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++) {
      const fmt_mt_op& op = b->ops[i];
      if (op.type == FMT_MT_INSERT) chars += fmt_mt_op_len(&op);
      if (op.flags & FMT_MT_F_LOADSEG) loadSegs++;
    }
    c->mtLoadSegs[d] = loadSegs;
    if (b->snapshots && b->snapshots[d].loaded) {
      const fmt_mt_snapshot_doc& sd = b->snapshots[d];
      for (uint64_t k = sd.first_seg; k < sd.first_seg + sd.n_header + sd.n_body; k++)
        if (b->snapshot_segs[k].props != FMT_MT_NO_PROPS) {
          c->mtSegProps[d] = 1;
          break;
        }
      for (uint64_t k = sd.first_seg; k < sd.first_seg + sd.n_header + sd.n_body; k++)
        chars += b->snapshot_segs[k].len & ~FMT_MT_SEG_MARKER;
    } else if (b->doc_init && b->doc_init[2 * d + 1] > 0) {
      c->mtStartSeg[d] = fmt_mt_snapshot_seg{b->doc_init[2 * d], b->doc_init[2 * d + 1], FMT_MT_NO_PROPS};
      chars += b->doc_init[2 * d + 1];
    }
    c->mtHugeOk[d] = ok;
    c->mtDocChars[d] = chars;
  }
  });
  // Summary-loaded documents past the large tier go to the huge tier; one that holds a feature the
  // huge tier lacks, or whose state does not fit in device memory, fails alone at load (its header
  // says why) and the rest of the batch replays.
  c->mtRefused.clear();
  std::vector<fmt_mt_doc_result> refusedHdr;
  auto refuse = [&](uint32_t d, int status) {
    fmt_mt_doc_result h{};
    h.status = status;
    h.fail_seq = b->snapshots[d].seq;
    h.cur_seq = b->snapshots[d].seq;
    h.min_seq = b->snapshots[d].min_seq;
    c->mtRefused.push_back(d);
    refusedHdr.push_back(h);
  };
  if (b->snapshots) {
    const fmt_kernels::MtCaps big = fmt_kernels::mergeTreeCaps(true);
    for (uint32_t d = 0; d < n; d++) {
      const fmt_mt_snapshot_doc& sd = b->snapshots[d];
      if (!sd.loaded) continue;
      uint64_t chars = 0;
      for (uint64_t k = sd.first_seg; k < sd.first_seg + sd.n_header + sd.n_body; k++)
        chars += b->snapshot_segs[k].len & ~FMT_MT_SEG_MARKER;
      // (a V1 summary with merge info brings its body as loader-segment ops: they count as loaded)
      const uint64_t loaded = sd.n_header + sd.n_body + c->mtLoadSegs[d];
      if (c->mtLoadSegs[d] > 0) chars = c->mtDocChars[d];
      if (loaded <= big.leaves && chars <= big.chars) continue;
      if (!c->mtHugeOk[d] || local) {  // (local-client records)
        refuse(d, FMT_E_UNSUPPORTED);
        continue;
      }
      const int rc = setupHugeDoc(c, b->text_len, b->n_props_ops, d, b->doc_op_offsets[d], b->doc_op_offsets[d + 1],
                                  c->mtSnapSegs.p + sd.first_seg, sd.n_header, sd.n_body, sd.min_seq, sd.seq,
                                  FMT_NON_COLLAB_CLIENT, 256,
                                  c->mtDocChars[d]);
      if (rc == FMT_E_CAPACITY) refuse(d, FMT_E_CAPACITY);
      else if (rc != FMT_OK) return rc;
    }
  }
  for (size_t i = 0; i < c->mtRefused.size(); i++)
    FMT_HIP(c, hipMemcpyAsync(c->mtHdr.p + c->mtRefused[i], &refusedHdr[i], sizeof(fmt_mt_doc_result), hipMemcpyHostToDevice,
                              c->stream));
  c->mtHugeLoaded = static_cast<uint32_t>(c->huge.size());
  c->mtUseList = !c->huge.empty() || !c->mtRefused.empty();
  if (c->mtUseList) {
    std::vector<uint8_t> skip(n, 0);
    for (uint32_t d : c->mtRefused) skip[d] = 1;
    std::vector<uint32_t> small;
    for (uint32_t d = 0; d < n; d++)
      if (c->mtHugeSlot[d] < 0 && !skip[d]) small.push_back(d);
    c->mtNSmall = static_cast<uint32_t>(small.size());
    FMT_HIP(c, c->mtSmallList.reserve(small.size()));
    FMT_HIP(c, cp(c->mtSmallList.p, small.data(), small.size() * sizeof(uint32_t)));
  }
  if (!c->huge.empty()) {
    const size_t nh = c->huge.size();
    FMT_HIP(c, c->hugeStates.reserve(nh));
    FMT_HIP(c, c->hugeInputs.reserve(nh));
    FMT_HIP(c, c->hugeOuts.reserve(nh));
    std::vector<fmt_huge::HugeState> hs(nh);
    std::vector<fmt_huge::HugeInputs> hi(nh);
    std::vector<fmt_kernels::HugeOut> ho(nh);
    for (size_t i = 0; i < nh; i++) {
      hs[i] = c->huge[i].state;
      hi[i] = c->huge[i].in;
      ho[i] = c->huge[i].out;
    }
    FMT_HIP(c, cp(c->hugeStates.p, hs.data(), nh * sizeof(fmt_huge::HugeState)));
    FMT_HIP(c, cp(c->hugeInputs.p, hi.data(), nh * sizeof(fmt_huge::HugeInputs)));
    FMT_HIP(c, cp(c->hugeOuts.p, ho.data(), nh * sizeof(fmt_kernels::HugeOut)));
  }
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  c->mtLoaded = true;
  return FMT_OK;
}

int fmt_mt_run(fmt_ctx* c) {
  if (c == nullptr || !c->mtLoaded) return setErr(c, FMT_E_USAGE, "fmt_mt_run before fmt_mt_load");
  FMT_HIP(c, hipSetDevice(c->device));
  // documents an earlier run of this load escalated into the huge tier start over: their state is
  // released, and only the load-time huge documents (c->mtHugeLoaded) run with the small tiers
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  for (size_t h = c->mtHugeLoaded; h < c->huge.size(); h++)
    for (void* q : c->huge[h].allocs) (void)hipFree(q);
  for (uint32_t d = 0; d < c->mtDocs; d++)
    if (c->mtHugeSlot[d] >= static_cast<int32_t>(c->mtHugeLoaded)) c->mtHugeSlot[d] = -1;
  c->huge.resize(c->mtHugeLoaded);
  fmt_kernels::MtDeviceBatch db{c->mtOps.p, c->mtOffs.p, c->mtDocs, c->mtText.p,
                                c->mtHasInit ? c->mtInit.p : nullptr, c->mtPropsOff.p, c->mtPropsKv.p, c->mtNProps,
                                c->mtHasCatchup ? c->mtCuOffs.p : nullptr,
                                c->mtHasSnap ? c->mtSnap.p : nullptr, c->mtHasSnap ? c->mtSnapSegs.p : nullptr,
                                c->mtHasRmOrder ? c->mtRmOffs.p : nullptr,
                                c->mtHasSnapInfo ? c->mtSnapInfo.p : nullptr, c->mtHasSnapInfo ? c->mtSnapStamps.p : nullptr,
                                c->mtHasSnapInfo ? c->mtNSnapSegs : 0u,
                                c->mtNRelpos ? c->mtRelpos.p : nullptr,
                                c->mtNRelpos, c->mtMarkerKey,
                                c->mtHasAdjust ? c->mtAdjTab.p : nullptr,
                                c->mtLocal ? c->mtLocTab.p : nullptr};
  fmt_kernels::MtDeviceOut dout{c->mtHdr.p, c->mtLeaves.p, c->mtChars.p, c->mtProps.p,
                                c->mtHasCatchup ? c->mtCatchup.p : nullptr, c->mtHasRmOrder ? c->mtRmOrder.p : nullptr,
                                !c->mtHasRmOrder && !c->mtHasAdjust && c->mtCkptOk ? c->mtCkpt.p : nullptr, nullptr, nullptr,
                                c->mtHasAdjust ? c->mtLegacy.p : nullptr};
  FMT_HIP(c, hipMemsetAsync(c->mtEsc.p, 0, sizeof(uint32_t), c->stream));
  FMT_HIP(c, hipMemsetAsync(c->mtEsc2.p, 0, sizeof(uint32_t), c->stream));
  FMT_HIP(c, hipMemsetAsync(c->mtSched.p, 0, 4 * sizeof(uint32_t), c->stream));
  FMT_HIP(c, hipEventRecord(c->ev0, c->stream));
  const bool hasHuge = c->mtHugeLoaded > 0, list = c->mtUseList;
  if (c->mtLocal) {
    // f4 (round 6): the small tier's local variant over every document (its Adj variant for
    // annotate-adjust batches); those listed in mtEsc replay from their first op in the large tier's
    // local variant below (mergetree_local.hip)
    if (!list || c->mtNSmall > 0)
      FMT_HIP(c, fmt_kernels::launchMergeTreeLocal(db, dout, list ? c->mtSmallList.p : nullptr, list ? c->mtNSmall : c->mtDocs,
                                                   c->mtEsc.p, c->mtEsc2.p, c->numCUs, c->stream, c->mtSched.p,
                                                   c->mtHasAdjust));
  } else if (!list || c->mtNSmall > 0)
    FMT_HIP(c, fmt_kernels::launchMergeTree(db, dout, list ? c->mtSmallList.p : nullptr, list ? c->mtNSmall : c->mtDocs,
                                            c->mtEsc.p, c->mtEsc2.p, c->mtEsc3.p, c->numCUs, c->stream,
                                            c->mtObliterate,
                                            c->mtHasRmOrder, c->mtSched.p, c->mtHasAdjust));
  if (hasHuge)
    FMT_HIP(c, fmt_kernels::launchHugeDocs(c->hugeStates.p, c->hugeInputs.p, c->hugeOuts.p, c->mtHugeLoaded, c->mtHasAdjust, c->mtHasRmOrder, c->stream));
  FMT_HIP(c, hipEventRecord(c->ev1, c->stream));  // device time excludes the host read-back below
  c->timed2 = false;
  // Documents that overflowed the small tier replay again, from their inputs, in the large tier.
  uint32_t nEsc = 0;
  c->mtGrown = 0;
  FMT_HIP(c, hipMemcpyAsync(&nEsc, c->mtEsc.p, sizeof nEsc, hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  c->mtBigSlot.assign(c->mtDocs, -1);
  if (nEsc > 0) {
    const fmt_kernels::MtCaps big = fmt_kernels::mergeTreeCaps(true);
    FMT_HIP(c, c->mtBigLeaves.reserve(static_cast<size_t>(nEsc) * big.leaves));
    FMT_HIP(c, c->mtBigChars.reserve(static_cast<size_t>(nEsc) * big.chars));
    FMT_HIP(c, c->mtBigProps.reserve(static_cast<size_t>(nEsc) * big.props));
    if (c->mtHasAdjust) FMT_HIP(c, c->mtBigLegacy.reserve(static_cast<size_t>(nEsc) * big.leaves));
    // every batch but a local one: a document the large tier is about to outgrow leaves a checkpoint
    // for the huge tier (huge_ckpt.h) instead of failing; without the slab it restarts there from its
    // first op
    const bool hugeCk = !c->mtLocal &&
                        c->mtHugeCk.reserve(static_cast<size_t>(nEsc) * fmt_ckpt::kWords) == hipSuccess;
    if (!hugeCk) (void)hipGetLastError();
    fmt_kernels::MtDeviceOut bout{c->mtHdr.p, c->mtBigLeaves.p, c->mtBigChars.p, c->mtBigProps.p,
                                  c->mtHasCatchup ? c->mtCatchup.p : nullptr, c->mtHasRmOrder ? c->mtRmOrder.p : nullptr,
                                  c->mtObliterate && !c->mtHasRmOrder && !c->mtHasAdjust && c->mtCkptOk ? c->mtCkpt.p : nullptr,
                                  !c->mtHasRmOrder ? c->mtLeaves.p : nullptr, !c->mtHasRmOrder ? c->mtChars.p : nullptr,
                                  c->mtHasAdjust ? c->mtBigLegacy.p : nullptr, hugeCk ? c->mtHugeCk.p : nullptr};
    FMT_HIP(c, hipEventRecord(c->ev2, c->stream));
    FMT_HIP(c, fmt_kernels::launchMergeTreeLarge(db, bout, c->mtEsc.p + 1, nEsc, c->numCUs, c->stream, c->mtObliterate,
                                                 c->mtHasRmOrder, c->mtSched.p + 2, c->mtHasAdjust, c->mtLocal));
    FMT_HIP(c, hipEventRecord(c->ev3, c->stream));
    c->timed2 = true;
    std::vector<uint32_t> list(nEsc);
    FMT_HIP(c, hipMemcpyAsync(list.data(), c->mtEsc.p + 1, nEsc * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    FMT_HIP(c, hipStreamSynchronize(c->stream));
    for (uint32_t i = 0; i < nEsc; i++) c->mtBigSlot[list[i]] = static_cast<int32_t>(i);
    // Documents the large tier could not hold (FMT_E_CAPACITY: leaves, text, blocks, prop sets)
    // replay again from their start in the huge tier, which has no such limit but device memory —
    // the reference grows a tree without bound (insertSegments, mergeTree.ts:1484-1517).
    std::vector<fmt_mt_doc_result> hb(nEsc);
    std::vector<uint32_t> grow;
    std::vector<int32_t> growSlot;  // the large-tier slot of a checkpointed document (-1: restart from op 0)
    for (uint32_t i = 0; i < nEsc; i++) {
      FMT_HIP(c, hipMemcpyAsync(&hb[i], c->mtHdr.p + list[i], sizeof(fmt_mt_doc_result), hipMemcpyDeviceToHost, c->stream));
    }
    FMT_HIP(c, hipStreamSynchronize(c->stream));
    for (uint32_t i = 0; i < nEsc; i++) {
      if ((hb[i].status == FMT_E_CAPACITY || hb[i].status == fmt_ckpt::kStatusHuge) && c->mtHugeOk[list[i]] &&
          c->mtHugeSlot[list[i]] < 0 && !c->mtLocal) {
        grow.push_back(list[i]);
        growSlot.push_back(hb[i].status == fmt_ckpt::kStatusHuge ? static_cast<int32_t>(i) : -1);
      }
    }
    if (!grow.empty()) {
      FMT_HIP(c, c->mtStartSegDev.reserve(grow.size()));
      std::vector<fmt_mt_snapshot_seg> starts(grow.size());
      for (size_t i = 0; i < grow.size(); i++) starts[i] = c->mtStartSeg[grow[i]];
      FMT_HIP(c, hipMemcpyAsync(c->mtStartSegDev.p, starts.data(), grow.size() * sizeof(fmt_mt_snapshot_seg),
                                hipMemcpyHostToDevice, c->stream));
      // (a document whose huge-tier state does not fit in device memory keeps the large tier's
      // FMT_E_CAPACITY header)
      for (size_t i = 0; i < grow.size(); i++) {
        const uint32_t d = grow[i];
        const uint64_t o0 = c->mtOffsHost[d], o1 = c->mtOffsHost[d + 1];
        int rc;
        if (c->mtSnapHost.size() > d && c->mtSnapHost[d].loaded) {
          const fmt_mt_snapshot_doc& sd = c->mtSnapHost[d];
          rc = setupHugeDoc(c, c->mtTextLen, c->mtNPropsOps, d, o0, o1, c->mtSnapSegs.p + sd.first_seg, sd.n_header,
                            sd.n_body, sd.min_seq, sd.seq, FMT_NON_COLLAB_CLIENT, 1024, c->mtDocChars[d]);
        } else {
          rc = setupHugeDoc(c, c->mtTextLen, c->mtNPropsOps, d, o0, o1, c->mtStartSegDev.p + i, starts[i].len > 0 ? 1 : 0,
                            0, 0, 0, FMT_LOCAL_CLIENT, 1024, c->mtDocChars[d]);
        }
        if (rc != FMT_OK && rc != FMT_E_CAPACITY) return rc;
        if (growSlot[i] >= 0) {
          if (rc == FMT_OK) {  // resume from the large tier's checkpoint and result slabs
            const size_t k = static_cast<size_t>(growSlot[i]);
            fmt_huge::HugeInputs& I = c->huge.back().in;
            I.ck = c->mtHugeCk.p + k * fmt_ckpt::kWords;
            I.ckLeaves = c->mtBigLeaves.p + k * big.leaves;
            I.ckChars = c->mtBigChars.p + k * big.chars;
            I.ckProps = c->mtBigProps.p + k * big.props;
          } else {  // (no room in device memory: the document reports FMT_E_CAPACITY)
            const int32_t st = FMT_E_CAPACITY;
            FMT_HIP(c, hipMemcpyAsync(&c->mtHdr.p[d].status, &st, sizeof st, hipMemcpyHostToDevice, c->stream));
            FMT_HIP(c, hipStreamSynchronize(c->stream));
          }
        }
      }
      const size_t ng = c->huge.size() - c->mtHugeLoaded;
      if (ng > 0) {
      FMT_HIP(c, c->hugeStates2.reserve(ng));
      FMT_HIP(c, c->hugeInputs2.reserve(ng));
      FMT_HIP(c, c->hugeOuts2.reserve(ng));
      std::vector<fmt_huge::HugeState> hs(ng);
      std::vector<fmt_huge::HugeInputs> hi(ng);
      std::vector<fmt_kernels::HugeOut> ho(ng);
      for (size_t i = 0; i < ng; i++) {
        const auto& H = c->huge[c->mtHugeLoaded + i];
        hs[i] = H.state;
        hi[i] = H.in;
        ho[i] = H.out;
      }
      FMT_HIP(c, hipMemcpyAsync(c->hugeStates2.p, hs.data(), ng * sizeof(fmt_huge::HugeState), hipMemcpyHostToDevice, c->stream));
      FMT_HIP(c, hipMemcpyAsync(c->hugeInputs2.p, hi.data(), ng * sizeof(fmt_huge::HugeInputs), hipMemcpyHostToDevice, c->stream));
      FMT_HIP(c, hipMemcpyAsync(c->hugeOuts2.p, ho.data(), ng * sizeof(fmt_kernels::HugeOut), hipMemcpyHostToDevice, c->stream));
      FMT_HIP(c, fmt_kernels::launchHugeDocs(c->hugeStates2.p, c->hugeInputs2.p, c->hugeOuts2.p, static_cast<uint32_t>(ng),
                                             c->mtHasAdjust, c->mtHasRmOrder, c->stream));
      FMT_HIP(c, hipStreamSynchronize(c->stream));
      }
      c->mtGrown = static_cast<uint32_t>(ng);
    }
  }
  c->timed = true;
  c->stats = fmt_stats{};
  c->stats.ops = c->mtNOps;
  c->stats.docs = c->mtDocs;
  // Algorithmic bytes: every op record and every inserted UTF-16 unit read once; results written
  // (headers + leaves + chars + prop sets) are added by fmt_mt_fetch_headers once sizes are known.
  c->stats.bytes_read = c->mtNOps * sizeof(fmt_mt_op) + (c->mtInsertChars + c->mtInitChars) * 2 +
                        (c->mtDocs + 1ull) * sizeof(uint64_t);
  c->stats.bytes_written = static_cast<uint64_t>(c->mtDocs) * sizeof(fmt_mt_doc_result);
  // compact + small tier (no remove-order recording) or small tier alone, then the large tier when it ran
  // (+1: the huge-tier pass over documents that outgrew the large tier, after the timed events)
  c->stats.launches = (!c->mtHasRmOrder ? 2 : 1) + (nEsc > 0 ? 1 : 0) + (c->mtGrown > 0 ? 1 : 0);
  return FMT_OK;
}

int fmt_mt_fetch_headers(fmt_ctx* c, fmt_mt_doc_result* out) {
  if (c == nullptr || out == nullptr || !c->mtLoaded) return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_headers: nothing loaded");
  FMT_HIP(c, hipMemcpyAsync(out, c->mtHdr.p, c->mtDocs * sizeof(fmt_mt_doc_result), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  uint64_t w = static_cast<uint64_t>(c->mtDocs) * sizeof(fmt_mt_doc_result);
  int status = FMT_OK;
  for (uint32_t d = 0; d < c->mtDocs; d++) {
    w += out[d].n_leaves * sizeof(fmt_mt_leaf) + out[d].n_chars * 2ull + out[d].n_props * sizeof(fmt_mt_propset);
    if (out[d].status != FMT_OK && status == FMT_OK) {
      status = out[d].status;
      char m[160];
      std::snprintf(m, sizeof m, "doc %u failed with status %d at seq %d", d, out[d].status, out[d].fail_seq);
      c->err = m;
    }
  }
  c->stats.bytes_written = w;
  return status;
}

int fmt_mt_fetch_doc(fmt_ctx* c, uint32_t doc, fmt_mt_leaf* leaves, uint32_t capLeaves, uint16_t* chars,
                     uint32_t capChars, fmt_mt_propset* props, uint32_t capProps) {
  if (c == nullptr || !c->mtLoaded || doc >= c->mtDocs) return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_doc: bad doc");
  const int32_t hslot = doc < c->mtHugeSlot.size() ? c->mtHugeSlot[doc] : -1;
  if (hslot >= 0) {  // a huge document: its own output buffers
    const fmt_kernels::HugeOut& O = c->huge[static_cast<size_t>(hslot)].out;
    fmt_mt_doc_result h;
    FMT_HIP(c, hipMemcpy(&h, c->mtHdr.p + doc, sizeof h, hipMemcpyDeviceToHost));
    const uint32_t nl = h.n_leaves < capLeaves ? h.n_leaves : capLeaves;
    const uint32_t nc = h.n_chars < capChars ? h.n_chars : capChars;
    const uint32_t np = h.n_props < capProps ? h.n_props : capProps;
    if (leaves && nl) FMT_HIP(c, hipMemcpy(leaves, O.leaves, nl * sizeof(fmt_mt_leaf), hipMemcpyDeviceToHost));
    if (chars && nc) FMT_HIP(c, hipMemcpy(chars, O.chars, nc * 2ull, hipMemcpyDeviceToHost));
    if (props && np) FMT_HIP(c, hipMemcpy(props, O.props, np * sizeof(fmt_mt_propset), hipMemcpyDeviceToHost));
    return FMT_OK;
  }
  const int32_t slot = doc < c->mtBigSlot.size() ? c->mtBigSlot[doc] : -1;
  const fmt_kernels::MtCaps caps = fmt_kernels::mergeTreeCaps(slot >= 0);
  const size_t at = slot >= 0 ? static_cast<size_t>(slot) : doc;
  const fmt_mt_leaf* dLeaves = slot >= 0 ? c->mtBigLeaves.p : c->mtLeaves.p;
  const uint16_t* dChars = slot >= 0 ? c->mtBigChars.p : c->mtChars.p;
  const fmt_mt_propset* dProps = slot >= 0 ? c->mtBigProps.p : c->mtProps.p;
  fmt_mt_doc_result h;
  FMT_HIP(c, hipMemcpy(&h, c->mtHdr.p + doc, sizeof h, hipMemcpyDeviceToHost));
  const uint32_t nl = h.n_leaves < capLeaves ? h.n_leaves : capLeaves;
  const uint32_t nc = h.n_chars < capChars ? h.n_chars : capChars;
  const uint32_t np = h.n_props < capProps ? h.n_props : capProps;
  if (leaves && nl) FMT_HIP(c, hipMemcpy(leaves, dLeaves + at * caps.leaves, nl * sizeof(fmt_mt_leaf), hipMemcpyDeviceToHost));
  if (chars && nc) FMT_HIP(c, hipMemcpy(chars, dChars + at * caps.chars, nc * 2ull, hipMemcpyDeviceToHost));
  if (props && np) FMT_HIP(c, hipMemcpy(props, dProps + at * caps.props, np * sizeof(fmt_mt_propset), hipMemcpyDeviceToHost));
  return FMT_OK;
}

// ------------------------------------------------------------------ bulk legacy summaries
namespace {

// JSON.stringify of a UTF-16 string (well-formed: lone surrogates as \udXXX), as UTF-8.
void jsonQuote16(std::string& o, const uint16_t* s, size_t n) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  for (size_t i = 0; i < n; i++) {
    const uint32_t c = s[i];
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c == '\b') o += "\\b";
    else if (c == '\f') o += "\\f";
    else if (c == '\n') o += "\\n";
    else if (c == '\r') o += "\\r";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20) {
      o += "\\u00";
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    } else if (c < 0x80) {
      o.push_back(static_cast<char>(c));
    } else if (c < 0x800) {
      o.push_back(static_cast<char>(0xC0 | (c >> 6)));
      o.push_back(static_cast<char>(0x80 | (c & 0x3F)));
    } else if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
      const uint32_t cp = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
      i++;
      o.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      o.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (c >= 0xD800 && c <= 0xDFFF) {
      o += "\\u";
      for (int k = 12; k >= 0; k -= 4) o.push_back(hex[(c >> k) & 15]);
    } else {
      o.push_back(static_cast<char>(0xE0 | (c >> 12)));
      o.push_back(static_cast<char>(0x80 | ((c >> 6) & 0x3F)));
      o.push_back(static_cast<char>(0x80 | (c & 0x3F)));
    }
  }
  o.push_back('"');
}

// A quoted key "digits" that is a canonical array index (< 2^32 - 1): its value, else -1.
int64_t arrayIndexOfQuoted(const std::string& q) {
  if (q.size() < 3 || q.size() > 12 || q.front() != '"' || q.back() != '"') return -1;
  const size_t n = q.size() - 2;
  if (n > 1 && q[1] == '0') return -1;
  int64_t v = 0;
  for (size_t i = 1; i + 1 < q.size(); i++) {
    if (q[i] < '0' || q[i] > '9') return -1;
    v = v * 10 + (q[i] - '0');
  }
  return v < 4294967295LL ? v : -1;
}

struct SumDict {
  std::vector<std::string> keys, values;  // keys JSON-quoted, values JSON texts (UTF-8)
  std::vector<int64_t> keyIndex;          // array-index value of each key, or -1
};

// A prop set as a JSON object in JS own-property order: array-index keys ascending, then the
// others in insertion order (properties' key order, snapshotChunks.ts via JSON.stringify).
// (ps: the set's first record; a set wider than FMT_MT_PROPS_MAX continues in the next records)
void propsObject(std::string& o, const fmt_mt_propset* ps, const SumDict& D, const std::vector<double>* nums,
                 uint32_t valueBase) {
  const uint32_t n = ps->n < FMT_MT_PROPS_KEYS_MAX ? ps->n : FMT_MT_PROPS_KEYS_MAX;
  uint32_t kvs[FMT_MT_PROPS_KEYS_MAX], order[FMT_MT_PROPS_KEYS_MAX];
  for (uint32_t i = 0; i < n; i++) kvs[i] = ps[i / FMT_MT_PROPS_MAX].kv[i % FMT_MT_PROPS_MAX];
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; i++)
    if (D.keyIndex[kvs[i] >> 16] >= 0) order[m++] = i;
  std::sort(order, order + m, [&](uint32_t a, uint32_t b) { return D.keyIndex[kvs[a] >> 16] < D.keyIndex[kvs[b] >> 16]; });
  for (uint32_t i = 0; i < n; i++)
    if (D.keyIndex[kvs[i] >> 16] < 0) order[m++] = i;
  o.push_back('{');
  for (uint32_t j = 0; j < m; j++) {
    if (j) o.push_back(',');
    const uint32_t kv = kvs[order[j]];
    o += D.keys[kv >> 16];
    o.push_back(':');
    const uint32_t v = kv & 0xFFFFu;
    if (nums != nullptr && v >= FMT_MT_VALUE_COMPUTED)  // an annotate-adjust result
      o += fmt_json::jsNumber((*nums)[v - FMT_MT_VALUE_COMPUTED]);
    else
      o += D.values[valueBase + v];
  }
  o.push_back('}');
}

// SnapshotLegacy.emit for one document (snapshotlegacy.ts:161-190 + snapshotChunks.ts:85-204):
// the header chunk (runs until >= chunk units) and, when runs remain, the body chunk.
void legacyBlobs(std::string& out, uint32_t* split, const fmt_kernels::SumRun* runs, uint32_t nRuns,
                 const uint16_t* text, const fmt_mt_propset* props, int32_t minSeq, uint32_t chunk,
                 const SumDict& D, const std::vector<double>* nums, uint32_t valueBase) {
  uint64_t total = 0;
  for (uint32_t i = 0; i < nRuns; i++) total += runs[i].len;
  std::vector<uint64_t> start(nRuns + 1, 0);
  for (uint32_t i = 0; i < nRuns; i++) start[i + 1] = start[i] + runs[i].len;
  auto emit = [&](uint32_t s0, uint64_t approx, bool header, uint32_t* count) {
    uint32_t n = 0;
    uint64_t len = 0;
    while (len < approx && s0 + n < nRuns) len += runs[s0 + n++].len;
    out += "{\"chunkStartSegmentIndex\":" + std::to_string(s0) + ",\"chunkSegmentCount\":" + std::to_string(n) +
           ",\"chunkLengthChars\":" + std::to_string(len) + ",\"totalLengthChars\":" + std::to_string(total) +
           ",\"totalSegmentCount\":" + std::to_string(nRuns) + ",\"chunkSequenceNumber\":" + std::to_string(minSeq) +
           ",\"segmentTexts\":[";
    for (uint32_t i = s0; i < s0 + n; i++) {
      if (i > s0) out.push_back(',');
      const fmt_kernels::SumRun& r = runs[i];
      const bool hasProps = r.props != 0xFFFFu && props[r.props].n > 0;
      if (r.flags & 1u) {  // Marker.toJSONObject
        out += "{\"marker\":{\"refType\":" + std::to_string(text[start[i]]) + "}";
        if (hasProps) {
          out += ",\"props\":";
          propsObject(out, props + r.props, D, nums, valueBase);
        }
        out.push_back('}');
      } else if (hasProps) {
        out += "{\"text\":";
        jsonQuote16(out, text + start[i], r.len);
        out += ",\"props\":";
        propsObject(out, props + r.props, D, nums, valueBase);
        out.push_back('}');
      } else {
        jsonQuote16(out, text + start[i], r.len);
      }
    }
    out.push_back(']');
    if (header) {
      out += ",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}";
      if (len < total) out += ",{\"id\":\"body\"}";
      out += "],\"sequenceNumber\":" + std::to_string(minSeq) + ",\"totalLength\":" + std::to_string(total) +
             ",\"totalSegmentCount\":" + std::to_string(nRuns) + "}";
    }
    out.push_back('}');
    *count = n;
  };
  uint32_t n1 = 0, n2 = 0;
  emit(0, chunk, true, &n1);
  *split = static_cast<uint32_t>(out.size());
  if (n1 < nRuns) emit(n1, total, false, &n2);
}

// Where each document's converged state lives: the small tier's slabs, a large-tier slab, or a
// huge document's own buffers.
void docViews(const fmt_ctx* c, std::vector<fmt_kernels::SumView>& views) {
  const uint32_t nd = c->mtDocs;
  views.resize(nd);
  for (uint32_t d = 0; d < nd; d++) {
    const int32_t hs = d < c->mtHugeSlot.size() ? c->mtHugeSlot[d] : -1;
    if (hs >= 0) {
      const fmt_kernels::HugeOut& O = c->huge[static_cast<size_t>(hs)].out;
      views[d] = {O.leaves, O.chars, O.props, c->mtHasAdjust ? O.legacy : nullptr, O.cls, O.leavesHi};
    } else {
      const int32_t slot = d < c->mtBigSlot.size() ? c->mtBigSlot[d] : -1;
      const fmt_kernels::MtCaps caps = fmt_kernels::mergeTreeCaps(slot >= 0);
      const size_t at = slot >= 0 ? static_cast<size_t>(slot) : d;
      views[d] = {(slot >= 0 ? c->mtBigLeaves.p : c->mtLeaves.p) + at * caps.leaves,
                  (slot >= 0 ? c->mtBigChars.p : c->mtChars.p) + at * caps.chars,
                  (slot >= 0 ? c->mtBigProps.p : c->mtProps.p) + at * caps.props,
                  c->mtHasAdjust ? (slot >= 0 ? c->mtBigLegacy.p : c->mtLegacy.p) + at * caps.leaves : nullptr};
    }
  }
}

}  // namespace

int fmt_mt_state_digest(fmt_ctx* c, uint64_t* out) {
  if (c == nullptr || out == nullptr || !c->mtLoaded) return setErr(c, FMT_E_USAGE, "fmt_mt_state_digest: nothing loaded");
  FMT_HIP(c, hipSetDevice(c->device));
  const uint32_t nd = c->mtDocs;
  std::vector<fmt_kernels::SumView> views;
  docViews(c, views);
  FMT_HIP(c, c->sumViews.reserve(nd));
  FMT_HIP(c, c->digests.reserve(nd));
  FMT_HIP(c, hipMemcpyAsync(c->sumViews.p, views.data(), nd * sizeof(fmt_kernels::SumView), hipMemcpyHostToDevice, c->stream));
  FMT_HIP(c, fmt_kernels::launchStateDigest(c->mtHdr.p, c->sumViews.p, nd, c->digests.p, c->numCUs, c->stream));
  FMT_HIP(c, hipMemcpyAsync(out, c->digests.p, nd * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  return FMT_OK;
}

int fmt_mt_summarize_legacy(fmt_ctx* c, const char* const* keys, uint32_t nKeys, const char* const* values,
                            uint32_t nValues, uint32_t chunk, uint32_t threads, fmt_summary_timing* timing) {
  if (c == nullptr || !c->mtLoaded || (nKeys && keys == nullptr) || (nValues && values == nullptr))
    return setErr(c, FMT_E_USAGE, "fmt_mt_summarize_legacy: bad arguments");
  using clk = std::chrono::steady_clock;
  FMT_HIP(c, hipSetDevice(c->device));
  const uint32_t nd = c->mtDocs;
  std::vector<fmt_mt_doc_result> hdr(nd);
  FMT_HIP(c, hipMemcpyAsync(hdr.data(), c->mtHdr.p, nd * sizeof(fmt_mt_doc_result), hipMemcpyDeviceToHost, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  // every document's result buffers (small tier, large-tier slab, or huge tier)
  std::vector<fmt_kernels::SumView> views;
  docViews(c, views);
  std::vector<fmt_mt_propset*> propsDev(nd);
  uint64_t capRuns = 0, capText = 0;
  for (uint32_t d = 0; d < nd; d++) {
    propsDev[d] = const_cast<fmt_mt_propset*>(views[d].props);
    capRuns += hdr[d].n_leaves;
    capText += hdr[d].n_chars;
  }
  FMT_HIP(c, c->sumViews.reserve(nd));
  FMT_HIP(c, c->sumRuns.reserve(capRuns));
  FMT_HIP(c, c->sumText.reserve(capText));
  FMT_HIP(c, c->sumCursors.reserve(2));
  FMT_HIP(c, c->sumDocs.reserve(nd));
  FMT_HIP(c, hipMemcpyAsync(c->sumViews.p, views.data(), nd * sizeof(fmt_kernels::SumView), hipMemcpyHostToDevice, c->stream));
  FMT_HIP(c, hipMemsetAsync(c->sumCursors.p, 0, 2 * sizeof(unsigned long long), c->stream));
  FMT_HIP(c, hipEventRecord(c->evS0, c->stream));  // (own events: fmt_get_stats keeps reporting the replay)
  FMT_HIP(c, fmt_kernels::launchSummaryRuns(c->mtHdr.p, c->sumViews.p, nd, c->sumRuns.p, c->sumText.p, c->sumCursors.p,
                                            c->sumDocs.p, c->numCUs, c->stream));
  FMT_HIP(c, hipEventRecord(c->evS1, c->stream));
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  float kms = 0.f;
  FMT_HIP(c, hipEventElapsedTime(&kms, c->evS0, c->evS1));
  // fetch: per-document spans, runs, text and every document's prop sets (packed on the device:
  // only the sets a document has, not its tier's whole table), staged into host buffers the ctx keeps
  const auto t0 = clk::now();
  unsigned long long cur[2];
  FMT_HIP(c, hipMemcpy(cur, c->sumCursors.p, sizeof cur, hipMemcpyDeviceToHost));
  constexpr uint32_t kPW = sizeof(fmt_mt_propset) / 4;
  std::vector<uint64_t> propOff(nd + 1ull, 0);
  std::vector<fmt_kernels::GatherSpan> sp;
  for (uint32_t d = 0; d < nd; d++) {
    propOff[d + 1] = propOff[d] + hdr[d].n_props;
    if (hdr[d].n_props)
      sp.push_back({reinterpret_cast<const uint32_t*>(propsDev[d]), propOff[d] * kPW, hdr[d].n_props * kPW, 0u});
  }
  if (!sp.empty()) {
    FMT_HIP(c, c->spans.reserve(sp.size()));
    FMT_HIP(c, c->packed.reserve(propOff[nd] * kPW));
    FMT_HIP(c, hipMemcpyAsync(c->spans.p, sp.data(), sp.size() * sizeof(fmt_kernels::GatherSpan), hipMemcpyHostToDevice,
                              c->stream));
    FMT_HIP(c, fmt_kernels::launchGatherSpans(c->spans.p, static_cast<uint32_t>(sp.size()), c->packed.p, c->numCUs, c->stream));
  }
  // (pinned destinations the ctx keeps: four DMAs back to back on the stream, one wait)
  FMT_HIP(c, c->sumHostDocs.reserve(nd));
  FMT_HIP(c, c->sumHostRuns.reserve(cur[0]));
  FMT_HIP(c, c->sumHostText.reserve(cur[1]));
  FMT_HIP(c, c->sumHostProps.reserve(propOff[nd] + 1));
  FMT_HIP(c, hipMemcpyAsync(c->sumHostDocs.p, c->sumDocs.p, nd * sizeof(fmt_kernels::SumDocOut), hipMemcpyDeviceToHost, c->stream));
  if (cur[0])
    FMT_HIP(c, hipMemcpyAsync(c->sumHostRuns.p, c->sumRuns.p, cur[0] * sizeof(fmt_kernels::SumRun), hipMemcpyDeviceToHost, c->stream));
  if (cur[1])
    FMT_HIP(c, hipMemcpyAsync(c->sumHostText.p, c->sumText.p, cur[1] * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream));
  if (propOff[nd])
    FMT_HIP(c, hipMemcpyAsync(c->sumHostProps.p, c->packed.p, propOff[nd] * sizeof(fmt_mt_propset), hipMemcpyDeviceToHost,
                              c->stream));
  const fmt_kernels::SumDocOut* docs = c->sumHostDocs.p;
  const fmt_kernels::SumRun* runs = c->sumHostRuns.p;
  const uint16_t* text = c->sumHostText.p;
  std::vector<const fmt_mt_propset*> propsHost(nd);
  for (uint32_t d = 0; d < nd; d++) propsHost[d] = c->sumHostProps.p + propOff[d];
  // computed annotate-adjust numbers of the documents that have any
  std::vector<std::vector<double>> docNums(c->mtHasAdjust ? nd : 0);
  if (c->mtHasAdjust) {
    std::vector<uint32_t> cnt(nd);
    FMT_HIP(c, hipMemcpyAsync(cnt.data(), c->mtNumCount.p, nd * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    FMT_HIP(c, hipStreamSynchronize(c->stream));
    for (uint32_t d = 0; d < nd; d++) {
      docNums[d].resize(cnt[d]);
      if (cnt[d])
        FMT_HIP(c, hipMemcpyAsync(docNums[d].data(), c->mtNums.p + c->mtNumOffsHost[d], cnt[d] * sizeof(double),
                                  hipMemcpyDeviceToHost, c->stream));
    }
  }
  FMT_HIP(c, hipStreamSynchronize(c->stream));
  const auto t1 = clk::now();
  // format on host threads
  SumDict D;
  D.keys.assign(keys, keys + nKeys);
  D.values.assign(values, values + nValues);
  D.keyIndex.resize(nKeys);
  for (uint32_t k = 0; k < nKeys; k++) D.keyIndex[k] = arrayIndexOfQuoted(D.keys[k]);
  c->sumBlobs.assign(nd, std::string());
  c->sumSplit.assign(nd, 0);
  c->sumStatus.assign(nd, FMT_OK);
  const uint32_t nt = threads ? threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < nt; t++)
    pool.emplace_back([&, t] {
      for (uint32_t d = t; d < nd; d += nt) {
        const fmt_kernels::SumDocOut& o = docs[d];
        if (static_cast<int32_t>(o.status) != FMT_OK) {
          c->sumStatus[d] = static_cast<int32_t>(o.status);
          continue;
        }
        const std::vector<double>* nums = c->mtHasAdjust ? &docNums[d] : nullptr;
        // value id v names values[vBase + v] (document-local ids: v <= vCount)
        const uint32_t vBase = c->mtValueBaseHost.empty() ? 0u : c->mtValueBaseHost[d];
        const uint64_t vEnd = c->mtValueBaseHost.empty() ? nValues : std::min<uint64_t>(nValues, c->mtValueBaseHost[d + 1] + 1ull);
        // every prop set a run names, and every key / value id in it, within the tables passed in
        bool bad = false;
        for (uint32_t i = 0; i < o.n_runs && !bad; i++) {
          const uint32_t p = runs[o.run_off + i].props;
          if (p == 0xFFFFu) continue;
          const uint32_t pn = p < hdr[d].n_props ? propsHost[d][p].n : 0u;
          if (p >= hdr[d].n_props || pn > FMT_MT_PROPS_KEYS_MAX || (pn > 0 && p + (pn - 1) / FMT_MT_PROPS_MAX >= hdr[d].n_props)) {
            bad = true;
            break;
          }
          for (uint32_t k = 0; k < pn; k++) {
            const uint32_t kv = propsHost[d][p + k / FMT_MT_PROPS_MAX].kv[k % FMT_MT_PROPS_MAX];
            const uint32_t v = kv & 0xFFFFu;
            const bool computed = nums != nullptr && v >= FMT_MT_VALUE_COMPUTED && v - FMT_MT_VALUE_COMPUTED < nums->size();
            if ((kv >> 16) >= nKeys || (vBase + static_cast<uint64_t>(v) >= vEnd && !computed)) bad = true;
          }
        }
        if (bad) {
          c->sumStatus[d] = FMT_E_DATA;
          continue;
        }
        c->sumBlobs[d].reserve(o.n_units + 64ull * o.n_runs + 256);
        legacyBlobs(c->sumBlobs[d], &c->sumSplit[d], runs + o.run_off, o.n_runs, text + o.text_off,
                    propsHost[d], hdr[d].min_seq, chunk ? chunk : 10000u, D, nums, vBase);
      }
    });
  for (auto& th : pool) th.join();
  const auto t2 = clk::now();
  if (timing) {
    timing->kernel_ms = kms;
    timing->fetch_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    timing->format_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    uint64_t bytes = 0;
    for (const auto& b : c->sumBlobs) bytes += b.size();
    timing->bytes = bytes;
    timing->threads = nt;
  }
  return FMT_OK;
}

int fmt_mt_summary_blobs(fmt_ctx* c, uint32_t doc, const char** header, size_t* headerLen, const char** body,
                         size_t* bodyLen) {
  if (c == nullptr || doc >= c->sumBlobs.size()) return setErr(c, FMT_E_USAGE, "fmt_mt_summary_blobs: no summary for doc");
  if (c->sumStatus[doc] != FMT_OK) return setErr(c, c->sumStatus[doc], "document has no summary (replay status)");
  const std::string& b = c->sumBlobs[doc];
  const size_t split = c->sumSplit[doc];
  if (header) *header = b.data();
  if (headerLen) *headerLen = split;
  if (body) *body = b.data() + split;
  if (bodyLen) *bodyLen = b.size() - split;
  return FMT_OK;
}

int fmt_mt_fetch_catchup(fmt_ctx* c, uint32_t doc, fmt_mt_catchup_range* out, uint32_t cap) {
  if (c == nullptr || !c->mtLoaded || doc >= c->mtDocs || (out == nullptr && cap > 0))
    return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_catchup: bad arguments");
  if (!c->mtHasCatchup) return FMT_OK;
  fmt_mt_doc_result h;
  FMT_HIP(c, hipMemcpy(&h, c->mtHdr.p + doc, sizeof h, hipMemcpyDeviceToHost));
  const uint32_t m = h.n_catchup < cap ? h.n_catchup : cap;
  if (m) FMT_HIP(c, hipMemcpy(out, c->mtCatchup.p + c->mtCuOffsHost[doc], m * sizeof(fmt_mt_catchup_range), hipMemcpyDeviceToHost));
  return FMT_OK;
}

int fmt_mt_fetch_catchup_all(fmt_ctx* c, uint64_t* offsets, fmt_mt_catchup_range* out, uint64_t cap) {
  if (c == nullptr || !c->mtLoaded || offsets == nullptr)
    return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_catchup_all: bad arguments");
  FMT_HIP(c, hipSetDevice(c->device));
  const uint32_t nd = c->mtDocs;
  offsets[0] = 0;
  if (!c->mtHasCatchup) {
    for (uint32_t d = 0; d < nd; d++) offsets[d + 1] = 0;
    return FMT_OK;
  }
  std::vector<fmt_mt_doc_result> hdr(nd);
  FMT_HIP(c, hipMemcpy(hdr.data(), c->mtHdr.p, nd * sizeof(fmt_mt_doc_result), hipMemcpyDeviceToHost));
  for (uint32_t d = 0; d < nd; d++) {
    const uint64_t slab = c->mtCuOffsHost[d + 1] - c->mtCuOffsHost[d];
    offsets[d + 1] = offsets[d] + std::min<uint64_t>(hdr[d].n_catchup, slab);
  }
  if (out == nullptr) return FMT_OK;
  if (cap < offsets[nd]) return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_catchup_all: cap below the ranges recorded");
  // each document's recorded prefix packed on the device (gatherSpansKernel), then one staged copy of
  // exactly the recorded ranges
  constexpr uint32_t kW = sizeof(fmt_mt_catchup_range) / 4;
  std::vector<fmt_kernels::GatherSpan> sp;
  sp.reserve(nd);
  for (uint32_t d = 0; d < nd; d++)
    if (offsets[d + 1] > offsets[d])
      sp.push_back({reinterpret_cast<const uint32_t*>(c->mtCatchup.p + c->mtCuOffsHost[d]), offsets[d] * kW,
                    static_cast<uint32_t>(offsets[d + 1] - offsets[d]) * kW, 0u});
  if (offsets[nd] == 0) return FMT_OK;
  FMT_HIP(c, c->spans.reserve(sp.size()));
  FMT_HIP(c, c->packed.reserve(offsets[nd] * kW));
  FMT_HIP(c, hipMemcpyAsync(c->spans.p, sp.data(), sp.size() * sizeof(fmt_kernels::GatherSpan), hipMemcpyHostToDevice,
                            c->stream));
  FMT_HIP(c, fmt_kernels::launchGatherSpans(c->spans.p, static_cast<uint32_t>(sp.size()), c->packed.p, c->numCUs, c->stream));
  FMT_HIP(c, stagedCopy(c, out, c->packed.p, offsets[nd] * sizeof(fmt_mt_catchup_range), false));
  return FMT_OK;
}

int fmt_mt_fetch_remove_order(fmt_ctx* c, uint32_t doc, fmt_mt_remove_order* out, uint32_t cap) {
  if (c == nullptr || !c->mtLoaded || doc >= c->mtDocs || (out == nullptr && cap > 0))
    return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_remove_order: bad arguments");
  if (!c->mtHasRmOrder) return FMT_OK;
  fmt_mt_doc_result h;
  FMT_HIP(c, hipMemcpy(&h, c->mtHdr.p + doc, sizeof h, hipMemcpyDeviceToHost));
  const uint32_t m = h.n_rm_order < cap ? h.n_rm_order : cap;
  if (m) FMT_HIP(c, hipMemcpy(out, c->mtRmOrder.p + c->mtRmOffsHost[doc], m * sizeof(fmt_mt_remove_order), hipMemcpyDeviceToHost));
  return FMT_OK;
}

// word 0 of every leaf (ids 64..127), or words 1 and 2 (ids 128..191, 192..253) with `upper`
static int fetchRmClientsHi(fmt_ctx* c, uint32_t doc, uint64_t* out, uint32_t cap, bool upper, const char* what) {
  if (c == nullptr || !c->mtLoaded || doc >= c->mtDocs || (out == nullptr && cap > 0))
    return setErr(c, FMT_E_USAGE, std::string(what) + ": bad arguments");
  fmt_mt_doc_result h;
  FMT_HIP(c, hipMemcpy(&h, c->mtHdr.p + doc, sizeof h, hipMemcpyDeviceToHost));
  const uint32_t per = upper ? fmt_huge::kHiOutWords - 1 : 1;
  const uint32_t m = h.n_leaves < cap / per ? h.n_leaves : cap / per;
  const int32_t hs = doc < c->mtHugeSlot.size() ? c->mtHugeSlot[doc] : -1;
  const uint64_t* src = hs >= 0 ? c->huge[static_cast<size_t>(hs)].out.leavesHi : nullptr;
  if (src != nullptr && m) {
    std::vector<uint64_t> all(static_cast<size_t>(m) * fmt_huge::kHiOutWords);
    FMT_HIP(c, hipMemcpy(all.data(), src, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < m; i++)
      for (uint32_t k = 0; k < per; k++) out[static_cast<size_t>(i) * per + k] = all[static_cast<size_t>(i) * fmt_huge::kHiOutWords + (upper ? 1 + k : 0)];
  } else if (m) {
    std::memset(out, 0, static_cast<size_t>(m) * per * sizeof(uint64_t));  // (the other tiers hold ids 0..63 only)
  }
  return FMT_OK;
}

int fmt_mt_fetch_rm_clients_hi(fmt_ctx* c, uint32_t doc, uint64_t* out, uint32_t cap) {
  return fetchRmClientsHi(c, doc, out, cap, false, "fmt_mt_fetch_rm_clients_hi");
}

int fmt_mt_fetch_rm_clients_hi2(fmt_ctx* c, uint32_t doc, uint64_t* out, uint32_t cap) {
  return fetchRmClientsHi(c, doc, out, cap, true, "fmt_mt_fetch_rm_clients_hi2");
}

int fmt_mt_fetch_legacy_props(fmt_ctx* c, uint32_t doc, uint16_t* out, uint32_t cap) {
  if (c == nullptr || !c->mtLoaded || doc >= c->mtDocs || (out == nullptr && cap > 0))
    return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_legacy_props: bad arguments");
  fmt_mt_doc_result h;
  FMT_HIP(c, hipMemcpy(&h, c->mtHdr.p + doc, sizeof h, hipMemcpyDeviceToHost));
  const uint32_t m = h.n_leaves < cap ? h.n_leaves : cap;
  if (m == 0) return FMT_OK;
  std::vector<fmt_kernels::SumView> views;
  docViews(c, views);
  if (views[doc].legacyProps != nullptr) {
    FMT_HIP(c, hipMemcpy(out, views[doc].legacyProps, m * sizeof(uint16_t), hipMemcpyDeviceToHost));
    if (out[0] == fmt_mt::kLegacyUnavailable)  // (the engine marks every leaf)
      return setErr(c, FMT_E_CAPACITY, "fmt_mt_fetch_legacy_props: the document's getAtSeq view did not fit its prop-set table");
    return FMT_OK;
  }
  std::vector<fmt_mt_leaf> lv(m);  // (no annotate-adjust in the batch: getAtSeq is the current properties)
  FMT_HIP(c, hipMemcpy(lv.data(), views[doc].leaves, m * sizeof(fmt_mt_leaf), hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < m; i++) out[i] = lv[i].props;
  return FMT_OK;
}

int fmt_mt_fetch_numbers(fmt_ctx* c, uint32_t doc, double* out, uint32_t cap, uint32_t* nOut) {
  if (c == nullptr || !c->mtLoaded || doc >= c->mtDocs || (out == nullptr && cap > 0))
    return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_numbers: bad arguments");
  uint32_t n = 0;
  if (c->mtHasAdjust) FMT_HIP(c, hipMemcpy(&n, c->mtNumCount.p + doc, sizeof n, hipMemcpyDeviceToHost));
  if (nOut) *nOut = n;
  const uint32_t m = n < cap ? n : cap;
  if (m) FMT_HIP(c, hipMemcpy(out, c->mtNums.p + c->mtNumOffsHost[doc], m * sizeof(double), hipMemcpyDeviceToHost));
  return FMT_OK;
}

int fmt_mt_fetch_regen(fmt_ctx* c, uint32_t doc, fmt_mt_op* ops, uint32_t capOps, uint16_t* text, uint32_t capText,
                       uint32_t* nOps, uint32_t* nText) {
  if (c == nullptr || !c->mtLoaded || doc >= c->mtDocs || (ops == nullptr && capOps > 0) || (text == nullptr && capText > 0))
    return setErr(c, FMT_E_USAGE, "fmt_mt_fetch_regen: bad arguments");
  uint32_t cnt[2] = {0, 0};
  if (c->mtLocal) FMT_HIP(c, hipMemcpy(cnt, c->mtLocRegenCount.p + 2ull * doc, sizeof cnt, hipMemcpyDeviceToHost));
  if (nOps) *nOps = cnt[0];
  if (nText) *nText = cnt[1];
  const uint32_t m = cnt[0] < capOps ? cnt[0] : capOps, t = cnt[1] < capText ? cnt[1] : capText;
  if (m) FMT_HIP(c, hipMemcpy(ops, c->mtLocRegen.p + c->mtLocRegenOffsHost[doc], m * sizeof(fmt_mt_op), hipMemcpyDeviceToHost));
  if (t) FMT_HIP(c, hipMemcpy(text, c->mtLocRegenText.p + c->mtLocRegenTextOffsHost[doc], t * sizeof(uint16_t), hipMemcpyDeviceToHost));
  return FMT_OK;
}

// Internal diagnostic (not part of fmt.h): shader-clock totals per phase of a huge document's last
// replay (huge_engine.h HugeDoc::prof), HugeDoc::kProf values; FMT_E_USAGE if `doc` is not a huge document.
int fmt_internal_huge_profile(fmt_ctx* c, uint32_t doc, uint64_t* out) {
  if (c == nullptr || out == nullptr || doc >= c->mtHugeSlot.size() || c->mtHugeSlot[doc] < 0) return FMT_E_USAGE;
  FMT_HIP(c, hipMemcpy(out, c->huge[static_cast<size_t>(c->mtHugeSlot[doc])].out.prof, fmt_huge::HugeDoc::kProf * sizeof(uint64_t),
                       hipMemcpyDeviceToHost));
  return FMT_OK;
}

// Test hook (not part of fmt.h): the summary formatters' JSON.stringify of a number (jsnum.h).
int fmt_internal_js_number(double x, char* out, int cap) { return out == nullptr || cap < 0 ? 0 : fmt_json::jsNumber(x, out, cap); }

// Internal diagnostic (not part of fmt.h): per-phase cycle totals of a FMT_PROFILE=1 build.
int fmt_internal_mt_profile(uint64_t* out, int n, int reset) {
  return fmt_kernels::mergeTreeProfile(out, n, reset != 0);
}

}  // extern "C"
