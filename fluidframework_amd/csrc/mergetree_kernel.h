// mergetree_kernel.h — the merge-tree replay kernel template (mt_engine.h) and its launcher, shared
// by the per-tier translation units (mergetree.hip: small tier; mergetree_compact.hip: compact tier;
// mergetree_large.hip: large tier), which compile in parallel.
//
// One wavefront replays one document end to end; several documents share a workgroup, each with its
// own LDS state (fmt_mt::Scratch). Documents are independent, so the grid simply strides over them;
// there is no inter-workgroup communication. The per-document sequential dependency (every op
// depends on the state its predecessors left) is the reason this kernel is issue/latency-bound rather
// than HBM-bound: its compulsory HBM traffic is the 32-byte op record plus payload per op and the
// converged state written once per document.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "mt_engine.h"

namespace fmt_kernels {

// Diagnostic build only: per-phase shader-clock totals summed over all waves (mt_engine.h stamp()),
// one copy per translation unit (no relocatable device code); mergeTreeProfile sums them.
static __device__ unsigned long long g_mtProfile[fmt_mt::kPfCount];

// This translation unit's profile totals added into out[0..n) (and zeroed with reset).
static inline int addTuProfile(uint64_t* out, int n, bool reset) {
  unsigned long long h[fmt_mt::kPfCount];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_mtProfile), sizeof h) != hipSuccess) return -1;
  for (int c = 0; c < n && c < fmt_mt::kPfCount; c++) out[c] += h[c];
  if (reset) {
    unsigned long long z[fmt_mt::kPfCount] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_mtProfile), z, sizeof z) != hipSuccess) return -1;
  }
  return fmt_mt::kPfCount;
}

// Result slabs: the compact and small tiers share the small tier's per-document strides (a document
// the compact tier overflows replays again into the same slab); the large tier has its own.
template <class C>
struct Slab {
  static constexpr size_t kLeaves = C::kHbmChars ? 64 * C::kRows : 64 * fmt_mt::SmallTier::kRows;
  static constexpr size_t kChars = C::kHbmChars ? C::kCapChars : fmt_mt::SmallTier::kCapChars;
  static constexpr size_t kProps = C::kHbmChars ? C::kPropCap : fmt_mt::SmallTier::kPropCap;
};

// LDS bytes per wave: batches without obliterates never touch the live-obliterate table at the end
// of Scratch (1.6 KiB), which is what lets the compact tier hold 4 waves per SIMD (16 × 9312 B).
template <class C, bool Ob>
constexpr size_t scratchBytes() {
  return Ob ? sizeof(fmt_mt::Scratch<C>) : (offsetof(fmt_mt::Scratch<C>, ob) + 15) & ~static_cast<size_t>(15);
}

// A tier over all documents (docList == nullptr) or a list of countDev[0] (when countDev is set:
// the overflow list a previous launch built on the device) or `count` documents. The large tier
// writes leaves/chars/props to slab i of the list (headers stay per document).
template <bool Ob, class C, bool Rm, int Waves, int WavesPerEU, bool Adj = false, bool Loc = false>
__global__ __launch_bounds__(64 * Waves, WavesPerEU) void mergeTreeKernel(MtDeviceBatch batch, MtDeviceOut out,
                                                                      const uint32_t* __restrict__ docList,
                                                                      uint32_t count, const uint32_t* countDev,
                                                                      uint32_t* next) {
  using Doc = fmt_mt::Doc<Ob, C, Rm, Adj, Loc>;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));  // wave-uniform
  FMT_LDS fmt_mt::Scratch<C>* scratch = (FMT_LDS fmt_mt::Scratch<C>*)(lds + wave * scratchBytes<C, Ob>());
  if (countDev != nullptr) count = __builtin_amdgcn_readfirstlane(*countDev);
  // Documents are dealt one at a time from a device counter (next != nullptr): a wave that finishes
  // early takes the next document, so the launch ends when the work does, not when the unluckiest
  // static share of documents does. Every wave leaves once the counter passes `count`.
  for (uint32_t i = next ? 0u : blockIdx.x * Waves + wave;; i += next ? 0u : gridDim.x * Waves) {
    if (next != nullptr) {
      uint32_t v = 0;
      if ((threadIdx.x & 63) == 0) v = atomicAdd(next, 1u);
      i = __builtin_amdgcn_readfirstlane(v);
    }
    if (i >= count) break;
    const uint32_t d = docList ? docList[i] : i;
    const size_t slot = C::kHbmChars ? i : d;
    fmt_mt::DocInputs in;
    in.ops = batch.ops;
    in.begin = batch.docOpOffsets[d];
    in.end = batch.docOpOffsets[d + 1];
    in.text = batch.text;
    in.initOff = batch.docInit ? batch.docInit[2 * d] : 0u;
    in.initLen = batch.docInit ? batch.docInit[2 * d + 1] : 0u;
    in.propsOff = batch.propsOff;
    in.propsKv = batch.propsKv;
    in.nPropsOps = batch.nPropsOps;
    in.relpos = batch.relpos;
    in.nRelpos = batch.relpos ? batch.nRelpos : 0u;
    in.markerKey = batch.markerKey;
    in.adj = batch.adj;
    in.loc = Loc ? batch.loc : nullptr;
    in.doc = d;
    in.infoAll = batch.snapshotInfo;
    in.stampsAll = batch.snapshotStamps;
    in.nInfoAll = batch.snapshotInfo ? batch.nSnapshotInfo : 0u;
    if (batch.snapshots && batch.snapshots[d].loaded) {
      const fmt_mt_snapshot_doc sd = batch.snapshots[d];
      in.snapSegs = batch.snapshotSegs + sd.first_seg;
      in.snapInfo = batch.snapshotInfo ? batch.snapshotInfo + sd.first_seg : nullptr;
      in.snapStamps = batch.snapshotStamps;
      in.nHeader = sd.n_header;
      in.nBody = sd.n_body;
      in.snapMinSeq = sd.min_seq;
      in.snapSeq = sd.seq;
      in.loaded = 1;
    } else {
      in.snapSegs = nullptr;
      in.snapInfo = nullptr;
      in.snapStamps = nullptr;
      in.nHeader = in.nBody = 0;
      in.snapMinSeq = in.snapSeq = 0;
      in.loaded = 0;
    }
    fmt_mt::DocOutputs o;
    o.header = out.headers + d;
    o.leaves = out.leaves + slot * Slab<C>::kLeaves;
    o.chars = out.chars + slot * Slab<C>::kChars;
    o.props = out.props + slot * Slab<C>::kProps;
    if (batch.catchupOffsets) {
      const uint64_t c0 = batch.catchupOffsets[d], c1 = batch.catchupOffsets[d + 1];
      o.catchup = out.catchup + c0;
      o.catchupCap = static_cast<uint32_t>(c1 - c0);
    } else {
      o.catchup = nullptr;
      o.catchupCap = 0;
    }
    if (Rm && batch.rmOrderOffsets) {
      const uint64_t r0 = batch.rmOrderOffsets[d], r1 = batch.rmOrderOffsets[d + 1];
      o.rmOrder = out.rmOrder + r0;
      o.rmOrderCap = static_cast<uint32_t>(r1 - r0);
    } else {
      o.rmOrder = nullptr;
      o.rmOrderCap = 0;
    }
    if (Doc::kSavesCkpt || Doc::kResumesCkpt || (Ob && Doc::kResumesBig)) {  // (large tier: live obliterates)
      o.ckpt = out.ckpt ? out.ckpt + static_cast<size_t>(d) * Doc::kCkptWords : nullptr;
      o.ckptResume = Doc::kResumesCkpt && o.ckpt != nullptr &&
                     __builtin_amdgcn_readfirstlane(out.headers[d].status) == fmt_mt::kCkptEscalate;
    } else {
      o.ckpt = nullptr;
      o.ckptResume = false;
    }
    o.bigCkpt = nullptr;
    o.bigCkptChars = nullptr;
    o.legacyProps = out.legacyProps ? out.legacyProps + slot * Slab<C>::kLeaves : nullptr;
    o.hugeCkpt = Doc::kSavesHuge && out.hugeCkpt != nullptr ? out.hugeCkpt + slot * static_cast<size_t>(fmt_ckpt::kWords) : nullptr;
    if constexpr (Doc::kSavesBig) {  // batches without remove order (out.ckpt set): the small tier's own slabs
      if (out.ckpt != nullptr) {
        o.bigCkpt = reinterpret_cast<uint32_t*>(o.leaves);
        o.bigCkptChars = o.chars;
      }
    }
    if constexpr (Doc::kResumesBig) {
      if (out.smallLeaves != nullptr) {
        o.bigCkpt = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(out.smallLeaves + d * Slab<fmt_mt::SmallTier>::kLeaves));
        o.bigCkptChars = const_cast<uint16_t*>(out.smallChars + d * Slab<fmt_mt::SmallTier>::kChars);
        o.ckptResume = __builtin_amdgcn_readfirstlane(out.headers[d].status) == fmt_mt::kCkptEscalate;
      }
    }
    Doc doc;
    doc.s = scratch;
    doc.run(in, o);
#if FMT_PROFILE && FMT_GPU
    if ((threadIdx.x & 63) == 0)
      for (int c = 0; c < fmt_mt::kPfCount; c++) atomicAdd(&g_mtProfile[c], static_cast<unsigned long long>(doc.prof[c]));
#endif
  }
}

// The documents a tier could not hold (FMT_E_CAPACITY) among docList[0..nDocs) (nDocs = countDev[0]
// when set): esc[0] = count, esc[1..] = ids. A limit the large tier shares (fmt_mt::kCapacityFinal)
// is reported as FMT_E_CAPACITY without escalation. Defined in mergetree.hip.
__global__ __launch_bounds__(256) void collectOverflowKernel(fmt_mt_doc_result* __restrict__ headers,
                                                             const uint32_t* __restrict__ docList, uint32_t nDocs,
                                                             const uint32_t* countDev, uint32_t* esc);

#ifdef FMT_MT_COLLECT_DEFINE
__global__ __launch_bounds__(256) void collectOverflowKernel(fmt_mt_doc_result* __restrict__ headers,
                                                             const uint32_t* __restrict__ docList, uint32_t nDocs,
                                                             const uint32_t* countDev, uint32_t* esc) {
  if (countDev != nullptr) nDocs = *countDev;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nDocs; i += gridDim.x * blockDim.x) {
    const uint32_t d = docList ? docList[i] : i;
    const int st = headers[d].status;
    if (st == fmt_mt::kCapacityFinal) headers[d].status = FMT_E_CAPACITY;
    if (st == FMT_E_CAPACITY || st == fmt_mt::kCkptEscalate) {
      const uint32_t k = atomicAdd(esc, 1u);
      esc[1 + k] = d;
    }
  }
}
#endif

// countDev: the list length lives on the device (an overflow list); `count` then bounds it (grid size).
template <bool Ob, class C, bool Rm, int Waves, int WavesPerEU, bool Adj = false, bool Loc = false>
static hipError_t launchTier(const MtDeviceBatch& batch, const MtDeviceOut& out, const uint32_t* docList,
                             uint32_t count, uint32_t* esc, int numCUs, hipStream_t stream,
                             const uint32_t* countDev = nullptr, uint32_t* next = nullptr) {
  const size_t lds = scratchBytes<C, Ob>() * Waves;
  // One resident wave of workgroups: every workgroup strides over the same number of documents,
  // so none waits behind the residency limit (VGPRs cap the small tier at 2 waves/SIMD).
  int blocksPerCU = 0;
  const hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocksPerCU, mergeTreeKernel<Ob, C, Rm, Waves, WavesPerEU, Adj, Loc>, 64 * Waves, lds);
  if (e != hipSuccess) return e;
  const uint32_t wanted = (count + Waves - 1) / Waves;
  const uint32_t cap = static_cast<uint32_t>(numCUs * (blocksPerCU > 0 ? blocksPerCU : 1));
  const uint32_t grid = wanted < cap ? (wanted > 0 ? wanted : 1) : cap;
  hipLaunchKernelGGL((mergeTreeKernel<Ob, C, Rm, Waves, WavesPerEU, Adj, Loc>), dim3(grid), dim3(64 * Waves), lds, stream, batch, out,
                     docList, count, countDev, next);
  if (esc != nullptr) {  // over the documents this launch replayed
    const uint32_t g = (count + 255) / 256;
    hipLaunchKernelGGL(collectOverflowKernel, dim3(g < 1024 ? (g > 0 ? g : 1) : 1024), dim3(256), 0, stream, out.headers,
                       docList, count, countDev, esc);
  }
  return hipGetLastError();
}

}  // namespace fmt_kernels
