// mt_emu.cpp — TEST INFRASTRUCTURE ONLY: the merge-tree engine source (mt_engine.h) compiled for the
// host with the 64-lane emulation of wave.h, so the CPU parity suite can check the exact kernel
// logic against the oracle without a GPU. Never loaded by the product (libfmt.so has no CPU path).
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "../../fluidframework_amd/csrc/mt_engine.h"

// Annotate-adjust state of the last emulated replay (the runtime's number slabs, fixed capacity
// here): the batch's host numbers sorted for number → id lookups, per-document number tables.
constexpr uint32_t kEmuNumCap = 4096;
static std::vector<double> g_numSorted, g_nums;
static std::vector<uint32_t> g_numSortedId, g_numCount;
static std::vector<uint64_t> g_numOffs;
static fmt_mt::AdjustTables g_adj;
// property-manager records (Doc::pm*) and the per-leaf legacy prop sets of the last replay
constexpr uint32_t kEmuPmCap = 1 << 14;
static std::vector<uint32_t> g_pm;
static std::vector<uint64_t> g_pmOffs;
static std::vector<uint16_t> g_legacy;
static size_t g_legacyStride = 0;

static std::vector<uint32_t> g_numSortedOffs;

static void prepareNumbers(const fmt_mt_batch* b) {
  g_numSorted.clear();
  g_numSortedId.clear();
  g_numSortedOffs.clear();
  g_nums.clear();
  g_numCount.assign(b->n_docs, 0u);
  if (b->adjusts == nullptr || b->value_num == nullptr) return;
  // the host numbers ascending with their first value id (runtime.cpp fmt_mt_load): one list, or per
  // document with local ids when value ids are document-local (doc_value_base)
  auto sortNumbers = [&](uint32_t lo, uint32_t hi, uint32_t base) {
    std::vector<std::pair<double, uint32_t>> v;
    for (uint32_t i = lo; i < hi; i++)
      if (b->value_num[base + i] == b->value_num[base + i]) v.emplace_back(b->value_num[base + i] == 0.0 ? 0.0 : b->value_num[base + i], i);
    std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    const size_t first = g_numSorted.size();
    for (const auto& [x, i] : v) {
      if (g_numSorted.size() > first && g_numSorted.back() == x) continue;  // the first id of an equal number
      g_numSorted.push_back(x);
      g_numSortedId.push_back(i);
    }
  };
  if (b->doc_value_base != nullptr) {
    g_numSortedOffs.assign(1, 0u);
    for (uint32_t d = 0; d < b->n_docs; d++) {
      sortNumbers(1, b->doc_value_base[d + 1] - b->doc_value_base[d] + 1, b->doc_value_base[d]);
      g_numSortedOffs.push_back(static_cast<uint32_t>(g_numSorted.size()));
    }
  } else {
    sortNumbers(0, b->n_values, 0);
  }
  g_nums.assign(static_cast<size_t>(b->n_docs) * kEmuNumCap, 0.0);
  g_numOffs.resize(b->n_docs + 1ull);
  for (uint32_t d = 0; d <= b->n_docs; d++) g_numOffs[d] = static_cast<uint64_t>(d) * kEmuNumCap;
  g_pm.assign(static_cast<size_t>(b->n_docs) * kEmuPmCap * 4, 0u);
  g_pmOffs.resize(b->n_docs + 1ull);
  for (uint32_t d = 0; d <= b->n_docs; d++) g_pmOffs[d] = static_cast<uint64_t>(d) * kEmuPmCap;
  g_adj = fmt_mt::AdjustTables{};
  g_adj.adjusts = b->adjusts;
  g_adj.nAdjusts = b->n_adjusts;
  g_adj.nValues = b->value_num ? b->n_values : 0u;
  g_adj.valueNum = b->value_num;
  g_adj.numSorted = g_numSorted.data();
  g_adj.numSortedId = g_numSortedId.data();
  g_adj.nNumSorted = static_cast<uint32_t>(g_numSorted.size());
  g_adj.valueBase = b->doc_value_base;
  g_adj.numSortedOffs = b->doc_value_base != nullptr ? g_numSortedOffs.data() : nullptr;
  g_adj.nums = g_nums.data();
  g_adj.numOffsets = g_numOffs.data();
  g_adj.numCount = g_numCount.data();
  g_adj.pm = g_pm.data();
  g_adj.pmOffsets = g_pmOffs.data();
}

// ckpt (plain batches): per-document tier checkpoints; the compact tier saves, the small tier resumes
// the documents whose header says kCkptEscalate and, with onlyEscalated, replays only those and the
// documents that overflowed (the runtime's cascade over the overflow list).
// f4 (the local client): per-document slabs of the last emu_mt_replay_local (fixed capacities)
constexpr uint32_t kEmuGroupCap = 4096, kEmuRecCap = 16384, kEmuRegenCap = 4096, kEmuRegenTextCap = 1 << 16,
                   kEmuScratchCap = 1 << 16;
static std::vector<uint32_t> g_lgroups, g_lrecs, g_lpm, g_lscratch, g_lregenCount;
static std::vector<uint64_t> g_lgroupOffs, g_lrecOffs, g_lpmOffs, g_lscratchOffs, g_lregenOffs, g_lregenTextOffs;
static std::vector<fmt_mt_op> g_lregen;
static std::vector<uint16_t> g_lregenText;
static fmt_mt::LocalTables g_loc;

static void prepareLocal(uint32_t nDocs) {
  auto offs = [&](std::vector<uint64_t>& v, uint64_t cap) {
    v.resize(nDocs + 1ull);
    for (uint32_t d = 0; d <= nDocs; d++) v[d] = static_cast<uint64_t>(d) * cap;
  };
  g_lgroups.assign(static_cast<size_t>(nDocs) * kEmuGroupCap * 8, 0u);
  g_lrecs.assign(static_cast<size_t>(nDocs) * kEmuRecCap * 2, 0u);
  g_lpm.assign(static_cast<size_t>(nDocs) * kEmuPmCap * 4, 0u);
  g_lscratch.assign(static_cast<size_t>(nDocs) * kEmuScratchCap, 0u);
  g_lregen.assign(static_cast<size_t>(nDocs) * kEmuRegenCap, fmt_mt_op{});
  g_lregenText.assign(static_cast<size_t>(nDocs) * kEmuRegenTextCap, 0u);
  g_lregenCount.assign(2ull * nDocs, 0u);
  offs(g_lgroupOffs, kEmuGroupCap);
  offs(g_lrecOffs, kEmuRecCap);
  offs(g_lpmOffs, kEmuPmCap);
  offs(g_lscratchOffs, kEmuScratchCap);
  offs(g_lregenOffs, kEmuRegenCap);
  offs(g_lregenTextOffs, kEmuRegenTextCap);
  g_loc = fmt_mt::LocalTables{g_lgroups.data(), g_lgroupOffs.data(), g_lrecs.data(), g_lrecOffs.data(),
                              g_lpm.data(), g_lpmOffs.data(), g_lregen.data(), g_lregenOffs.data(),
                              g_lregenText.data(), g_lregenTextOffs.data(), g_lregenCount.data(),
                              g_lscratch.data(), g_lscratchOffs.data()};
}

template <bool Ob, class C, bool Rm = false, bool Adj = false, bool Loc = false>
static int replayAll(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                     fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup,
                     fmt_mt_remove_order* rmOrder, uint32_t capRm, uint32_t* ckpt = nullptr,
                     bool onlyEscalated = false, size_t leafStride = 0, size_t charStride = 0,
                     const fmt_mt_leaf* smallLeaves = nullptr, const uint16_t* smallChars = nullptr,
                     uint16_t* legacy = nullptr, uint32_t* hugeCk = nullptr) {
  using Doc = fmt_mt::Doc<Ob, C, Rm, Adj, Loc>;
  auto scratch = std::make_unique<fmt_mt::Scratch<C>>();
  auto doc = std::make_unique<Doc>();
  int status = FMT_OK;
  for (uint32_t d = 0; d < b->n_docs; d++) {
    if (onlyEscalated && headers[d].status != FMT_E_CAPACITY && headers[d].status != fmt_mt::kCkptEscalate) continue;
    std::memset(scratch.get(), 0xCD, sizeof(fmt_mt::Scratch<C>));  // poison: state must be initialized
    fmt_mt::DocInputs in;
    in.ops = b->ops;
    in.begin = b->doc_op_offsets[d];
    in.end = b->doc_op_offsets[d + 1];
    in.text = b->text;
    in.initOff = b->doc_init ? b->doc_init[2 * d] : 0u;
    in.initLen = b->doc_init ? b->doc_init[2 * d + 1] : 0u;
    in.propsOff = b->props_off;
    in.propsKv = b->props_kv;
    in.nPropsOps = b->n_props_ops;
    in.relpos = b->relpos;
    in.nRelpos = b->relpos ? b->n_relpos : 0u;
    in.markerKey = b->marker_id_key;
    in.adj = g_nums.empty() ? nullptr : &g_adj;
    in.doc = d;
    in.loc = Loc ? &g_loc : nullptr;
    in.infoAll = b->snapshot_info;
    in.stampsAll = b->snapshot_stamps;
    in.nInfoAll = b->snapshot_info ? b->n_snapshot_segs : 0u;
    if (b->snapshots && b->snapshots[d].loaded) {
      const fmt_mt_snapshot_doc sd = b->snapshots[d];
      in.snapSegs = b->snapshot_segs + sd.first_seg;
      in.snapInfo = b->snapshot_info ? b->snapshot_info + sd.first_seg : nullptr;
      in.snapStamps = b->snapshot_stamps;
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
    o.header = headers + d;
    o.leaves = leaves + static_cast<size_t>(d) * (leafStride ? leafStride : Doc::kCapLeaves);
    o.chars = chars + static_cast<size_t>(d) * (charStride ? charStride : Doc::kCapChars);
    o.props = props + static_cast<size_t>(d) * Doc::kPropCap;
    o.catchup = catchup ? catchup + static_cast<size_t>(d) * capCatchup : nullptr;
    o.catchupCap = catchup ? capCatchup : 0u;
    o.rmOrder = rmOrder ? rmOrder + static_cast<size_t>(d) * capRm : nullptr;
    o.rmOrderCap = rmOrder ? capRm : 0u;
    o.ckpt = ckpt && (Doc::kSavesCkpt || Doc::kResumesCkpt || (Ob && Doc::kResumesBig))
                 ? ckpt + static_cast<size_t>(d) * Doc::kCkptWords : nullptr;
    o.ckptResume = o.ckpt != nullptr && Doc::kResumesCkpt && headers[d].status == fmt_mt::kCkptEscalate;
    o.bigCkpt = nullptr;
    o.bigCkptChars = nullptr;
    o.legacyProps = legacy ? legacy + static_cast<size_t>(d) * (leafStride ? leafStride : Doc::kCapLeaves) : nullptr;
    o.hugeCkpt = Doc::kSavesHuge && hugeCk != nullptr ? hugeCk + static_cast<size_t>(d) * fmt_ckpt::kWords : nullptr;
    if (Doc::kSavesBig && ckpt != nullptr) {  // the small tier of a cascade: its own slabs
      o.bigCkpt = reinterpret_cast<uint32_t*>(o.leaves);
      o.bigCkptChars = o.chars;
    }
    if (Doc::kResumesBig && smallLeaves != nullptr) {
      o.bigCkpt = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(smallLeaves + static_cast<size_t>(d) * 512));
      o.bigCkptChars = const_cast<uint16_t*>(smallChars + static_cast<size_t>(d) * fmt_mt::SmallTier::kCapChars);
      o.ckptResume = headers[d].status == fmt_mt::kCkptEscalate;
    }
    new (doc.get()) Doc();
    doc->s = scratch.get();
    doc->run(in, o);
    if (headers[d].status == fmt_mt::kCapacityFinal) headers[d].status = FMT_E_CAPACITY;  // as collectOverflowKernel
    if (headers[d].status == fmt_mt::kCkptEscalate) continue;  // the small tier resumes it
    if (headers[d].status == fmt_ckpt::kStatusHuge) continue;  // the huge tier resumes it
    if (headers[d].status != FMT_OK && status == FMT_OK) status = headers[d].status;
  }
  return status;
}

// The runtime's compact → small cascade with checkpoints (results at small-tier strides).
template <bool Ob>
static int cascadeCompactSmall(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                               fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup,
                               fmt_mt_remove_order* rmOrder, uint32_t capRm) {
  using S = fmt_mt::SmallTier;
  using D = fmt_mt::Doc<Ob, fmt_mt::CompactTier>;
  std::unique_ptr<uint32_t[]> ck(new uint32_t[static_cast<size_t>(b->n_docs) * D::kCkptWords]);
  const size_t stride = fmt_mt::Doc<Ob, S>::kCapLeaves;
  replayAll<Ob, fmt_mt::CompactTier>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm, ck.get(),
                                     false, stride, S::kCapChars);
  return replayAll<Ob, S>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm, ck.get(), true);
}

// The whole cascade: compact → small → large with both checkpoints (results at large-tier strides).
template <bool Ob>
static int fullCascade(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                       fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup,
                       fmt_mt_remove_order* rmOrder, uint32_t capRm) {
  using S = fmt_mt::SmallTier;
  using G = fmt_mt::LargeTier;
  using D = fmt_mt::Doc<Ob, fmt_mt::CompactTier>;
  using DS = fmt_mt::Doc<Ob, S>;
  using DL = fmt_mt::Doc<Ob, G>;
  const size_t n = b->n_docs;
  std::unique_ptr<uint32_t[]> ck(new uint32_t[n * D::kCkptWords]);
  std::unique_ptr<fmt_mt_leaf[]> sl(new fmt_mt_leaf[n * DS::kCapLeaves]);
  std::unique_ptr<uint16_t[]> sc(new uint16_t[n * S::kCapChars]);
  std::unique_ptr<fmt_mt_propset[]> sp(new fmt_mt_propset[n * S::kPropCap]);
  replayAll<Ob, fmt_mt::CompactTier>(b, headers, sl.get(), sc.get(), sp.get(), catchup, capCatchup, rmOrder, capRm,
                                     ck.get(), false, DS::kCapLeaves, S::kCapChars);
  replayAll<Ob, S>(b, headers, sl.get(), sc.get(), sp.get(), catchup, capCatchup, rmOrder, capRm, ck.get(), true);
  for (size_t d = 0; d < n; d++) {  // documents done below the large tier: results to the large strides
    const fmt_mt_doc_result& h = headers[d];
    if (h.status == FMT_E_CAPACITY || h.status == fmt_mt::kCkptEscalate) continue;
    std::memcpy(leaves + d * DL::kCapLeaves, sl.get() + d * DS::kCapLeaves, h.n_leaves * sizeof(fmt_mt_leaf));
    std::memcpy(chars + d * G::kCapChars, sc.get() + d * S::kCapChars, h.n_chars * sizeof(uint16_t));
    std::memcpy(props + d * G::kPropCap, sp.get() + d * S::kPropCap, h.n_props * sizeof(fmt_mt_propset));
  }
  // (the large tier reads the live-obliterate table from the checkpoint slots, Ob only)
  return replayAll<Ob, G>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm, Ob ? ck.get() : nullptr,
                          true, 0, 0, sl.get(), sc.get());
}

// Batches with annotate-adjust: the small tier (Doc<true, S, Rm, true>) over every document; with
// large, documents it cannot hold replay again from their first op in the large tier (results at
// large strides), as the runtime runs them.
static int adjustCascade(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                         fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup,
                         fmt_mt_remove_order* rmOrder, uint32_t capRm, int large, bool rm) {
  using S = fmt_mt::SmallTier;
  using G = fmt_mt::LargeTier;
  if (large == 0 || large == 3) {
    g_legacyStride = fmt_mt::Doc<true, S>::kCapLeaves;
    g_legacy.assign(b->n_docs * g_legacyStride, 0xFFFFu);
    return rm ? replayAll<true, S, true, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm,
                                               nullptr, false, 0, 0, nullptr, nullptr, g_legacy.data())
              : replayAll<true, S, false, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm,
                                                nullptr, false, 0, 0, nullptr, nullptr, g_legacy.data());
  }
  using DS = fmt_mt::Doc<true, S, false, true>;
  using DL = fmt_mt::Doc<true, G, false, true>;
  const size_t n = b->n_docs;
  std::unique_ptr<fmt_mt_leaf[]> sl(new fmt_mt_leaf[n * DS::kCapLeaves]);
  std::unique_ptr<uint16_t[]> sc(new uint16_t[n * S::kCapChars]);
  std::unique_ptr<fmt_mt_propset[]> sp(new fmt_mt_propset[n * S::kPropCap]);
  std::vector<uint16_t> smallLegacy(n * DS::kCapLeaves, 0xFFFFu);
  if (rm) replayAll<true, S, true, true>(b, headers, sl.get(), sc.get(), sp.get(), catchup, capCatchup, rmOrder, capRm,
                                         nullptr, false, 0, 0, nullptr, nullptr, smallLegacy.data());
  else replayAll<true, S, false, true>(b, headers, sl.get(), sc.get(), sp.get(), catchup, capCatchup, rmOrder, capRm,
                                       nullptr, false, 0, 0, nullptr, nullptr, smallLegacy.data());
  g_legacyStride = DL::kCapLeaves;
  g_legacy.assign(n * g_legacyStride, 0xFFFFu);
  for (size_t d = 0; d < n; d++) {
    const fmt_mt_doc_result& h = headers[d];
    if (h.status == FMT_E_CAPACITY) continue;
    std::memcpy(leaves + d * DL::kCapLeaves, sl.get() + d * DS::kCapLeaves, h.n_leaves * sizeof(fmt_mt_leaf));
    std::memcpy(chars + d * G::kCapChars, sc.get() + d * S::kCapChars, h.n_chars * sizeof(uint16_t));
    std::memcpy(props + d * G::kPropCap, sp.get() + d * S::kPropCap, h.n_props * sizeof(fmt_mt_propset));
    std::memcpy(g_legacy.data() + d * DL::kCapLeaves, smallLegacy.data() + d * DS::kCapLeaves, h.n_leaves * sizeof(uint16_t));
  }
  return rm ? replayAll<true, G, true, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm, nullptr,
                                             true, 0, 0, nullptr, nullptr, g_legacy.data())
            : replayAll<true, G, false, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm, nullptr,
                                              true, 0, 0, nullptr, nullptr, g_legacy.data());
}

template <bool Adj>
static int replayLocal(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                       fmt_mt_propset* props, int largeOnly) {
  using G = fmt_mt::LargeTier;
  using K = fmt_mt::CompactTier;
  using S = fmt_mt::SmallTier;
  using DS = fmt_mt::Doc<false, S>;
  using DL = fmt_mt::Doc<false, G, false, Adj, true>;
  const size_t n = b->n_docs;
  // (annotate-adjust batches: the legacy getAtSeq views, emu_mt_legacy_props, at large strides)
  std::vector<uint16_t> smallLegacy(Adj ? n * DS::kCapLeaves : 0, 0xFFFFu);
  if (Adj) {
    g_legacyStride = DL::kCapLeaves;
    g_legacy.assign(n * g_legacyStride, 0xFFFFu);
  }
  if (largeOnly == 1)
    return replayAll<false, G, false, Adj, true>(b, headers, leaves, chars, props, nullptr, 0, nullptr, 0, nullptr, false, 0,
                                                 0, nullptr, nullptr, Adj ? g_legacy.data() : nullptr);
  std::unique_ptr<fmt_mt_leaf[]> sl(new fmt_mt_leaf[n * DS::kCapLeaves]);
  std::unique_ptr<uint16_t[]> sc(new uint16_t[n * S::kCapChars]);
  std::unique_ptr<fmt_mt_propset[]> sp(new fmt_mt_propset[n * S::kPropCap]);
  if (largeOnly == 2 || largeOnly == 3)
    replayAll<false, K, false, Adj, true>(b, headers, sl.get(), sc.get(), sp.get(), nullptr, 0, nullptr, 0, nullptr, false,
                                          DS::kCapLeaves, S::kCapChars, nullptr, nullptr,
                                          Adj ? smallLegacy.data() : nullptr);
  if (largeOnly == 2) return FMT_OK;  // (diagnostics: the compact tier's statuses alone)
  // the small tier's local variant over the documents the compact tier could not hold (from op 0);
  // mode 0 (the runtime's default, mergetree_local.hip FMT_LOCAL_PATH 1) starts here with every document
  replayAll<false, S, false, Adj, true>(b, headers, sl.get(), sc.get(), sp.get(), nullptr, 0, nullptr, 0, nullptr,
                                        largeOnly == 3, 0, 0, nullptr, nullptr, Adj ? smallLegacy.data() : nullptr);
  for (size_t d = 0; d < n; d++) {  // documents done below the large tier: results to the large strides
    const fmt_mt_doc_result& h = headers[d];
    if (h.status == FMT_E_CAPACITY) continue;
    std::memcpy(leaves + d * DL::kCapLeaves, sl.get() + d * DS::kCapLeaves, h.n_leaves * sizeof(fmt_mt_leaf));
    std::memcpy(chars + d * G::kCapChars, sc.get() + d * S::kCapChars, h.n_chars * sizeof(uint16_t));
    std::memcpy(props + d * G::kPropCap, sp.get() + d * S::kPropCap, h.n_props * sizeof(fmt_mt_propset));
    if (Adj) std::memcpy(g_legacy.data() + d * DL::kCapLeaves, smallLegacy.data() + d * DS::kCapLeaves, h.n_leaves * sizeof(uint16_t));
  }
  return replayAll<false, G, false, Adj, true>(b, headers, leaves, chars, props, nullptr, 0, nullptr, 0, nullptr, true, 0, 0,
                                               nullptr, nullptr, Adj ? g_legacy.data() : nullptr);
}

extern "C" {

// large = 0: the small tier (registers + LDS text); 1: the large tier (HBM text) that the runtime
// replays overflowing documents in; 2: the compact tier (4 register rows) plain batches start in;
// 3: the compact → small cascade with checkpoints (small-tier strides); 4: the whole compact → small
// → large cascade (large-tier strides).
int emu_mt_capacity(int large, uint32_t* leaves, uint32_t* chars, uint32_t* props) {
  if (large == 3) large = 0;
  if (large == 4) large = 1;
  if (large == 2) {
    *leaves = fmt_mt::Doc<false, fmt_mt::CompactTier>::kCapLeaves;
    *chars = fmt_mt::CompactTier::kCapChars;
    *props = fmt_mt::CompactTier::kPropCap;
  } else if (large) {
    *leaves = fmt_mt::Doc<false, fmt_mt::LargeTier>::kCapLeaves;
    *chars = fmt_mt::LargeTier::kCapChars;
    *props = fmt_mt::LargeTier::kPropCap;
  } else {
    *leaves = fmt_mt::Doc<false, fmt_mt::SmallTier>::kCapLeaves;
    *chars = fmt_mt::SmallTier::kCapChars;
    *props = fmt_mt::SmallTier::kPropCap;
  }
  return 0;
}

// Same strides as the GPU result buffers of the tier (kCapLeaves / kCapChars / kPropCap per
// document). Like the runtime, batches holding obliterates run the Doc<true> variant (or always,
// with forceOb).
int emu_mt_replay(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                  fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup, int forceOb, int large,
                  fmt_mt_remove_order* rmOrder, uint32_t capRm) {
  prepareNumbers(b);
  g_legacyStride = 0;
  if (b->adjusts != nullptr) {  // the runtime's annotate-adjust path: Adj variants, no checkpoints
    bool rmA = false;
    for (uint64_t i = 0; i < b->n_ops && !rmA; i++) rmA = (b->ops[i].flags & FMT_MT_F_RMORDER) != 0;
    return adjustCascade(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm, large, rmA);
  }
  bool ob = forceOb != 0;
  for (uint64_t i = 0; i < b->n_ops && !ob; i++) ob = b->ops[i].type == FMT_MT_OBLITERATE || b->ops[i].type == FMT_MT_OBLITERATE_SIDED;
  using S = fmt_mt::SmallTier;
  using G = fmt_mt::LargeTier;
  bool rm = false;
  for (uint64_t i = 0; i < b->n_ops && !rm; i++) rm = (b->ops[i].flags & FMT_MT_F_RMORDER) != 0;
  if (large == 2 && !rm)
    return ob ? replayAll<true, fmt_mt::CompactTier>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm)
              : replayAll<false, fmt_mt::CompactTier>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
  if (large == 4 && !rm)  // the whole cascade: compact → small → large, results at large strides
    return ob ? fullCascade<true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm)
              : fullCascade<false>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
  if (large == 3 && !rm)  // the runtime's cascade: compact tier with checkpoints, then the small tier
    return ob ? cascadeCompactSmall<true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm)
              : cascadeCompactSmall<false>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
  if (large == 1) {
    if (ob && rm) return replayAll<true, G, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
    if (ob) return replayAll<true, G>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
    if (rm) return replayAll<false, G, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
    return replayAll<false, G>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
  }
  if (ob && rm) return replayAll<true, S, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
  if (ob) return replayAll<true, S>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
  if (rm) return replayAll<false, S, true>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
  return replayAll<false, S>(b, headers, leaves, chars, props, catchup, capCatchup, rmOrder, capRm);
}

// The large tier over every document from its first op, each document it is about to outgrow
// stopping with its large → huge checkpoint (hugeCk: fmt_ckpt::kWords words per document; header
// status fmt_ckpt::kStatusHuge) for emu_huge_resume (results at large strides).
// Annotate-adjust batches run the large tier's Adj variant (Doc<true, G, false, true>, as the runtime):
// the legacy views of the documents it finishes via emu_mt_legacy_props, and each document's
// PropertiesManager records and computed numbers, which the huge tier resumes with, via emu_mt_adj_slab.
int emu_mt_replay_large_ckpt(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                             fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup, uint32_t* hugeCk) {
  g_nums.clear();
  g_legacyStride = 0;
  if (b->adjusts != nullptr) {
    prepareNumbers(b);
    using DL = fmt_mt::Doc<true, fmt_mt::LargeTier, false, true>;
    g_legacyStride = DL::kCapLeaves;
    g_legacy.assign(static_cast<size_t>(b->n_docs) * g_legacyStride, 0xFFFFu);
    return replayAll<true, fmt_mt::LargeTier, false, true>(b, headers, leaves, chars, props, catchup, capCatchup, nullptr, 0,
                                                           nullptr, false, 0, 0, nullptr, nullptr, g_legacy.data(), hugeCk);
  }
  bool ob = false;
  for (uint64_t i = 0; i < b->n_ops && !ob; i++) ob = b->ops[i].type == FMT_MT_OBLITERATE || b->ops[i].type == FMT_MT_OBLITERATE_SIDED;
  using G = fmt_mt::LargeTier;
  return ob ? replayAll<true, G>(b, headers, leaves, chars, props, catchup, capCatchup, nullptr, 0, nullptr, false, 0, 0,
                                 nullptr, nullptr, nullptr, hugeCk)
            : replayAll<false, G>(b, headers, leaves, chars, props, catchup, capCatchup, nullptr, 0, nullptr, false, 0, 0,
                                  nullptr, nullptr, nullptr, hugeCk);
}

// As emu_mt_replay_large_ckpt for a batch with remove-order recording (the large tier's Rm variant):
// rmOrder[n_docs x capRm] receives the entries, which keep their leaf ids in a stopped document.
int emu_mt_replay_large_ckpt_rm(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                                fmt_mt_propset* props, fmt_mt_remove_order* rmOrder, uint32_t capRm, uint32_t* hugeCk) {
  g_nums.clear();
  g_legacyStride = 0;
  bool ob = false;
  for (uint64_t i = 0; i < b->n_ops && !ob; i++) ob = b->ops[i].type == FMT_MT_OBLITERATE || b->ops[i].type == FMT_MT_OBLITERATE_SIDED;
  using G = fmt_mt::LargeTier;
  return ob ? replayAll<true, G, true>(b, headers, leaves, chars, props, nullptr, 0, rmOrder, capRm, nullptr, false, 0, 0,
                                       nullptr, nullptr, nullptr, hugeCk)
            : replayAll<false, G, true>(b, headers, leaves, chars, props, nullptr, 0, rmOrder, capRm, nullptr, false, 0, 0,
                                        nullptr, nullptr, nullptr, hugeCk);
}

uint32_t emu_huge_ckpt_words() { return fmt_ckpt::kWords; }

// f4 batches (local submissions, acks, rollbacks, reconnects), as the runtime runs them (round 6): the
// small tier's Loc variant over every document, then the large tier's over the documents it could not
// hold, from their first op (results at large strides). Mode 3: the compact tier's Loc variant first,
// the small tier's over what it could not hold, then the large tier's (FMT_LOCAL_PATH 2). largeOnly: every
// document in the large tier (round 5's path); 2: the compact tier alone (its statuses, diagnostics).
// Annotate-adjust batches run the Adj local variants (Doc<false, C, false, true, true>), with the
// batch's number tables (emu_mt_numbers) and legacy views (emu_mt_legacy_props).
int emu_mt_replay_local(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                        fmt_mt_propset* props, int largeOnly) {
  g_nums.clear();
  g_legacyStride = 0;
  prepareLocal(b->n_docs);
  if (b->adjusts != nullptr) {
    prepareNumbers(b);
    return replayLocal<true>(b, headers, leaves, chars, props, largeOnly);
  }
  return replayLocal<false>(b, headers, leaves, chars, props, largeOnly);
}

// Document d's regenerated ops (and their text) after the last emu_mt_replay_local: copies <= the
// caps, returns the op count; *nText = the text units.
int emu_mt_regen(uint32_t d, fmt_mt_op* ops, uint32_t capOps, uint16_t* text, uint32_t capText, uint32_t* nText) {
  if (2ull * d + 1 >= g_lregenCount.size()) return -1;
  const uint32_t n = g_lregenCount[2 * d], t = g_lregenCount[2 * d + 1];
  for (uint32_t k = 0; k < n && k < capOps; k++) ops[k] = g_lregen[static_cast<size_t>(d) * kEmuRegenCap + k];
  for (uint32_t k = 0; k < t && k < capText; k++) text[k] = g_lregenText[static_cast<size_t>(d) * kEmuRegenTextCap + k];
  *nText = t;
  return static_cast<int>(n);
}

// Document d's legacy prop sets (getAtSeq at minSeq, per leaf) after the last emu_mt_replay of a batch
// with adjusts: copies <= cap, returns the count (0 without adjusts).
int emu_mt_legacy_props(uint32_t d, uint16_t* out, uint32_t cap) {
  if (g_legacyStride == 0 || (d + 1) * g_legacyStride > g_legacy.size()) return 0;
  for (uint32_t k = 0; k < cap && k < g_legacyStride; k++) out[k] = g_legacy[d * g_legacyStride + k];
  return static_cast<int>(g_legacyStride);
}

// Document d's annotate-adjust slabs after the last emu_mt_replay_large_ckpt: its PropertiesManager
// records (capRecs x 4 words from the slab's start) and computed numbers (<= capNums, *nNums = count).
int emu_mt_adj_slab(uint32_t d, uint32_t* pm, uint32_t capRecs, double* nums, uint32_t capNums, uint32_t* nNums) {
  if (g_nums.empty() || d >= g_numCount.size()) return -1;
  for (size_t k = 0; k < 4ull * capRecs && k < 4ull * kEmuPmCap; k++) pm[k] = g_pm[static_cast<size_t>(d) * kEmuPmCap * 4 + k];
  const uint32_t n = g_numCount[d];
  for (uint32_t k = 0; k < n && k < capNums; k++) nums[k] = g_nums[static_cast<size_t>(d) * kEmuNumCap + k];
  *nNums = n;
  return 0;
}

// Document d's computed numbers after the last emu_mt_replay: returns their count, copies <= cap.
int emu_mt_numbers(uint32_t d, double* out, uint32_t cap) {
  if (d >= g_numCount.size()) return 0;
  const uint32_t n = g_numCount[d];
  for (uint32_t k = 0; k < n && k < cap; k++) out[k] = g_nums[static_cast<size_t>(d) * kEmuNumCap + k];
  return static_cast<int>(n);
}

}  // extern "C"
