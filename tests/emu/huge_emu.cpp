// huge_emu.cpp — TEST INFRASTRUCTURE ONLY: the huge-document engine (huge_engine.h, BASELINE
// config 5 / T3) compiled for the host with the 64-lane emulation of wave.h, so the CPU suite checks
// its logic against the oracle without a GPU. Never loaded by the product.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#ifdef FMT_HUGE_CHECK_BUILD
#define FMT_HUGE_CHECK 1
#endif

#include "../../fluidframework_amd/csrc/huge_engine.h"

using namespace fmt_huge;

// Annotate-adjust tables of the last replay (runtime.cpp fmt_mt_load's, one document's slabs here):
// the host numbers ascending with their first value id, the computed-number slab and the
// PropertiesManager records.
namespace {
constexpr uint32_t kEmuNumCap = 1 << 16;
constexpr uint32_t kEmuPmCap = 1 << 20;
std::vector<double> g_numSorted, g_nums;
std::vector<uint32_t> g_numSortedId, g_numSortedOffs, g_numCount, g_pm;
std::vector<uint64_t> g_numOffs, g_pmOffs;
fmt_mt::AdjustTables g_adj;

const fmt_mt::AdjustTables* prepareNumbers(const fmt_mt_batch* b) {
  g_numSorted.clear();
  g_numSortedId.clear();
  g_numSortedOffs.clear();
  if (b->adjusts == nullptr || b->value_num == nullptr) return nullptr;
  auto sortNumbers = [&](uint32_t lo, uint32_t hi, uint32_t base) {
    std::vector<std::pair<double, uint32_t>> v;
    for (uint32_t i = lo; i < hi; i++)
      if (b->value_num[base + i] == b->value_num[base + i]) v.emplace_back(b->value_num[base + i] == 0.0 ? 0.0 : b->value_num[base + i], i);
    std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    const size_t first = g_numSorted.size();
    for (const auto& [x, i] : v) {
      if (g_numSorted.size() > first && g_numSorted.back() == x) continue;
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
  // every document indexes its own slabs; only the replayed one gets room
  g_nums.assign(kEmuNumCap, 0.0);
  g_numCount.assign(b->n_docs, 0u);
  g_pm.assign(static_cast<size_t>(kEmuPmCap) * 4, 0u);
  g_adj = fmt_mt::AdjustTables{};
  g_adj.adjusts = b->adjusts;
  g_adj.nAdjusts = b->n_adjusts;
  g_adj.nValues = b->n_values;
  g_adj.valueNum = b->value_num;
  g_adj.numSorted = g_numSorted.data();
  g_adj.numSortedId = g_numSortedId.data();
  g_adj.nNumSorted = static_cast<uint32_t>(g_numSorted.size());
  g_adj.valueBase = b->doc_value_base;
  g_adj.numSortedOffs = b->doc_value_base != nullptr ? g_numSortedOffs.data() : nullptr;
  g_adj.nums = g_nums.data();
  g_adj.numCount = g_numCount.data();
  g_adj.pm = g_pm.data();
  return &g_adj;
}
// emu_huge_replay_hi: the per-leaf output of remove clients 64..253 (kHiOutWords words per leaf) for the
// next replay (or nullptr)
uint64_t* g_hiOut = nullptr;
// emu_huge_resume: the large tier's checkpoint record and result slabs for the next replay (or nullptr)
const uint32_t* g_ck = nullptr;
const fmt_mt_leaf* g_ckLeaves = nullptr;
const uint16_t* g_ckChars = nullptr;
const fmt_mt_propset* g_ckProps = nullptr;
uint64_t g_resumedAt = 0;
// emu_huge_resume_adj: the large tier's PropertiesManager records and computed numbers of the document
// (in the runtime the huge tier reads the same HBM slabs; the two emulators keep their own)
const uint32_t* g_seedPm = nullptr;
uint32_t g_seedPmRecs = 0;
const double* g_seedNums = nullptr;
uint32_t g_seedNumN = 0;
}  // namespace

extern "C" {

// Replays document d of the batch (a summary-loaded document, header chunk only) into the caller's
// output arrays (fmt_mt_fetch_doc layout). Returns the document status.
// A document that does not start from a summary starts from its initial text (one segment stamped
// {0, FMT_LOCAL_CLIENT}) or empty, as the runtime replays documents that outgrow the large tier.
// With catchup != nullptr the catch-up ranges of FMT_MT_F_CATCHUP ops go there (capCatchup ranges).
// With an annotate-adjust batch, legacy (one entry per output leaf) receives the getAtSeq(minSeq) prop
// sets and nums / *nNums the document's computed numbers.
int emu_huge_replay_adj(const fmt_mt_batch* b, uint32_t d, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves, uint64_t capLeaves,
                        uint16_t* chars, uint64_t capChars, fmt_mt_propset* props, fmt_mt_catchup_range* catchup,
                        uint32_t capCatchup, fmt_mt_remove_order* rmOrder, uint32_t capRm, uint16_t* legacy, double* nums,
                        uint32_t capNums, uint32_t* nNums) {
  const bool loaded = b->snapshots != nullptr && b->snapshots[d].loaded;
  fmt_mt_snapshot_doc sd{};
  fmt_mt_snapshot_seg initSeg{};
  if (loaded) sd = b->snapshots[d];
  else if (b->doc_init != nullptr && b->doc_init[2 * d + 1] > 0) {
    initSeg = {b->doc_init[2 * d], b->doc_init[2 * d + 1], FMT_MT_NO_PROPS};
    sd.n_header = 1;
  }
  const uint64_t nOps = b->doc_op_offsets[d + 1] - b->doc_op_offsets[d];
  const uint32_t N = sd.n_header + (loaded ? sd.n_body : 0);
  std::vector<uint32_t> shape;  // (runtime.cpp setupHugeDoc)
  uint64_t shapeBlocks = 0;
  if (loaded && sd.n_body > 0) {
    loadShape(sd.n_header, sd.n_body, shape);
    for (uint32_t l = 0; l < shape[0]; l++) shapeBlocks += shape[1 + l];
  }
  bool segProps = false;
  if (loaded)
    for (uint64_t k = sd.first_seg; k < sd.first_seg + N; k++) segProps = segProps || b->snapshot_segs[k].props != FMT_MT_NO_PROPS;
  HugeState S{};
  S.blockCap = static_cast<uint32_t>(shapeBlocks + 2 * (N / 7 + 1) + 2 * nOps + 1024);
  S.idCap = static_cast<uint32_t>(N + 3 * nOps + 16);
  S.winCap = S.idCap;  // every leaf can be in the window (wide removes)
  uint64_t docChars = initSeg.len;  // (runtime.cpp setupHugeDoc; the snapshot's text counts below)
  for (uint64_t i = b->doc_op_offsets[d]; i < b->doc_op_offsets[d + 1]; i++)
    if (b->ops[i].type == FMT_MT_INSERT) docChars += fmt_mt_op_len(&b->ops[i]);
  if (loaded)
    for (uint64_t k = sd.first_seg; k < sd.first_seg + N; k++) docChars += b->snapshot_segs[k].len & ~FMT_MT_SEG_MARKER;
  uint64_t textCap = b->text_len + std::max<uint64_t>((loaded ? 256 : 1024) * nOps + 65536, 4 * docChars + 131072);
  if (const char* e = std::getenv("FMT_EMU_TEXTCAP")) textCap = std::strtoull(e, nullptr, 10);
  // (device buffers start with arbitrary contents: hipMalloc, no memset, runtime.cpp setupHugeDoc; so the
  // emulated ones start poisoned, and a read of a never-written slot shows as a wild value here too)
  constexpr uint32_t kPoison = 0xCDCDCDCDu;
  std::vector<uint32_t> u32(static_cast<size_t>(S.blockCap) * 8 * 6, kPoison);
  std::vector<int32_t> i32(static_cast<size_t>(S.blockCap) * 8 * 2, static_cast<int32_t>(kPoison));
  size_t o = 0, oi = 0;
  auto U = [&](size_t n) { uint32_t* p = u32.data() + o; o += n; return p; };
  auto I = [&](size_t n) { int32_t* p = i32.data() + oi; oi += n; return p; };
  const size_t nl = static_cast<size_t>(S.blockCap) * 8;
  S.lLen = U(nl); S.lMlo = U(nl); S.lMhi = U(nl); S.lId = U(nl); S.lText = U(nl); S.lMeta = U(nl);
  S.lIns = I(nl); S.lRm = I(nl);
  std::vector<uint32_t> blk(static_cast<size_t>(S.blockCap) * 14, kPoison);
  std::vector<int32_t> bsc(S.blockCap, static_cast<int32_t>(kPoison));
  S.bCount = blk.data(); S.bParent = S.bCount + S.blockCap; S.bLeaf = S.bParent + S.blockCap;
  S.bChild = S.bLeaf + S.blockCap; S.bGroup = S.bChild + 8ull * S.blockCap; S.bSlot = S.bGroup + S.blockCap;
  S.freeBlk = S.bSlot + S.blockCap; S.bScour = bsc.data();
  std::vector<uint32_t> gsb(static_cast<size_t>(kGroupCap) * kSlotCap, kPoison);
  std::vector<int32_t> gss(static_cast<size_t>(kGroupCap) * kSlotCap, static_cast<int32_t>(kPoison));
  S.gSlotBlk = gsb.data(); S.gSlotStable = gss.data();
  std::vector<uint32_t> ids(2ull * S.idCap, kPoison);
  S.leafBlk = ids.data(); S.winIdx = ids.data() + S.idCap;
  std::vector<uint32_t> wu(8ull * S.winCap, kPoison);
  S.wRec = wu.data(); S.wMask = S.wRec + 4ull * S.winCap; S.wBlk = S.wMask + 2ull * S.winCap; S.wLeaf = S.wBlk + S.winCap;
  // the merge area only: the batch text is read in place (runtime.cpp setupHugeDoc)
  std::vector<uint16_t> text(textCap - b->text_len);
  S.base = b->text;
  S.text = text.data() - b->text_len; S.textLen = b->text_len; S.textCap = textCap;
  std::vector<uint32_t> pr(static_cast<size_t>(kPropCap) * kPropWords);
  S.props = pr.data();
  std::vector<uint32_t> pcl(kPropCap), phead(2ull * kPropHash), pnext(2ull * kPropCap);
  S.pClass = pcl.data();
  S.pHead = phead.data();
  S.pNext = pnext.data();
  std::vector<uint32_t> cuIds(catchup != nullptr ? S.idCap : 0);
  S.cuIds = catchup != nullptr ? cuIds.data() : nullptr;
  std::vector<uint32_t> rmIds(rmOrder != nullptr ? S.idCap : 0);
  S.rmIds = rmOrder != nullptr ? rmIds.data() : nullptr;
  bool obl = false;  // (runtime.cpp: the live-obliterate table of batches with obliterates)
  for (uint64_t i = 0; i < b->n_ops && !obl; i++) obl = b->ops[i].type == FMT_MT_OBLITERATE || b->ops[i].type == FMT_MT_OBLITERATE_SIDED;
  const uint64_t obCap = std::max<uint64_t>(nOps, fmt_ckpt::kObSlots);  // (runtime.cpp setupHugeDoc)
  std::vector<uint32_t> obTab(obl ? 9ull * obCap : 0, 0xCDCDCDCDu);
  S.obCap = obl ? static_cast<uint32_t>(obCap) : 0u;
  S.obRec = obl ? obTab.data() : nullptr;
  S.obUsed = obl ? obTab.data() + 6ull * obCap : nullptr;
  S.obSeq = obl ? S.obUsed + obCap : nullptr;
  S.obStart = obl ? S.obSeq + obCap : nullptr;
  std::vector<uint32_t> hiMask(g_hiOut != nullptr ? static_cast<size_t>(kHiWords) * S.idCap : 0, 0u);  // (runtime.cpp: zeroed)
  S.hiMask = g_hiOut != nullptr ? hiMask.data() : nullptr;
  auto lds = std::make_unique<HugeLds>();
  std::memset(lds.get(), 0xCD, sizeof(HugeLds));
  const fmt_mt::AdjustTables* adj = prepareNumbers(b);
  if (adj != nullptr && g_seedPm != nullptr) {
    std::copy(g_seedPm, g_seedPm + 4ull * std::min(g_seedPmRecs, kEmuPmCap), g_pm.begin());
    std::copy(g_seedNums, g_seedNums + std::min(g_seedNumN, kEmuNumCap), g_nums.begin());
    g_numCount[d] = std::min(g_seedNumN, kEmuNumCap);
  }
  auto replay = [&](auto* doc) {  // (HugeDocT<true> for annotate-adjust batches, as the runtime launches)
  doc->S = S;
  doc->L = lds.get();
  HugeInputs in;
  in.ops = b->ops;
  in.begin = b->doc_op_offsets[d];
  in.end = b->doc_op_offsets[d + 1];
  in.propsOff = b->props_off;
  in.propsKv = b->props_kv;
  in.nPropsOps = b->n_props_ops;
  in.segs = loaded ? b->snapshot_segs + sd.first_seg : &initSeg;
  in.nSegs = N;
  in.shape = shape.empty() ? nullptr : shape.data();
  in.segProps = segProps ? 1u : 0u;
  in.info = loaded && b->snapshot_info != nullptr ? b->snapshot_info + sd.first_seg : nullptr;
  in.stamps = b->snapshot_stamps;
  in.infoAll = b->snapshot_info;
  in.nInfoAll = b->snapshot_info != nullptr ? b->n_snapshot_segs : 0;
  in.catchup = catchup;
  in.catchupCap = capCatchup;
  in.rmOrder = rmOrder;
  in.rmOrderCap = capRm;
  in.relpos = b->relpos;
  in.nRelpos = b->relpos ? b->n_relpos : 0;
  in.markerKey = b->marker_id_key;
  std::vector<uint32_t> mkIds(b->relpos != nullptr ? S.idCap : 0);
  doc->S.mkIds = b->relpos != nullptr ? mkIds.data() : nullptr;
  doc->S.mkCap = S.idCap;
  std::vector<uint64_t> numOffs(b->n_docs + 1ull, kEmuNumCap), pmOffs(b->n_docs + 1ull, kEmuPmCap);
  for (uint32_t k = 0; k <= d && k <= b->n_docs; k++) numOffs[k] = pmOffs[k] = 0;  // (document d: [0, cap))
  g_adj.numOffsets = numOffs.data();
  g_adj.pmOffsets = pmOffs.data();
  in.adj = adj;
  in.doc = d;
  std::vector<uint32_t> outIdx(adj != nullptr ? S.idCap : 0);
  doc->S.outIdx = adj != nullptr ? outIdx.data() : nullptr;
  in.snapMinSeq = sd.min_seq;
  in.snapSeq = sd.seq;
  in.initClient = loaded ? FMT_NON_COLLAB_CLIENT : FMT_LOCAL_CLIENT;
  in.ck = g_ck;
  in.ckLeaves = g_ckLeaves;
  in.ckChars = g_ckChars;
  in.ckProps = g_ckProps;
  doc->run(in);
  g_resumedAt = doc->prof[24];
  doc->writeOutputs(hdr, leaves, capLeaves, chars, capChars, props, adj != nullptr ? legacy : nullptr, g_hiOut);
  if (nNums) *nNums = adj != nullptr ? g_numCount[d] : 0u;
  for (uint32_t k = 0; adj != nullptr && nums != nullptr && k < g_numCount[d] && k < capNums; k++) nums[k] = g_nums[k];
  if (std::getenv("FMT_EMU_TEXTCAP"))
    std::fprintf(stderr, "textTop %llu of %llu, compactions %llu\n", (unsigned long long)doc->textTop, (unsigned long long)textCap,
                 (unsigned long long)doc->prof[22]);
  };
  const bool rm = rmOrder != nullptr;  // (the runtime launches the Rm variant for batches that record)
  if (adj != nullptr && rm) replay(std::make_unique<HugeDocT<true, true>>().get());
  else if (adj != nullptr) replay(std::make_unique<HugeDocT<true, false>>().get());
  else if (rm) replay(std::make_unique<HugeDocT<false, true>>().get());
  else replay(std::make_unique<HugeDocT<false, false>>().get());
  return hdr->status;
}

int emu_huge_replay_rec(const fmt_mt_batch* b, uint32_t d, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves, uint64_t capLeaves,
                        uint16_t* chars, uint64_t capChars, fmt_mt_propset* props, fmt_mt_catchup_range* catchup,
                        uint32_t capCatchup, fmt_mt_remove_order* rmOrder, uint32_t capRm) {
  return emu_huge_replay_adj(b, d, hdr, leaves, capLeaves, chars, capChars, props, catchup, capCatchup, rmOrder, capRm,
                             nullptr, nullptr, 0, nullptr);
}

int emu_huge_replay(const fmt_mt_batch* b, uint32_t d, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves, uint64_t capLeaves,
                    uint16_t* chars, uint64_t capChars, fmt_mt_propset* props) {
  return emu_huge_replay_rec(b, d, hdr, leaves, capLeaves, chars, capChars, props, nullptr, 0, nullptr, 0);
}

// Document d resumed in the huge tier from the large tier's checkpoint (emu_mt_replay_large_ckpt: its
// record ck and its result slabs at large strides, leaves / chars / props of document d). Returns the
// status; *resumedAt = the op index within the document it resumed at.
int emu_huge_resume(const fmt_mt_batch* b, uint32_t d, const uint32_t* ck, const fmt_mt_leaf* ckLeaves,
                    const uint16_t* ckChars, const fmt_mt_propset* ckProps, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves,
                    uint64_t capLeaves, uint16_t* chars, uint64_t capChars, fmt_mt_propset* props,
                    fmt_mt_catchup_range* catchup, uint32_t capCatchup, uint64_t* resumedAt) {
  g_ck = ck;
  g_ckLeaves = ckLeaves;
  g_ckChars = ckChars;
  g_ckProps = ckProps;
  g_resumedAt = 0;
  const int st = emu_huge_replay_rec(b, d, hdr, leaves, capLeaves, chars, capChars, props, catchup, capCatchup, nullptr, 0);
  g_ck = nullptr;
  g_ckLeaves = nullptr;
  g_ckChars = nullptr;
  g_ckProps = nullptr;
  if (resumedAt) *resumedAt = g_resumedAt;
  return st;
}

// emu_huge_resume for a batch with remove-order recording: rmOrder[capRm] holds the document's entries
// as the large tier left them (leaf ids; the count is in the record) and receives the final ones.
int emu_huge_resume_rm(const fmt_mt_batch* b, uint32_t d, const uint32_t* ck, const fmt_mt_leaf* ckLeaves,
                       const uint16_t* ckChars, const fmt_mt_propset* ckProps, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves,
                       uint64_t capLeaves, uint16_t* chars, uint64_t capChars, fmt_mt_propset* props,
                       fmt_mt_remove_order* rmOrder, uint32_t capRm, uint64_t* resumedAt) {
  g_ck = ck;
  g_ckLeaves = ckLeaves;
  g_ckChars = ckChars;
  g_ckProps = ckProps;
  g_resumedAt = 0;
  const int st = emu_huge_replay_rec(b, d, hdr, leaves, capLeaves, chars, capChars, props, nullptr, 0, rmOrder, capRm);
  g_ck = nullptr;
  g_ckLeaves = nullptr;
  g_ckChars = nullptr;
  g_ckProps = nullptr;
  if (resumedAt) *resumedAt = g_resumedAt;
  return st;
}

// emu_huge_resume for an annotate-adjust batch: pm (pmRecs records) and nums (nNumsIn) are the
// document's slabs as the large tier left them (emu_mt_adj_slab); legacy / nums / *nNums as
// emu_huge_replay_adj.
int emu_huge_resume_adj(const fmt_mt_batch* b, uint32_t d, const uint32_t* ck, const fmt_mt_leaf* ckLeaves,
                        const uint16_t* ckChars, const fmt_mt_propset* ckProps, const uint32_t* pm, uint32_t pmRecs,
                        const double* numsIn, uint32_t nNumsIn, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves,
                        uint64_t capLeaves, uint16_t* chars, uint64_t capChars, fmt_mt_propset* props, uint16_t* legacy,
                        double* nums, uint32_t capNums, uint32_t* nNums, uint64_t* resumedAt) {
  g_ck = ck;
  g_ckLeaves = ckLeaves;
  g_ckChars = ckChars;
  g_ckProps = ckProps;
  g_seedPm = pm;
  g_seedPmRecs = pmRecs;
  g_seedNums = numsIn;
  g_seedNumN = nNumsIn;
  g_resumedAt = 0;
  const int st = emu_huge_replay_adj(b, d, hdr, leaves, capLeaves, chars, capChars, props, nullptr, 0, nullptr, 0, legacy,
                                     nums, capNums, nNums);
  g_ck = nullptr;
  g_ckLeaves = nullptr;
  g_ckChars = nullptr;
  g_ckProps = nullptr;
  g_seedPm = nullptr;
  g_seedNums = nullptr;
  if (resumedAt) *resumedAt = g_resumedAt;
  return st;
}

// As emu_huge_replay, with the remove-client side table for short ids 64..253 (the runtime allocates
// it for batches that name such clients): hi[capLeaves x kHiOutWords] receives each leaf's ids 64..127,
// 128..191 and 192..253.
int emu_huge_replay_hi(const fmt_mt_batch* b, uint32_t d, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves, uint64_t capLeaves,
                       uint16_t* chars, uint64_t capChars, fmt_mt_propset* props, uint64_t* hi) {
  g_hiOut = hi;
  const int st = emu_huge_replay_rec(b, d, hdr, leaves, capLeaves, chars, capChars, props, nullptr, 0, nullptr, 0);
  g_hiOut = nullptr;
  return st;
}

}  // extern "C"
