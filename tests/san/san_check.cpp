// san_check.cpp — TEST INFRASTRUCTURE ONLY (sanitizer counterpart): the oracle and the
// merge-tree engine source under host emulation (tests/emu/mt_emu.cpp), built with
// -fsanitize=address,undefined, replay generated conflict farms; every document's header must
// agree. Any out-of-bounds access, use-after-free or undefined behaviour in either aborts the run.
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/fmt.h"

extern "C" {
void* fmtgen_conflict_farm_new(uint32_t n_docs, uint32_t n_clients, uint32_t ops_per_doc, uint32_t min_length_fixed,
                               uint32_t seed, uint32_t annotate_props_base, uint32_t threads, uint64_t* n_ops,
                               uint64_t* n_text, uint32_t doc_base);
int fmtgen_conflict_farm_copy(void* handle, uint32_t replicas, fmt_mt_op* out_ops, uint64_t* out_offsets,
                              uint16_t* out_text, uint32_t threads);
void fmtgen_free(void* handle);
int orc_mt_replay_batch(const fmt_mt_batch* b, uint32_t docBegin, uint32_t docEnd, uint32_t nThreads,
                        fmt_mt_doc_result* hdrs, fmt_mt_leaf* leaves, uint32_t capLeaves, uint16_t* chars,
                        uint32_t capChars, fmt_mt_propset* props, uint32_t capProps, fmt_mt_catchup_range* catchup,
                        uint32_t capCatchup, double* seconds, double* nums, uint32_t capNums, uint32_t* nNums);
int emu_mt_capacity(int large, uint32_t* leaves, uint32_t* chars, uint32_t* props);
int emu_mt_replay(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                  fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup, int forceOb, int large,
                  fmt_mt_remove_order* rmOrder, uint32_t capRm);
}

// adjust: every annotate is an annotate-adjust of key 0 (four rows: plain, clamped, null max) over
// values that are numbers ("1".."64"): the Adj engine variants and the oracle's computePropertyValue.
static int run(uint32_t nDocs, uint32_t clients, uint32_t ops, uint32_t minLength, uint32_t seed, int tier,
               bool adjust = false) {
  uint64_t nOps = 0, nText = 0;
  void* g = fmtgen_conflict_farm_new(nDocs, clients, ops, minLength, seed, 0, 1, &nOps, &nText, 0);
  std::vector<fmt_mt_op> o(nOps);
  std::vector<uint64_t> offs(nDocs + 1);
  std::vector<uint16_t> text(nText + 1);
  fmtgen_conflict_farm_copy(g, 1, o.data(), offs.data(), text.data(), 1);
  fmtgen_free(g);
  // props op i = {"client": i}: one (key 0, value i + 1) pair each (workloads.conflict_farm's table)
  std::vector<uint32_t> propsOff(65), propsKv(adjust ? 128 : 64);
  for (uint32_t i = 0; i < 64; i++) {
    propsOff[i + 1] = adjust ? 2 * (i + 1) : i + 1;
    if (adjust) {
      propsKv[2 * i] = FMT_MT_VALUE_ADJUST;
      propsKv[2 * i + 1] = i % 4;
    } else {
      propsKv[i] = i + 1;
    }
  }
  const fmt_mt_adjust rows[4] = {{1.0, 0, 0, 0, 0}, {0.5, -1.0, 2.0, FMT_MT_ADJ_MIN | FMT_MT_ADJ_MAX, 0},
                                 {-0.25, 0, 0, FMT_MT_ADJ_MAX | FMT_MT_ADJ_MAX_NULL, 0}, {3.0, 0, 4.0, FMT_MT_ADJ_MAX, 0}};
  std::vector<double> valueNum(65);
  for (uint32_t i = 0; i < 65; i++) valueNum[i] = i == 0 ? __builtin_nan("") : double(i);
  fmt_mt_batch b;
  std::memset(&b, 0, sizeof b);
  b.ops = o.data();
  b.n_ops = nOps;
  b.doc_op_offsets = offs.data();
  b.n_docs = nDocs;
  b.text = text.data();
  b.text_len = nText;
  b.props_off = propsOff.data();
  b.n_props_ops = 64;
  b.props_kv = propsKv.data();
  b.marker_id_key = FMT_MT_NO_MARKER;
  if (adjust) {
    b.adjusts = rows;
    b.n_adjusts = 4;
    b.value_num = valueNum.data();
    b.n_values = 65;
  }
  uint32_t cl, cc, cp;
  emu_mt_capacity(tier, &cl, &cc, &cp);
  std::vector<fmt_mt_doc_result> oh(nDocs), eh(nDocs);
  std::vector<fmt_mt_leaf> ol(size_t(nDocs) * cl), el(size_t(nDocs) * cl);
  std::vector<uint16_t> oc(size_t(nDocs) * cc), ec(size_t(nDocs) * cc);
  std::vector<fmt_mt_propset> op(size_t(nDocs) * cp), ep(size_t(nDocs) * cp);
  orc_mt_replay_batch(&b, 0, nDocs, 1, oh.data(), ol.data(), cl, oc.data(), cc, op.data(), cp, nullptr, 0, nullptr,
                      nullptr, 0, nullptr);
  emu_mt_replay(&b, eh.data(), el.data(), ec.data(), ep.data(), nullptr, 0, 0, tier, nullptr, 0);
  int bad = 0;
  for (uint32_t d = 0; d < nDocs; d++) {
    if (eh[d].status == FMT_E_CAPACITY) continue;  // beyond this tier (the runtime escalates it)
    bool same = oh[d].status == eh[d].status && oh[d].n_leaves == eh[d].n_leaves &&
                oh[d].n_chars == eh[d].n_chars && oh[d].visible_len == eh[d].visible_len &&
                oh[d].min_seq == eh[d].min_seq && oh[d].n_blocks == eh[d].n_blocks && oh[d].depth == eh[d].depth;
    for (uint32_t j = 0; same && j < eh[d].n_leaves; j++) {  // the fields tests/mt_compare.py compares
      const fmt_mt_leaf &a = ol[size_t(d) * cl + j], &e = el[size_t(d) * cl + j];
      same = a.ins_seq == e.ins_seq && a.rm_seq == e.rm_seq && a.rm_clients == e.rm_clients && a.char_off == e.char_off &&
             a.len == e.len && a.ins_client == e.ins_client && a.block == e.block && a.pad == e.pad;
    }
    if (!same) {
      std::fprintf(stderr, "tier %d clients %u minLength %u doc %u differs (status %d/%d leaves %u/%u)\n", tier,
                   clients, minLength, d, oh[d].status, eh[d].status, oh[d].n_leaves, eh[d].n_leaves);
      bad++;
    }
  }
  std::printf("tier %d: %u docs x %u ops, %u clients, minLength %u: %d mismatches\n", tier, nDocs, ops, clients,
              minLength, bad);
  return bad;
}

int main() {
  int bad = 0;
  bad += run(24, 8, 1500, 0, 3, 0);      // small tier
  bad += run(24, 8, 1500, 0, 4, 3);      // compact → small with checkpoints
  bad += run(16, 8, 2000, 3000, 5, 4);   // compact → small → large, long texts
  bad += run(12, 40, 1200, 0, 6, 4);     // 40 writers: the small tier hands over to the large tier
  bad += run(8, 8, 1500, 0, 7, 1);       // large tier alone
  bad += run(12, 8, 1500, 0, 8, 0, true);   // annotate-adjust, small tier
  bad += run(12, 8, 1500, 0, 9, 4, true);   // annotate-adjust, small → large restart
  return bad == 0 ? 0 : 1;
}
