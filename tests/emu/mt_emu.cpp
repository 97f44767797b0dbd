// mt_emu.cpp — TEST INFRASTRUCTURE ONLY: the merge-tree engine source (mt_engine.h) compiled for the
// host with the 64-lane emulation of wave.h, so the CPU parity suite can check the exact kernel
// logic against the oracle without a GPU. Never loaded by the product (libfmt.so has no CPU path).
#include <cstring>
#include <memory>

#include "../../fluidframework_amd/csrc/mt_engine.h"

template <bool Ob, class C, bool Rm = false>
static int replayAll(const fmt_mt_batch* b, fmt_mt_doc_result* headers, fmt_mt_leaf* leaves, uint16_t* chars,
                     fmt_mt_propset* props, fmt_mt_catchup_range* catchup, uint32_t capCatchup,
                     fmt_mt_remove_order* rmOrder, uint32_t capRm) {
  using Doc = fmt_mt::Doc<Ob, C, Rm>;
  auto scratch = std::make_unique<fmt_mt::Scratch<C>>();
  auto doc = std::make_unique<Doc>();
  int status = FMT_OK;
  for (uint32_t d = 0; d < b->n_docs; d++) {
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
    if (b->snapshots && b->snapshots[d].loaded) {
      const fmt_mt_snapshot_doc sd = b->snapshots[d];
      in.snapSegs = b->snapshot_segs + sd.first_seg;
      in.nHeader = sd.n_header;
      in.nBody = sd.n_body;
      in.snapMinSeq = sd.min_seq;
      in.snapSeq = sd.seq;
      in.loaded = 1;
    } else {
      in.snapSegs = nullptr;
      in.nHeader = in.nBody = 0;
      in.snapMinSeq = in.snapSeq = 0;
      in.loaded = 0;
    }
    fmt_mt::DocOutputs o;
    o.header = headers + d;
    o.leaves = leaves + static_cast<size_t>(d) * Doc::kCapLeaves;
    o.chars = chars + static_cast<size_t>(d) * Doc::kCapChars;
    o.props = props + static_cast<size_t>(d) * Doc::kPropCap;
    o.catchup = catchup ? catchup + static_cast<size_t>(d) * capCatchup : nullptr;
    o.catchupCap = catchup ? capCatchup : 0u;
    o.rmOrder = rmOrder ? rmOrder + static_cast<size_t>(d) * capRm : nullptr;
    o.rmOrderCap = rmOrder ? capRm : 0u;
    new (doc.get()) Doc();
    doc->s = scratch.get();
    doc->run(in, o);
    if (headers[d].status == fmt_mt::kCapacityFinal) headers[d].status = FMT_E_CAPACITY;  // as collectOverflowKernel
    if (headers[d].status != FMT_OK && status == FMT_OK) status = headers[d].status;
  }
  return status;
}

extern "C" {

// large = 0: the small tier (registers + LDS text); 1: the large tier (HBM text) that the runtime
// replays overflowing documents in; 2: the compact tier (4 register rows) plain batches start in.
int emu_mt_capacity(int large, uint32_t* leaves, uint32_t* chars, uint32_t* props) {
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
  bool ob = forceOb != 0;
  for (uint64_t i = 0; i < b->n_ops && !ob; i++) ob = b->ops[i].type == FMT_MT_OBLITERATE || b->ops[i].type == FMT_MT_OBLITERATE_SIDED;
  using S = fmt_mt::SmallTier;
  using G = fmt_mt::LargeTier;
  bool rm = false;
  for (uint64_t i = 0; i < b->n_ops && !rm; i++) rm = (b->ops[i].flags & FMT_MT_F_RMORDER) != 0;
  if (large == 2 && !ob && !rm) return replayAll<false, fmt_mt::CompactTier>(b, headers, leaves, chars, props, catchup,
                                                                             capCatchup, rmOrder, capRm);
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

}  // extern "C"
