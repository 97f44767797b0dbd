// oracle/capi.cpp — TEST INFRASTRUCTURE ONLY: extern "C" surface of the parity oracle for ctypes.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
// Result layouts are the product's (include/fmt.h) so tests compare GPU and oracle field by field.
#include <deque>
#include <algorithm>
#include <atomic>
#include <cmath>
#include <memory>
#include <mutex>
#include <chrono>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "map.hpp"
#include "mergetree.hpp"

using orc::MergeTree;

namespace {

thread_local std::string g_err;

int fail(const char* what) {
  g_err = what;
  return FMT_E_DATA;
}

// Applies ops[0..n): a record flagged FMT_MT_F_GROUP_CONT continues the previous message.
// f4 (FMT_MT_F_LOCAL / ACK / ROLLBACK / REGEN): the local client's events; REGEN appends its new ops
// (and their insert text) to *regen / *regenText.
int applyOps(MergeTree* mt, const fmt_mt_op* ops, uint64_t n, const uint16_t* arena,
             const uint32_t* propsOff, const uint32_t* propsKv, int32_t* failSeq,
             std::vector<fmt_mt_catchup_range>* catchup = nullptr, std::vector<fmt_mt_op>* regen = nullptr,
             std::u16string* regenText = nullptr) {
  for (uint64_t i = 0; i < n; i++) {
    const fmt_mt_op& op = ops[i];
    try {
      if (op.flags & (FMT_MT_F_LOCAL | FMT_MT_F_ROLLBACK | FMT_MT_F_REGEN)) {  // no collab-window update
        if (op.flags & FMT_MT_F_LOCAL) mt->applyLocal(op, arena, propsOff, propsKv);
        else if (op.flags & FMT_MT_F_ROLLBACK) mt->rollback(op);
        else mt->regeneratePending(regen ? regen : &mt->regenOps, regenText ? regenText : &mt->regenText);
        continue;
      }
      mt->catchupOut = (catchup && (op.flags & FMT_MT_F_CATCHUP)) ? catchup : nullptr;
      mt->catchupOp = static_cast<uint32_t>(i);
      if (op.flags & FMT_MT_F_ACK) mt->ackOp(op, propsOff, propsKv);
      else mt->applyRemote(op, arena, propsOff, propsKv);
      mt->catchupOut = nullptr;
      // (loader segments: no collab-window update; a batch of them is not a GROUP message)
      if ((op.flags & FMT_MT_F_LOADSEG) == 0 &&
          (i + 1 == n || (ops[i + 1].flags & (FMT_MT_F_GROUP_CONT | FMT_MT_F_LOADSEG)) != FMT_MT_F_GROUP_CONT))
        mt->updateSeqNumbers(std::min(op.min_seq, mt->minInflightRef()), op.seq);
    } catch (const orc::UsageError& e) {
      if (failSeq) *failSeq = op.seq;
      fail(e.what());
      return FMT_E_USAGE;
    } catch (const std::exception& e) {
      if (failSeq) *failSeq = op.seq;
      return fail(e.what());
    }
  }
  return FMT_OK;
}

// rmHi (optional): per leaf, its remove clients with short ids 64..253 as three words (64..127, 128..191,
// 192..253: fmt_mt_fetch_rm_clients_hi / _hi2).
void dumpDoc(const MergeTree* mt, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves, uint32_t capLeaves,
             uint16_t* chars, uint32_t capChars, fmt_mt_propset* props, uint32_t capProps,
             std::vector<uint64_t>* rmHi = nullptr) {
  std::vector<const orc::Seg*> segs;
  std::vector<int> blockOf;
  int nBlocks = 0, depth = 0;
  mt->collectLeaves(segs, blockOf, &nBlocks, &depth);
  if (rmHi) rmHi->assign(3 * segs.size(), 0);
  std::vector<const orc::PropMap*> sets;
  std::vector<uint32_t> setRec;  // first record of each set (a set wider than 8 entries takes several)
  uint32_t nRec = 0;
  uint32_t charOff = 0;
  for (size_t i = 0; i < segs.size(); i++) {
    const orc::Seg* s = segs[i];
    uint16_t pid = 0xffff;
    if (s->props.defined) {
      size_t j = 0;
      for (; j < sets.size(); j++)
        if (sets[j]->kv == s->props.kv) break;
      if (j == sets.size()) {
        sets.push_back(&s->props);
        setRec.push_back(nRec);
        const size_t n = s->props.kv.size();
        nRec += n > FMT_MT_PROPS_MAX ? static_cast<uint32_t>((n + FMT_MT_PROPS_MAX - 1) / FMT_MT_PROPS_MAX) : 1u;
      }
      pid = static_cast<uint16_t>(setRec[j]);
    }
    if (leaves && i < capLeaves) {
      fmt_mt_leaf& L = leaves[i];
      std::memset(&L, 0, sizeof(L));
      // (a stamp pending its ack: FMT_MT_LOCAL_SEQ_BASE | localSeq, the engine's encoding)
      auto seqOf = [](const orc::Stamp& st) { return orc::isLocal(st) ? FMT_MT_LOCAL_SEQ_BASE | st.localSeq : st.seq; };
      L.ins_seq = seqOf(s->ins);
      L.ins_client = static_cast<int16_t>(s->ins.client);
      L.rm_seq = s->removed() ? seqOf(s->removes[0]) : FMT_NOT_REMOVED;
      uint64_t mask = 0;
      for (const auto& r : s->removes) {
        if (r.client >= 0 && r.client < 64) mask |= 1ull << r.client;
        else if (r.client >= 64 && r.client < 256 && rmHi) (*rmHi)[3 * i + (r.client - 64) / 64] |= 1ull << ((r.client - 64) % 64);
      }
      L.rm_clients = mask;
      L.char_off = charOff;
      L.len = static_cast<uint32_t>(s->len());
      L.props = pid;
      L.block = static_cast<uint16_t>(blockOf[i]);
      L.pad = static_cast<uint16_t>((static_cast<uint32_t>(blockOf[i]) >> 16) | (s->marker ? FMT_MT_LEAF_MARKER : 0u));
    }
    for (int k = 0; k < s->len(); k++) {
      if (chars && charOff + k < capChars) chars[charOff + k] = static_cast<uint16_t>(s->text[k]);
    }
    charOff += static_cast<uint32_t>(s->len());
  }
  if (props) {
    for (size_t j = 0; j < sets.size(); j++) {
      const size_t n = sets[j]->kv.size();
      const size_t rec = n > FMT_MT_PROPS_MAX ? (n + FMT_MT_PROPS_MAX - 1) / FMT_MT_PROPS_MAX : 1;
      for (size_t q = 0; q < rec && setRec[j] + q < capProps; q++) {
        fmt_mt_propset& P = props[setRec[j] + q];
        std::memset(&P, 0, sizeof(P));
        P.n = q == 0 ? static_cast<uint32_t>(n) : FMT_MT_PROPS_CONT;
        for (size_t k = 0; k < FMT_MT_PROPS_MAX && q * FMT_MT_PROPS_MAX + k < n; k++) {
          const auto& e = sets[j]->kv[q * FMT_MT_PROPS_MAX + k];
          P.kv[k] = (static_cast<uint32_t>(e.first) << 16) | e.second;
        }
      }
    }
  }
  if (hdr) {
    hdr->cur_seq = mt->currentSeq;
    hdr->min_seq = mt->minSeq;
    hdr->n_leaves = static_cast<uint32_t>(segs.size());
    hdr->n_chars = charOff;
    hdr->n_props = nRec;
    hdr->n_blocks = static_cast<uint32_t>(nBlocks);
    hdr->depth = static_cast<uint32_t>(depth);
    hdr->visible_len = static_cast<uint32_t>(mt->getLocalLength());
  }
}

// The state digest of DESIGN.md §2 (what fmt_mt_state_digest computes on the device), restated over
// the oracle's dumped state: mix(Σ elem(tag, index, word) mod 2^64), mix = the splitmix64 finalizer.
uint64_t dgMix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t dgElem(uint64_t tag, uint64_t i, uint64_t w) { return dgMix(dgMix((tag << 56) ^ i) ^ w); }

uint64_t digestOf(const fmt_mt_doc_result& h, const fmt_mt_leaf* leaves, const uint16_t* chars, const fmt_mt_propset* props,
                  const std::vector<uint64_t>* rmHi = nullptr) {
  uint64_t acc = 0;
  if (h.status != FMT_OK)
    return dgMix(dgElem(1, 0, static_cast<uint32_t>(h.status)) + dgElem(1, 1, static_cast<uint32_t>(h.fail_seq)));
  const uint32_t f[8] = {static_cast<uint32_t>(h.status), static_cast<uint32_t>(h.cur_seq), static_cast<uint32_t>(h.min_seq),
                         h.n_leaves, h.n_chars, h.n_blocks, h.depth, h.visible_len};
  for (uint32_t k = 0; k < 8; k++) acc += dgElem(1, k, f[k]);
  for (uint32_t i = 0; i < h.n_leaves; i++) {
    const fmt_mt_leaf& L = leaves[i];
    acc += dgElem(2, i, static_cast<uint32_t>(L.ins_seq) | static_cast<uint64_t>(static_cast<uint32_t>(L.rm_seq)) << 32);
    acc += dgElem(3, i, L.rm_clients);
    acc += dgElem(4, i, L.char_off | static_cast<uint64_t>(L.len) << 32);
    acc += dgElem(5, i, static_cast<uint16_t>(L.ins_client) | static_cast<uint64_t>(L.block) << 16 |
                            static_cast<uint64_t>(L.pad) << 32);
    if (L.props == 0xFFFFu) {
      acc += dgElem(6, i, ~0ull);
    } else {
      const fmt_mt_propset& P = props[L.props];
      acc += dgElem(6, i, P.n);
      for (uint32_t k = 0; k < P.n && k < FMT_MT_PROPS_KEYS_MAX && L.props + k / FMT_MT_PROPS_MAX < h.n_props; k++) {
        const uint32_t w = props[L.props + k / FMT_MT_PROPS_MAX].kv[k % FMT_MT_PROPS_MAX];
        acc += k < FMT_MT_PROPS_MAX ? dgElem(7, static_cast<uint64_t>(i) * 8 + k, w) : dgElem(9, static_cast<uint64_t>(i) * 64 + k, w);
      }
    }
  }
  if (rmHi)  // remove clients 64..127 / 128..191 / 192..253 (tags 10 / 11 / 12), on the leaves that have any
    for (uint32_t i = 0; i < h.n_leaves && 3 * i + 2 < rmHi->size(); i++)
      for (int k = 0; k < 3; k++)
        if ((*rmHi)[3 * i + k] != 0) acc += dgElem(10 + k, i, (*rmHi)[3 * i + k]);
  for (uint32_t u = 0; u < h.n_chars; u++) acc += dgElem(8, u, chars[u]);
  return dgMix(acc);
}

template <class F>
void parallelFor(uint32_t begin, uint32_t end, uint32_t nThreads, F&& fn) {
  if (nThreads <= 1 || end - begin <= 1) {
    for (uint32_t d = begin; d < end; d++) fn(d);
    return;
  }
  std::atomic<uint32_t> next{begin};
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < nThreads; t++) {
    pool.emplace_back([&] {
      for (uint32_t d = next.fetch_add(1); d < end; d = next.fetch_add(1)) fn(d);
    });
  }
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

const char* orc_last_error() { return g_err.c_str(); }

// ---------------------------------------------------------------- merge-tree, one document
void* orc_mt_new() { return new MergeTree(); }
void orc_mt_free(void* h) { delete static_cast<MergeTree*>(h); }

int orc_mt_insert_local(void* h, int pos, const uint16_t* text, int len) {
  try {
    static_cast<MergeTree*>(h)->insertLocal(pos, std::u16string(reinterpret_cast<const char16_t*>(text), len));
  } catch (const std::exception& e) {
    return fail(e.what());
  }
  return FMT_OK;
}

int orc_mt_annotate_local(void* h, int start, int end, const uint32_t* kv, int n) {
  std::vector<std::pair<uint16_t, uint16_t>> props;
  for (int i = 0; i < n; i++) props.emplace_back(kv[i] >> 16, kv[i] & 0xffff);
  try {
    static_cast<MergeTree*>(h)->annotateLocal(start, end, props);
  } catch (const std::exception& e) {
    return fail(e.what());
  }
  return FMT_OK;
}

int orc_mt_remove_local(void* h, int start, int end) {
  try {
    static_cast<MergeTree*>(h)->removeLocal(start, end);
  } catch (const std::exception& e) {
    return fail(e.what());
  }
  return FMT_OK;
}

int orc_mt_start_collab(void* h, int client) {
  static_cast<MergeTree*>(h)->startCollaboration(client, 0, 0);
  return FMT_OK;
}

int orc_mt_apply_ops(void* h, const fmt_mt_op* ops, uint64_t n, const uint16_t* arena,
                     const uint32_t* propsOff, const uint32_t* propsKv) {
  return applyOps(static_cast<MergeTree*>(h), ops, n, arena, propsOff, propsKv, nullptr);
}

// Annotate-adjust rows and the value numbers (NaN: not a number) for the ops applied next to the
// interactive document (batch-global value ids; computed numbers take ids of their own).
void orc_mt_set_adjusts(void* h, const fmt_mt_adjust* adjusts, uint32_t nAdjusts, const double* valueNum,
                        uint32_t nValues) {
  MergeTree* mt = static_cast<MergeTree*>(h);
  mt->adjusts = adjusts;
  mt->nAdjusts = nAdjusts;
  mt->valueNum = valueNum;
  mt->nValues = valueNum ? nValues : 0u;
}

// Legacy relative positions for the ops applied next to the interactive document: the batch's
// relpos table (fmt_mt_relpos rows) and the key id of "markerId".
void orc_mt_set_relpos(void* h, const fmt_mt_relpos* relpos, uint32_t n, uint32_t markerIdKey) {
  MergeTree* mt = static_cast<MergeTree*>(h);
  mt->relpos = relpos;
  mt->nRelpos = n;
  mt->markerIdKey = markerIdKey;
}

// 1 when a marker whose "markerId" is value id `id` is in the interactive document and not removed
// (getMarkerFromId, mergeTree.ts:1450-1453: a locally removed one counts as removed), else 0.
int orc_mt_marker_present(void* h, uint32_t id) {
  return static_cast<const MergeTree*>(h)->markerPresent(id) ? 1 : 0;
}

// Returns the text length; copies min(len, cap) UTF-16 units.
// f4: the local length (getLength, client.ts:1696) and the ops REGEN events produced since the last
// take (their insert text in `text`, payloads relative to it); *nOps / *nText are the full counts. With
// out and text both NULL only the counts are reported; otherwise the buffers are handed over and cleared.
int orc_mt_local_length(void* h) { return static_cast<MergeTree*>(h)->getLocalLength(); }
int orc_mt_pending_groups(void* h) { return static_cast<int>(static_cast<MergeTree*>(h)->pendingGroups()); }
int orc_mt_regen_take(void* h, fmt_mt_op* out, uint32_t cap, uint16_t* text, uint32_t textCap, uint32_t* nOps,
                      uint32_t* nText) {
  MergeTree* mt = static_cast<MergeTree*>(h);
  *nOps = static_cast<uint32_t>(mt->regenOps.size());
  *nText = static_cast<uint32_t>(mt->regenText.size());
  if (out == nullptr && text == nullptr) return FMT_OK;  // (counts only)
  for (uint32_t i = 0; i < *nOps && i < cap; i++) out[i] = mt->regenOps[i];
  for (uint32_t i = 0; i < *nText && i < textCap; i++) text[i] = static_cast<uint16_t>(mt->regenText[i]);
  mt->regenOps.clear();
  mt->regenText.clear();
  return FMT_OK;
}

int orc_mt_text(void* h, uint16_t* buf, int cap) {
  const std::u16string t = static_cast<MergeTree*>(h)->getText();
  for (int i = 0; i < static_cast<int>(t.size()) && i < cap; i++) buf[i] = static_cast<uint16_t>(t[i]);
  return static_cast<int>(t.size());
}

int orc_mt_dump(void* h, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves, uint32_t capLeaves,
                uint16_t* chars, uint32_t capChars, fmt_mt_propset* props, uint32_t capProps) {
  dumpDoc(static_cast<MergeTree*>(h), hdr, leaves, capLeaves, chars, capChars, props, capProps);
  return FMT_OK;
}

// Legacy summary blobs (header, then body); returns the byte count needed for header+body.
// (orc_mt_replay_summary: the same for document d of a batch after its replay)
int orc_mt_summary(void* h, const char* const* keys, int nKeys, const char* const* values,
                   int nValues, int chunkSize, char* out, int cap, int* headerLen, int* bodyLen) {
  std::vector<std::string> k(keys, keys + nKeys), v(values, values + nValues);
  orc::Summary s = static_cast<MergeTree*>(h)->summarize(k, v, chunkSize);
  *headerLen = static_cast<int>(s.header.size());
  *bodyLen = static_cast<int>(s.body.size());
  const std::string all = s.header + s.body;
  if (out) std::memcpy(out, all.data(), std::min<size_t>(all.size(), static_cast<size_t>(cap)));
  return static_cast<int>(all.size());
}

std::atomic<int> g_indexed{0};  // orc_set_index: replays use the remote-length index (BlockIdx)

// The host's numbers of a batch (value ids whose JSON text is a number), sorted, the first id of
// each number (annotate-adjust results equal to one of them take its id).
std::vector<std::pair<double, uint32_t>> hostNumbers(const fmt_mt_batch* b) {
  std::vector<std::pair<double, uint32_t>> v, uniq;
  for (uint32_t i = 0; b->adjusts && b->value_num && i < b->n_values; i++)
    if (!std::isnan(b->value_num[i])) v.emplace_back(b->value_num[i] == 0 ? 0.0 : b->value_num[i], i);
  std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  for (const auto& e : v)
    if (uniq.empty() || uniq.back().first != e.first) uniq.push_back(e);
  return uniq;
}

// The document's initial state: a loaded summary (f3) or its initial text, then collaboration.
void startDoc(MergeTree& mt, const fmt_mt_batch* b, uint32_t d,
              const std::vector<std::pair<double, uint32_t>>* hostNums = nullptr) {
  if (g_indexed.load()) mt.enableIndex();
  mt.relpos = b->relpos;
  mt.nRelpos = b->relpos ? b->n_relpos : 0;
  mt.markerIdKey = b->marker_id_key;
  if (b->adjusts != nullptr) {  // annotate-adjust: rows, host numbers (sorted once per batch)
    mt.adjusts = b->adjusts;
    mt.nAdjusts = b->n_adjusts;
    mt.valueNum = b->value_num;
    mt.nValues = b->value_num ? b->n_values : 0u;
    mt.hostNumbers = hostNums;
    if (b->doc_value_base != nullptr && b->value_num != nullptr) {
      // document-local value ids (fmt.h doc_value_base): id v names value v + base; the host numbers
      // are this document's own, with local ids
      const uint32_t base = b->doc_value_base[d], cnt = b->doc_value_base[d + 1] - base;
      mt.valueNum = b->value_num + base;
      mt.nValues = cnt + 1;
      std::vector<std::pair<double, uint32_t>> v;
      for (uint32_t i = 1; i <= cnt; i++)
        if (!std::isnan(mt.valueNum[i])) v.emplace_back(mt.valueNum[i] == 0 ? 0.0 : mt.valueNum[i], i);
      std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      mt.docNumbers.clear();
      for (const auto& e : v)
        if (mt.docNumbers.empty() || mt.docNumbers.back().first != e.first) mt.docNumbers.push_back(e);
      mt.hostNumbers = &mt.docNumbers;
    }
  }
  mt.snapInfo = b->snapshot_info;
  mt.snapStamps = b->snapshot_stamps;
  mt.nSnapInfo = b->snapshot_info ? b->n_snapshot_segs : 0;
  if (b->snapshots != nullptr && b->snapshots[d].loaded) {
    const fmt_mt_snapshot_doc& sd = b->snapshots[d];
    std::vector<MergeTree::LoadedSeg> head, body;
    for (uint32_t k = 0; k < sd.n_header + sd.n_body; k++) {
      const fmt_mt_snapshot_seg& sg = b->snapshot_segs[sd.first_seg + k];
      MergeTree::LoadedSeg l;
      l.marker = (sg.len & FMT_MT_SEG_MARKER) != 0;
      l.text.assign(reinterpret_cast<const char16_t*>(b->text + sg.text), sg.len & ~FMT_MT_SEG_MARKER);
      if (sg.props != FMT_MT_NO_PROPS) {
        l.hasProps = true;
        for (uint32_t t = b->props_off[sg.props]; t < b->props_off[sg.props + 1]; t++)
          l.props.emplace_back(static_cast<uint16_t>(b->props_kv[t] >> 16), static_cast<uint16_t>(b->props_kv[t] & 0xffff));
      }
      if (b->snapshot_info != nullptr) {  // SnapshotV1 merge info (header segments)
        const fmt_mt_snapshot_info& inf = b->snapshot_info[sd.first_seg + k];
        l.ins = orc::Stamp{inf.ins_seq, inf.ins_client};
        for (uint32_t t = 0; t < inf.rm_count; t++) {
          const fmt_mt_stamp& st = b->snapshot_stamps[inf.rm_first + t];
          l.removes.push_back(orc::Stamp{st.seq, st.client, static_cast<int>(st.kind)});
        }
      }
      (k < sd.n_header ? head : body).push_back(std::move(l));
    }
    mt.loadSnapshot(head, body, sd.min_seq, sd.seq);
  } else {
    if (b->doc_init != nullptr && b->doc_init[2 * d + 1] > 0) {
      const uint32_t off = b->doc_init[2 * d], len = b->doc_init[2 * d + 1];
      mt.insertLocal(0, std::u16string(reinterpret_cast<const char16_t*>(b->text + off), len));
    }
    mt.startCollaboration(0, 0, 0);
  }
}

// ---------------------------------------------------------------- merge-tree, batch replay
// Replays documents [docBegin, docEnd) of a batch with nThreads host threads (one doc per task).
// Output arrays are indexed by (doc - docBegin) with the given per-doc strides; any may be NULL.
int orc_mt_replay_batch(const fmt_mt_batch* b, uint32_t docBegin, uint32_t docEnd,
                        uint32_t nThreads, fmt_mt_doc_result* hdrs, fmt_mt_leaf* leaves,
                        uint32_t capLeaves, uint16_t* chars, uint32_t capChars,
                        fmt_mt_propset* props, uint32_t capProps, fmt_mt_catchup_range* catchup,
                        uint32_t capCatchup, double* seconds, double* nums, uint32_t capNums, uint32_t* nNums) {
  const auto t0 = std::chrono::steady_clock::now();
  std::atomic<int> status{FMT_OK};
  const auto hn = hostNumbers(b);
  parallelFor(docBegin, docEnd, nThreads, [&](uint32_t d) {
    MergeTree mt;
    const size_t i = d - docBegin;
    int32_t failSeq = 0;
    int st = FMT_OK;
    startDoc(mt, b, d, &hn);
    const uint64_t o0 = b->doc_op_offsets[d], o1 = b->doc_op_offsets[d + 1];
    std::vector<fmt_mt_catchup_range> cu;
    st = applyOps(&mt, b->ops + o0, o1 - o0, b->text, b->props_off, b->props_kv, &failSeq,
                  catchup ? &cu : nullptr);
    if (st != FMT_OK) status = st;
    fmt_mt_doc_result* h = hdrs ? &hdrs[i] : nullptr;
    if (h) std::memset(h, 0, sizeof(*h));
    if (hdrs || leaves || chars || props) {
      dumpDoc(&mt, h, leaves ? leaves + i * capLeaves : nullptr, capLeaves,
              chars ? chars + i * static_cast<size_t>(capChars) : nullptr, capChars,
              props ? props + i * capProps : nullptr, capProps);
    }
    if (h) {
      h->status = st;
      h->fail_seq = failSeq;
      h->n_catchup = static_cast<uint32_t>(cu.size());
    }
    if (catchup)
      for (size_t k = 0; k < cu.size() && k < capCatchup; k++) catchup[i * capCatchup + k] = cu[k];
    if (nNums) nNums[i] = static_cast<uint32_t>(mt.numbers.size());
    if (nums)
      for (size_t k = 0; k < mt.numbers.size() && k < capNums; k++) nums[i * capNums + k] = mt.numbers[k];
  });
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return status.load();
}

// f4: document d of a batch replayed; its REGEN events' ops (fmt_mt_fetch_regen's layout: insert
// payloads index `text`). Returns the replay status.
int orc_mt_replay_regen(const fmt_mt_batch* b, uint32_t d, fmt_mt_op* out, uint32_t cap, uint16_t* text,
                        uint32_t textCap, uint32_t* nOps, uint32_t* nText) {
  MergeTree mt;
  startDoc(mt, b, d);
  int32_t failSeq = 0;
  std::vector<fmt_mt_op> ops;
  std::u16string t;
  const uint64_t o0 = b->doc_op_offsets[d], o1 = b->doc_op_offsets[d + 1];
  const int st = applyOps(&mt, b->ops + o0, o1 - o0, b->text, b->props_off, b->props_kv, &failSeq, nullptr, &ops, &t);
  *nOps = static_cast<uint32_t>(ops.size());
  *nText = static_cast<uint32_t>(t.size());
  for (uint32_t i = 0; i < *nOps && i < cap; i++) out[i] = ops[i];
  for (uint32_t i = 0; i < *nText && i < textCap; i++) text[i] = static_cast<uint16_t>(t[i]);
  return st;
}

// Replays documents [docBegin, docEnd) like orc_mt_replay_batch and digests each final state
//  into digests[d - docBegin], so the bench's CPU baseline doubles as its parity check.
// *seconds is the wall time of the pass minus the digests' share: every thread sums the time it
// spent digesting, and the total divided by the thread count comes off (the pool deals documents
// dynamically, so the threads stay balanced).
int orc_mt_replay_digest(const fmt_mt_batch* b, uint32_t docBegin, uint32_t docEnd, uint32_t nThreads,
                         uint64_t* digests, int32_t* statuses, double* seconds) {
  using clk = std::chrono::steady_clock;
  const auto hn = hostNumbers(b);
  std::atomic<int> status{FMT_OK};
  std::atomic<int64_t> digestNs{0};
  const auto t0 = clk::now();
  parallelFor(docBegin, docEnd, nThreads, [&](uint32_t d) {
    const size_t i = d - docBegin;
    MergeTree mt;
    startDoc(mt, b, d, &hn);
    const uint64_t o0 = b->doc_op_offsets[d], o1 = b->doc_op_offsets[d + 1];
    int32_t fs = 0;
    const int st = applyOps(&mt, b->ops + o0, o1 - o0, b->text, b->props_off, b->props_kv, &fs);
    if (st != FMT_OK) status = st;
    const auto td = clk::now();
    fmt_mt_doc_result h{};
    std::vector<const orc::Seg*> segs;
    std::vector<int> blockOf;
    int nb = 0, dp = 0;
    mt.collectLeaves(segs, blockOf, &nb, &dp);
    std::vector<fmt_mt_leaf> lv(segs.size() + 1);
    size_t units = 0;
    for (const orc::Seg* s : segs) units += static_cast<size_t>(s->len());
    std::vector<uint16_t> ch(units + 1);
    std::vector<fmt_mt_propset> pr(segs.size() * (FMT_MT_PROPS_KEYS_MAX / FMT_MT_PROPS_MAX) + 1);  // (wide sets: several records)
    std::vector<uint64_t> hi;
    dumpDoc(&mt, &h, lv.data(), static_cast<uint32_t>(lv.size()), ch.data(), static_cast<uint32_t>(ch.size()), pr.data(),
            static_cast<uint32_t>(pr.size()), &hi);
    h.status = st;
    h.fail_seq = fs;
    if (statuses) statuses[i] = st;
    digests[i] = digestOf(h, lv.data(), ch.data(), pr.data(), &hi);
    digestNs += std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - td).count();
  });
  const double wall = std::chrono::duration<double>(clk::now() - t0).count();
  const uint32_t nt = std::max(1u, std::min(nThreads, docEnd - docBegin));
  if (seconds) *seconds = std::max(0.0, wall - digestNs.load() * 1e-9 / nt);
  return status.load();
}

// The state digest of one dumped document: a test hook pinning the definition.
uint64_t orc_state_digest(const fmt_mt_doc_result* h, const fmt_mt_leaf* leaves, const uint16_t* chars,
                          const fmt_mt_propset* props) {
  return digestOf(*h, leaves, chars, props);
}

// Replays ONE document: its initial state, then at most maxOps of its ops (all with maxOps = 0), timing
// the load and the ops separately (the T3 CPU baseline times the ops). Dumps like orc_mt_replay_batch.
int orc_mt_replay_timed(const fmt_mt_batch* b, uint32_t d, uint64_t maxOps, double* loadSeconds,
                        double* opsSeconds, uint64_t* opsDone, fmt_mt_doc_result* hdr, fmt_mt_leaf* leaves,
                        uint32_t capLeaves, uint16_t* chars, uint32_t capChars, fmt_mt_propset* props,
                        uint32_t capProps) {
  MergeTree mt;
  const auto hn = hostNumbers(b);
  const auto t0 = std::chrono::steady_clock::now();
  startDoc(mt, b, d, &hn);
  const auto t1 = std::chrono::steady_clock::now();
  const uint64_t o0 = b->doc_op_offsets[d];
  uint64_t n = b->doc_op_offsets[d + 1] - o0;
  if (maxOps && maxOps < n) {
    n = maxOps;  // stop at a message boundary
    while (n < b->doc_op_offsets[d + 1] - o0 && (b->ops[o0 + n].flags & FMT_MT_F_GROUP_CONT)) n++;
  }
  int32_t failSeq = 0;
  const int st = applyOps(&mt, b->ops + o0, n, b->text, b->props_off, b->props_kv, &failSeq);
  const auto t2 = std::chrono::steady_clock::now();
  if (loadSeconds) *loadSeconds = std::chrono::duration<double>(t1 - t0).count();
  if (opsSeconds) *opsSeconds = std::chrono::duration<double>(t2 - t1).count();
  if (opsDone) *opsDone = n;
  if (hdr) std::memset(hdr, 0, sizeof(*hdr));
  if (hdr || leaves || chars || props) dumpDoc(&mt, hdr, leaves, capLeaves, chars, capChars, props, capProps);
  if (hdr) {
    hdr->status = st;
    hdr->fail_seq = failSeq;
  }
  return st;
}

void orc_set_index(int on) { g_indexed = on; }

// ---------------------------------------------------------------- SharedMap
// Every remove stamp of every final leaf of document d, in stamp order: (leaf index, client, seq,
// kind) quads into out[4 * k] (kind 0 = setRemove, 1 = sliceRemove), at most cap quads. Returns the
// number of quads, or a negative FMT_E_* code.
// Document d of a batch replayed, then its legacy summary (orc_mt_summary's layout and return value;
// a negative FMT_E_* code when the replay fails).
int orc_mt_replay_summary(const fmt_mt_batch* b, uint32_t d, const char* const* keys, int nKeys,
                          const char* const* values, int nValues, int chunkSize, char* out, int cap,
                          int* headerLen, int* bodyLen) {
  MergeTree mt;
  const auto hn = hostNumbers(b);
  startDoc(mt, b, d, &hn);
  const uint64_t o0 = b->doc_op_offsets[d], o1 = b->doc_op_offsets[d + 1];
  const int st = applyOps(&mt, b->ops + o0, o1 - o0, b->text, b->props_off, b->props_kv, nullptr);
  if (st != FMT_OK) return st;
  return orc_mt_summary(&mt, keys, nKeys, values, nValues, chunkSize, out, cap, headerLen, bodyLen);
}

// Document d of a batch replayed ONCE (a T3 document takes minutes): its state digest, legacy
// summary blobs and catch-up ranges, kept until the next call and read with orc_mt_full_take.
namespace {
struct FullResult {
  std::string blobs;
  int headerLen = 0, bodyLen = 0;
  std::vector<fmt_mt_catchup_range> cu;
  uint64_t digest = 0;
  int32_t minSeq = 0;
};
FullResult g_full;
}  // namespace

int orc_mt_replay_full(const fmt_mt_batch* b, uint32_t d, const char* const* keys, int nKeys, const char* const* values,
                       int nValues, int chunkSize, uint64_t* digest, int* headerLen, int* bodyLen, uint32_t* nCatchup) {
  g_full = FullResult{};
  MergeTree mt;
  const auto hn = hostNumbers(b);
  startDoc(mt, b, d, &hn);
  const uint64_t o0 = b->doc_op_offsets[d], o1 = b->doc_op_offsets[d + 1];
  int32_t fs = 0;
  const int st = applyOps(&mt, b->ops + o0, o1 - o0, b->text, b->props_off, b->props_kv, &fs, &g_full.cu);
  if (st != FMT_OK) return st;
  {
    fmt_mt_doc_result h{};
    std::vector<const orc::Seg*> segs;
    std::vector<int> blockOf;
    int nb = 0, dp = 0;
    mt.collectLeaves(segs, blockOf, &nb, &dp);
    std::vector<fmt_mt_leaf> lv(segs.size() + 1);
    size_t units = 0;
    for (const orc::Seg* s : segs) units += static_cast<size_t>(s->len());
    std::vector<uint16_t> ch(units + 1);
    std::vector<fmt_mt_propset> pr(segs.size() * (FMT_MT_PROPS_KEYS_MAX / FMT_MT_PROPS_MAX) + 1);
    std::vector<uint64_t> hi;
    dumpDoc(&mt, &h, lv.data(), static_cast<uint32_t>(lv.size()), ch.data(), static_cast<uint32_t>(ch.size()), pr.data(),
            static_cast<uint32_t>(pr.size()), &hi);
    h.status = st;
    h.fail_seq = fs;
    g_full.digest = digestOf(h, lv.data(), ch.data(), pr.data(), &hi);
    g_full.minSeq = h.min_seq;
  }
  int hl = 0, bl = 0;
  const int n = orc_mt_summary(&mt, keys, nKeys, values, nValues, chunkSize, nullptr, 0, &hl, &bl);
  if (n < 0) return n;
  g_full.blobs.resize(static_cast<size_t>(n));
  orc_mt_summary(&mt, keys, nKeys, values, nValues, chunkSize, g_full.blobs.data(), n, &hl, &bl);
  g_full.headerLen = hl;
  g_full.bodyLen = bl;
  if (digest) *digest = g_full.digest;
  if (headerLen) *headerLen = hl;
  if (bodyLen) *bodyLen = bl;
  if (nCatchup) *nCatchup = static_cast<uint32_t>(g_full.cu.size());
  return FMT_OK;
}

// The blobs (header then body) and catch-up ranges of the last orc_mt_replay_full.
void orc_mt_full_take(char* blobs, fmt_mt_catchup_range* cu) {
  if (blobs) std::memcpy(blobs, g_full.blobs.data(), g_full.blobs.size());
  if (cu && !g_full.cu.empty()) std::memcpy(cu, g_full.cu.data(), g_full.cu.size() * sizeof(fmt_mt_catchup_range));
}

int orc_mt_removers(const fmt_mt_batch* b, uint32_t d, int32_t* out, uint32_t cap) {
  MergeTree mt;
  const auto hn = hostNumbers(b);
  startDoc(mt, b, d, &hn);
  const uint64_t o0 = b->doc_op_offsets[d], o1 = b->doc_op_offsets[d + 1];
  const int st = applyOps(&mt, b->ops + o0, o1 - o0, b->text, b->props_off, b->props_kv, nullptr);
  if (st != FMT_OK) return st;
  std::vector<const orc::Seg*> segs;
  std::vector<int> blockOf;
  int nBlocks = 0, depth = 0;
  mt.collectLeaves(segs, blockOf, &nBlocks, &depth);
  uint32_t k = 0;
  for (size_t i = 0; i < segs.size(); i++)
    for (const auto& r : segs[i]->removes) {
      if (k < cap) {
        out[4 * k] = static_cast<int32_t>(i);
        out[4 * k + 1] = r.client;
        out[4 * k + 2] = r.seq;
        out[4 * k + 3] = r.kind;
      }
      k++;
    }
  return static_cast<int>(k);
}

int orc_map_replay(const fmt_map_op* ops, const uint64_t* offs, uint32_t nDocs, uint32_t keyBound,
                   fmt_map_slot* out, uint32_t nThreads, double* seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  std::atomic<int> status{FMT_OK};
  parallelFor(0, nDocs, nThreads, [&](uint32_t d) {
    orc::MapState m(keyBound);
    for (uint64_t i = offs[d]; i < offs[d + 1]; i++) {
      const fmt_map_op& op = ops[i];
      const uint32_t kind = op.kind_value >> FMT_MAP_KIND_SHIFT;
      if (kind == FMT_MAP_CLEAR) {
        m.clear();
      } else if (op.key >= keyBound) {
        status = FMT_E_DATA;
      } else if (kind == FMT_MAP_DELETE) {
        m.del(op.key);
      } else {
        m.set(op.key, op.kind_value & FMT_MAP_VALUE_MASK, op.seq);
      }
    }
    if (out) m.toSlots(out + static_cast<size_t>(d) * keyBound, keyBound);
  });
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return status.load();
}

// The sparse path's oracle (any key pool): per document its live entries in Map order, written at
// the document's op offset (entries[offs[d] ..], counts[d] of them) as fmt_map_entry does on the GPU
// before packing.
int orc_map_replay_sparse(const fmt_map_op* ops, const uint64_t* offs, uint32_t nDocs, uint32_t keyBound,
                          uint32_t* counts, fmt_map_entry* entries, uint32_t nThreads, double* seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  std::atomic<int> status{FMT_OK};
  parallelFor(0, nDocs, nThreads, [&](uint32_t d) {
    orc::MapState m(keyBound, true);
    for (uint64_t i = offs[d]; i < offs[d + 1]; i++) {
      const fmt_map_op& op = ops[i];
      const uint32_t kind = op.kind_value >> FMT_MAP_KIND_SHIFT;
      if (kind == FMT_MAP_CLEAR) m.clear();
      else if (op.key >= keyBound) status = FMT_E_DATA;
      else if (kind == FMT_MAP_DELETE) m.del(op.key);
      else m.set(op.key, op.kind_value & FMT_MAP_VALUE_MASK, op.seq);
    }
    const auto es = m.entries();
    counts[d] = static_cast<uint32_t>(es.size());
    if (entries)
      for (size_t j = 0; j < es.size(); j++) entries[offs[d] + j] = {es[j].key, es[j].value, es[j].birth};
  });
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return status.load();
}

// The local-client pending state's oracle: each document's sequenced entries (as the sparse path),
// then its local events through PendingMap; the optimistic entries at offs[d] + evOffs[d] (counts,
// status per document) as fmt_map_pending_run writes them before packing. Submissions are named by
// their index within the document's events; ACK resolves the oldest unacknowledged one, ROLLBACK
// the newest (PendingStateManager's order), and the event must repeat that submission's op.
int orc_map_pending(const fmt_map_op* ops, const uint64_t* offs, uint32_t nDocs, uint32_t keyBound,
                    const fmt_map_local_op* events, const uint64_t* evOffs, uint32_t* counts, int32_t* status,
                    fmt_map_entry* entries) {
  for (uint32_t d = 0; d < nDocs; d++) {
    orc::MapState m(keyBound, true);
    for (uint64_t i = offs[d]; i < offs[d + 1]; i++) {
      const uint32_t kind = ops[i].kind_value >> FMT_MAP_KIND_SHIFT;
      if (kind == FMT_MAP_CLEAR) m.clear();
      else if (kind == FMT_MAP_DELETE) m.del(ops[i].key);
      else m.set(ops[i].key, ops[i].kind_value & FMT_MAP_VALUE_MASK, ops[i].seq);
    }
    orc::PendingMap p;
    std::deque<uint32_t> unacked;
    bool ok = true;
    for (uint64_t i = evOffs[d]; i < evOffs[d + 1] && ok; i++) {
      const fmt_map_local_op& e = events[i];
      const uint32_t sub = static_cast<uint32_t>(i - evOffs[d]);
      const uint32_t kind = e.kind_value >> FMT_MAP_KIND_SHIFT;
      if (e.event == FMT_MAP_EV_SUBMIT) {
        unacked.push_back(static_cast<uint32_t>(i));
        if (kind == FMT_MAP_SET) p.set(e.key, e.kind_value & FMT_MAP_VALUE_MASK, sub);
        else if (kind == FMT_MAP_DELETE) p.del(e.key, sub);
        else p.clear(sub);
        continue;
      }
      if (unacked.empty()) {
        ok = false;
        break;
      }
      const uint32_t s = e.event == FMT_MAP_EV_ACK ? unacked.front() : unacked.back();
      if (e.event == FMT_MAP_EV_ACK) unacked.pop_front();
      else unacked.pop_back();
      const fmt_map_local_op& so = events[s];
      if (so.kind_value != e.kind_value || (kind != FMT_MAP_CLEAR && so.key != e.key)) {
        ok = false;
        break;
      }
      const uint32_t ssub = static_cast<uint32_t>(s - evOffs[d]);
      ok = e.event == FMT_MAP_EV_ACK ? p.ack(kind, so.key, ssub) : p.rollback(kind, so.key, ssub);
    }
    status[d] = ok ? FMT_OK : FMT_E_DATA;
    counts[d] = 0;
    if (!ok) continue;
    const auto es = p.iterate(m.entries());
    counts[d] = static_cast<uint32_t>(es.size());
    for (size_t j = 0; j < es.size(); j++) entries[offs[d] + evOffs[d] + j] = {es[j].key, es[j].value, es[j].birth};
  }
  return FMT_OK;
}

// Summary of one document: header then each blobN, NUL-separated; returns bytes needed.
int orc_map_summary(const fmt_map_op* ops, uint64_t begin, uint64_t end, uint32_t keyBound,
                    const char* const* keys, int nKeys, const char* const* values, int nValues,
                    char* out, int cap, int* nBlobs) {
  orc::MapState m(keyBound);
  for (uint64_t i = begin; i < end; i++) {
    const uint32_t kind = ops[i].kind_value >> FMT_MAP_KIND_SHIFT;
    if (kind == FMT_MAP_CLEAR) m.clear();
    else if (kind == FMT_MAP_DELETE) m.del(ops[i].key);
    else m.set(ops[i].key, ops[i].kind_value & FMT_MAP_VALUE_MASK, ops[i].seq);
  }
  std::vector<std::string> k(keys, keys + nKeys), v(values, values + nValues);
  orc::MapSummary s = orc::summarizeMap(m.entries(), k, v);
  std::string all = s.header;
  all.push_back('\0');
  for (auto& bl : s.blobs) {
    all += bl;
    all.push_back('\0');
  }
  *nBlobs = static_cast<int>(s.blobs.size());
  if (out) std::memcpy(out, all.data(), std::min<size_t>(all.size(), static_cast<size_t>(cap)));
  return static_cast<int>(all.size());
}

// ---------------------------------------------------------------- PRNG known answers
void orc_xsadd_uint32(const uint32_t* seed, int nSeed, uint32_t* out, int n) {
  orc::XSadd x(std::vector<uint32_t>(seed, seed + nSeed));
  for (int i = 0; i < n; i++) out[i] = x.uint32();
}

// kind 0: float64, 1: uint32 (as double), 2: uint53 — one call per sample in the given order.
void orc_xsadd_mixed(const uint32_t* seed, int nSeed, const int* kinds, double* out, int n) {
  orc::XSadd x(std::vector<uint32_t>(seed, seed + nSeed));
  for (int i = 0; i < n; i++) {
    switch (kinds[i]) {
      case 0: out[i] = x.float64(); break;
      case 1: out[i] = static_cast<double>(x.uint32()); break;
      default: out[i] = x.uint53(); break;
    }
  }
}

}  // extern "C"
