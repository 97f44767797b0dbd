// fmtgen.cpp — synthetic sequenced op streams for the engine's benchmarks and parity tests.
//
// Workload synthesis only (not the engine, not the oracle). It reproduces the SHAPE of the
// reference's own stochastic workloads with the reference's PRNG:
//   - SharedMap: the map fuzz generator, set:delete:clear = 20:20:1 over keys "0".."19",
//     values pick(int 1..50, base58 string of length 3..7) (map/src/test/mocha/fuzzUtils.ts:108-146,
//     stochastic-test-utils/src/generators.ts:46-91);
//   - merge-tree: the conflict farm (merge-tree/src/test/mergeTreeOperationRunner.ts:285-429,
//     client.conflictFarm.spec.ts:70-126): rounds of 1,2,4,...,128 ops, every op of a round
//     referencing the round start (refSeq = msn = round start), a random writer client, a forced
//     insert while the client's view is shorter than minLength, otherwise one of
//     remove / annotate / insert over random positions of the client's view.
// Positions are drawn against the length of the op's own perspective, PriorPerspective(refSeq,
// client) (perspective.ts:80-93), computed on a flat observer model of the document. Ordering and
// tie-breaks follow the merge-tree's rules for remote ops, so every generated op is valid.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../../include/fmt.h"

namespace {

// XSadd (stochastic-test-utils/src/xsadd.ts:38-89) and the makeRandom distributions.
class Rng {
 public:
  Rng(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    int32_t s[4] = {static_cast<int32_t>(a), static_cast<int32_t>(b), static_cast<int32_t>(c),
                    static_cast<int32_t>(d)};
    for (int i = 1; i < 8 || (s[0] | s[1] | s[2] | s[3]) == 0; i++) {
      const uint32_t p = static_cast<uint32_t>(s[(i - 1) & 3]);
      s[i & 3] = static_cast<int32_t>(static_cast<uint32_t>(s[i & 3]) ^
                                      (static_cast<uint32_t>(i) + 0x6c078965u * (p ^ (p >> 30))));
    }
    x_ = s[0], y_ = s[1], z_ = s[2], w_ = s[3];
    for (int i = 0; i < 8; i++) next();
  }
  uint32_t next() {
    uint32_t t = x_;
    x_ = y_, y_ = z_, z_ = w_;
    t ^= t << 15;
    t ^= t >> 18;
    t ^= w_ << 11;
    w_ = t;
    return w_ + z_;
  }
  double uint53() {
    const double hi = static_cast<double>(next() >> 6);
    return hi * 134217728.0 + static_cast<double>(next() >> 5);
  }
  double float64() { return uint53() / 9007199254740992.0; }
  int64_t integer(int64_t min, int64_t max) {
    const double range = static_cast<double>(max - min + 1);
    const double divisor = std::trunc(9007199254740992.0 / range);
    double r;
    do r = uint53() / divisor;
    while (r >= range);
    return static_cast<int64_t>(r) + min;
  }
  double real(double min, double max) {
    const double a = float64();
    return (1 - a) * min + a * max;
  }

 private:
  uint32_t x_, y_, z_, w_;
};

template <class F>
void parallelFor(uint32_t n, uint32_t threads, F&& fn) {
  if (threads <= 1) {
    for (uint32_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < threads; t++)
    pool.emplace_back([&] {
      for (uint32_t i = next.fetch_add(1); i < n; i = next.fetch_add(1)) fn(i);
    });
  for (auto& th : pool) th.join();
}

// ---------------------------------------------------------------------------------------------
// Flat observer model of one document for position drawing.
// ---------------------------------------------------------------------------------------------
struct FlatSeg {
  int len;
  int insSeq;
  int insClient;
  int rmSeq;      // lowest remove seq, INT_MAX if not removed
  uint64_t rmMask[4];  // remove clients 0..253
};

class FlatDoc {
 public:
  int lengthFor(int refSeq, int client) const {
    int n = 0;
    for (const auto& s : segs_)
      if (present(s, refSeq, client)) n += s.len;
    return n;
  }
  void insert(int pos, int len, int seq, int refSeq, int client) {
    splitAt(pos, refSeq, client);
    // first leaf at which the remaining position reaches 0 (remote-op tie-break, mergeTree.ts:1811)
    int rem = pos;
    size_t i = 0;
    for (; i < segs_.size(); i++) {
      if (rem == 0) break;
      rem -= present(segs_[i], refSeq, client) ? segs_[i].len : 0;
    }
    segs_.insert(segs_.begin() + static_cast<long>(i), FlatSeg{len, seq, client, 0x7fffffff, {0, 0, 0, 0}});
  }
  void removeRange(int start, int end, int seq, int refSeq, int client) {
    splitAt(start, refSeq, client);
    splitAt(end, refSeq, client);
    int pos = 0;
    for (auto& s : segs_) {
      if (pos >= end) break;
      if (!present(s, refSeq, client)) continue;
      if (pos >= start) {
        s.rmSeq = std::min(s.rmSeq, seq);
        s.rmMask[client >> 6] |= 1ull << (client & 63);
      }
      pos += s.len;
    }
  }
  void annotateRange(int start, int end, int refSeq, int client) {
    splitAt(start, refSeq, client);
    splitAt(end, refSeq, client);
  }
  // Tombstones removed at or below minSeq are invisible to every later perspective.
  void setMinSeq(int minSeq) {
    segs_.erase(std::remove_if(segs_.begin(), segs_.end(), [&](const FlatSeg& s) { return s.rmSeq <= minSeq; }),
                segs_.end());
  }

 private:
  static bool present(const FlatSeg& s, int refSeq, int client) {
    if (!(s.insSeq <= refSeq || s.insClient == client)) return false;
    if (s.rmSeq <= refSeq || ((s.rmMask[client >> 6] >> (client & 63)) & 1)) return false;
    return true;
  }
  void splitAt(int pos, int refSeq, int client) {
    int p = 0;
    for (size_t i = 0; i < segs_.size(); i++) {
      if (!present(segs_[i], refSeq, client)) continue;
      if (pos <= p) return;  // already a boundary
      const int l = segs_[i].len;
      if (pos < p + l) {
        FlatSeg tail = segs_[i];
        tail.len = p + l - pos;
        segs_[i].len = pos - p;
        segs_.insert(segs_.begin() + static_cast<long>(i) + 1, tail);
        return;
      }
      p += l;
    }
  }
  std::vector<FlatSeg> segs_;
};

struct GenDoc {
  std::vector<fmt_mt_op> ops;
  std::vector<uint16_t> text;
};

// Client names as in mergeTreeOperationRunner.ts generateClientNames: 'A'.. (A = observer).
inline uint16_t clientChar(int client) {
  if (client < 26) return static_cast<uint16_t>('A' + client);
  if (client < 52) return static_cast<uint16_t>('a' + client - 26);
  return static_cast<uint16_t>('0' + client - 52);
}

void genConflictFarmDoc(GenDoc& out, uint32_t docId, uint32_t nClients, uint32_t nOps, uint32_t minLength,
                        uint32_t seed, uint32_t annotatePropsBase) {
  Rng rng(0xdeadbeefu, 0xfeedbedu, minLength, docId ^ (seed * 0x9E3779B9u));
  FlatDoc doc;
  int seq = 0;
  uint32_t produced = 0;
  int opsPerRound = 1;
  while (produced < nOps) {
    const int roundStart = seq;
    for (int i = 0; i < opsPerRound && produced < nOps; i++) {
      const int client = static_cast<int>(rng.integer(1, nClients));
      const int len = doc.lengthFor(roundStart, client);
      fmt_mt_op op{};
      op.seq = ++seq;
      op.ref_seq = roundStart;
      op.min_seq = roundStart;
      op.client = static_cast<uint8_t>(client);
      int kind;
      int start = 0, end = 0;
      if (len == 0 || len < static_cast<int>(minLength)) {
        kind = FMT_MT_INSERT;
        start = static_cast<int>(rng.integer(0, len));
      } else {
        const int which = static_cast<int>(rng.integer(0, 2));
        start = static_cast<int>(rng.integer(0, len - 1));
        end = static_cast<int>(rng.integer(start + 1, len));
        kind = which == 0 ? FMT_MT_REMOVE : which == 1 ? FMT_MT_ANNOTATE : FMT_MT_INSERT;
        if (kind == FMT_MT_INSERT) start = static_cast<int>(rng.integer(0, len));
      }
      op.type = static_cast<uint8_t>(kind);
      op.pos1 = start;
      if (kind == FMT_MT_INSERT) {
        const int reps = static_cast<int>(rng.integer(1, 3));
        op.pos2 = -1;
        op.payload = static_cast<uint32_t>(out.text.size());
        op.len = static_cast<uint16_t>(reps);
        for (int r = 0; r < reps; r++) out.text.push_back(clientChar(client));
        doc.insert(start, reps, op.seq, roundStart, client);
      } else if (kind == FMT_MT_REMOVE) {
        op.pos2 = end;
        doc.removeRange(start, end, op.seq, roundStart, client);
      } else {
        op.pos2 = end;
        op.payload = annotatePropsBase + static_cast<uint32_t>(client);  // props op {"client": name}
        doc.annotateRange(start, end, roundStart, client);
      }
      out.ops.push_back(op);
      produced++;
    }
    // all of the round's messages are sequenced; the next round references its end
    doc.setMinSeq(roundStart);
    opsPerRound = opsPerRound >= 128 ? 1 : opsPerRound * 2;
  }
}

}  // namespace

extern "C" {

// SharedMap fuzz-shaped stream: n_docs × ops_per_doc ops, keys 0..key_pool-1.
// Value ids: 0..49 ↔ integers 1..50; ≥ 50 ↔ an opaque base58 string (id = 50 + per-doc ordinal).
// out_ops must hold n_docs * ops_per_doc records; out_offsets n_docs + 1 entries.
int fmtgen_map(uint32_t n_docs, uint32_t ops_per_doc, uint32_t key_pool, uint32_t seed,
               fmt_map_op* out_ops, uint64_t* out_offsets, uint32_t threads) {
  if (key_pool == 0 || key_pool > 0x3fffffff) return FMT_E_USAGE;
  for (uint32_t d = 0; d <= n_docs; d++) out_offsets[d] = static_cast<uint64_t>(d) * ops_per_doc;
  parallelFor(n_docs, threads, [&](uint32_t d) {
    Rng rng(0xdeadbeefu, 0xfeedbedu, d, seed);
    fmt_map_op* o = out_ops + static_cast<uint64_t>(d) * ops_per_doc;
    uint32_t strings = 0;
    for (uint32_t i = 0; i < ops_per_doc; i++) {
      // createWeightedGenerator over [set 20, delete 20, clear 1]
      const double w = rng.real(0, 41);
      const uint32_t kind = w <= 20 ? FMT_MAP_SET : (w <= 40 ? FMT_MAP_DELETE : FMT_MAP_CLEAR);
      uint32_t key = 0, value = 0;
      if (kind != FMT_MAP_CLEAR) key = static_cast<uint32_t>(rng.integer(0, key_pool - 1));
      if (kind == FMT_MAP_SET) {
        if (rng.integer(0, 1) == 0) {
          value = static_cast<uint32_t>(rng.integer(1, 50) - 1);
        } else {
          const int n = static_cast<int>(rng.integer(3, 7));
          for (int c = 0; c < n; c++) rng.integer(0, 57);
          value = 50 + (strings++ % 0x3ffffff0u);
        }
      }
      o[i] = fmt_map_op{d, key, i + 1, (kind << FMT_MAP_KIND_SHIFT) | (value & FMT_MAP_VALUE_MASK)};
    }
  });
  return FMT_OK;
}

// Conflict-farm merge-tree streams (generated once into a handle, then copied out).
//   n_clients writer clients (short ids 1..n_clients; 0 is the observer), ops_per_doc messages per
//   document, min_length cycling over 1,2,4,...,512 by document id unless min_length_fixed > 0.
// Annotate ops reference props op (annotate_props_base + client) = {"client": <client name>}.
// Documents are deterministic in (doc id, seed).
struct CfHandle {
  std::vector<GenDoc> docs;
  std::vector<uint64_t> opOff, textOff;
};

// Documents doc_base .. doc_base + n_docs - 1 of the (conceptually unbounded) document set: a shard
// of a large batch (T2) is generated by its own rank with the same per-document streams.
void* fmtgen_conflict_farm_new(uint32_t n_docs, uint32_t n_clients, uint32_t ops_per_doc,
                               uint32_t min_length_fixed, uint32_t seed, uint32_t annotate_props_base,
                               uint32_t threads, uint64_t* n_ops, uint64_t* n_text, uint32_t doc_base) {
  if (n_clients == 0 || n_clients > 253) return nullptr;  // (short ids 1..253; 0xFE names NonCollab)
  auto* h = new CfHandle();
  h->docs.resize(n_docs);
  parallelFor(n_docs, threads, [&](uint32_t i) {
    const uint32_t d = doc_base + i;
    const uint32_t minLength = min_length_fixed ? min_length_fixed : (1u << (d % 10));
    genConflictFarmDoc(h->docs[i], d, n_clients, ops_per_doc, minLength, seed, annotate_props_base);
  });
  h->opOff.assign(n_docs + 1, 0);
  h->textOff.assign(n_docs + 1, 0);
  for (uint32_t d = 0; d < n_docs; d++) {
    h->opOff[d + 1] = h->opOff[d] + h->docs[d].ops.size();
    h->textOff[d + 1] = h->textOff[d] + h->docs[d].text.size();
  }
  *n_ops = h->opOff[n_docs];
  *n_text = h->textOff[n_docs];
  return h;
}

// Copies the streams; `replicas` copies of the whole set are laid out back to back (each replica
// with its own ops and text, so replicated documents share no bytes in HBM).
int fmtgen_conflict_farm_copy(void* handle, uint32_t replicas, fmt_mt_op* out_ops,
                              uint64_t* out_offsets, uint16_t* out_text, uint32_t threads) {
  auto* h = static_cast<CfHandle*>(handle);
  const uint32_t n = static_cast<uint32_t>(h->docs.size());
  const uint64_t opsPer = h->opOff[n], textPer = h->textOff[n];
  if (textPer * replicas >= 0xffffffffull) return FMT_E_CAPACITY;  // payload offsets are 32-bit
  parallelFor(n * replicas, threads, [&](uint32_t i) {
    const uint32_t r = i / n, d = i % n;
    const uint64_t ob = r * opsPer + h->opOff[d], tb = r * textPer + h->textOff[d];
    const GenDoc& g = h->docs[d];
    for (size_t k = 0; k < g.ops.size(); k++) {
      fmt_mt_op o = g.ops[k];
      if (o.type == FMT_MT_INSERT) o.payload += static_cast<uint32_t>(tb);
      out_ops[ob + k] = o;
    }
    std::memcpy(out_text + tb, g.text.data(), g.text.size() * sizeof(uint16_t));
    out_offsets[i] = ob;
  });
  out_offsets[static_cast<uint64_t>(n) * replicas] = opsPer * replicas;
  return FMT_OK;
}

void fmtgen_free(void* handle) { delete static_cast<CfHandle*>(handle); }

// T3 (BASELINE config 5): ONE SharedString loaded from a summary of n_segments segments (length
// U[1,8], letters a..z, no props), then n_ops sequenced messages from n_clients writers (short ids
// 1..n_clients) with deep refSeq windows: every op's refSeq lags its seq by U[0, max_lag) (clamped to
// stay non-decreasing per client) and msn = min over clients of their latest refSeq (the MSN rule of
// mocks.ts:587-604 / deli clientSeqManager.ts:131). Op kinds insert / remove / annotate with equal
// weight as in the conflict farm (mergeTreeOperationRunner.ts:341-429), but remove / annotate ranges
// are local edits of U[1, max_range] chars: the farm's end = U[start+1, len] would delete a third of
// a 10M-segment document per remove, leaving no large document after a few dozen ops.
// Positions are drawn below a lower bound of the op's perspective length (PriorPerspective(refSeq,
// client), perspective.ts:80-93): initial chars + all inserted chars - all remove range lengths -
// the chars inserted by messages the op has not seen (seq > refSeq), so every op is valid.
// Outputs: out_segs[n_segments] = (text offset, len, FMT_MT_NO_PROPS); out_text (capacity
// n_segments * 8 + n_ops * 3 units) = the segments' text, then the insert payloads; out_ops[n_ops].
// Returns the number of text units written, or a negative FMT_E_* code.
int64_t fmtgen_t3(uint32_t n_segments, uint32_t n_ops, uint32_t n_clients, uint32_t max_lag, uint32_t max_range,
                  uint32_t seed, uint32_t annotate_props_base, fmt_mt_snapshot_seg* out_segs, uint16_t* out_text,
                  fmt_mt_op* out_ops) {
  if (n_clients == 0 || n_clients > 253 || max_lag == 0 || max_range == 0) return FMT_E_USAGE;
  Rng rng(0xdeadbeefu, 0xfeedbedu, 0x7733u, seed);
  uint64_t t = 0;
  int64_t chars = 0;
  for (uint32_t k = 0; k < n_segments; k++) {
    const uint32_t len = static_cast<uint32_t>(rng.integer(1, 8));
    out_segs[k] = fmt_mt_snapshot_seg{static_cast<uint32_t>(t), len, FMT_MT_NO_PROPS};
    for (uint32_t c = 0; c < len; c++) out_text[t++] = static_cast<uint16_t>('a' + rng.integer(0, 25));
    chars += len;
  }
  // lower bound of every perspective's length, and the inserted chars per seq (for the unseen ones)
  int64_t lb = chars;
  std::vector<int64_t> insPrefix(static_cast<size_t>(n_ops) + 1, 0);  // chars inserted by seqs 1..s
  std::vector<int32_t> lastRef(n_clients + 1, 0);
  int32_t msn = 0;
  for (uint32_t i = 0; i < n_ops; i++) {
    const int32_t seq = static_cast<int32_t>(i + 1);
    const int client = static_cast<int>(rng.integer(1, n_clients));
    const int32_t lagCap = std::min<int32_t>(seq - 1, static_cast<int32_t>(max_lag) - 1);
    const int32_t lag = lagCap > 0 ? static_cast<int32_t>(rng.integer(0, lagCap)) : 0;
    const int32_t ref = std::max(lastRef[client], seq - 1 - lag);
    lastRef[client] = ref;
    int32_t m = ref;
    for (uint32_t c = 1; c <= n_clients; c++) m = std::min(m, lastRef[c]);
    msn = std::max(msn, m);
    const int64_t unseen = insPrefix[i] - insPrefix[static_cast<size_t>(ref)];
    const int64_t len = std::max<int64_t>(0, lb - unseen);
    fmt_mt_op op{};
    op.seq = seq;
    op.ref_seq = ref;
    op.min_seq = msn;
    op.client = static_cast<uint8_t>(client);
    int kind = len == 0 ? FMT_MT_INSERT : static_cast<int>(rng.integer(0, 2));
    kind = kind == 0 ? FMT_MT_REMOVE : kind == 1 ? FMT_MT_ANNOTATE : FMT_MT_INSERT;
    if (len == 0) kind = FMT_MT_INSERT;
    op.type = static_cast<uint8_t>(kind);
    insPrefix[i + 1] = insPrefix[i];
    if (kind == FMT_MT_INSERT) {
      const int reps = static_cast<int>(rng.integer(1, 3));
      op.pos1 = static_cast<int32_t>(rng.integer(0, len));
      op.pos2 = -1;
      op.payload = static_cast<uint32_t>(t);
      op.len = static_cast<uint16_t>(reps);
      for (int r = 0; r < reps; r++) out_text[t++] = clientChar(client);
      lb += reps;
      insPrefix[i + 1] += reps;
    } else {
      const int64_t start = rng.integer(0, len - 1);
      const int64_t n = rng.integer(1, max_range);
      const int64_t end = std::min(start + n, len);
      op.pos1 = static_cast<int32_t>(start);
      op.pos2 = static_cast<int32_t>(end);
      if (kind == FMT_MT_REMOVE) {
        lb -= end - start;
      } else {
        op.payload = annotate_props_base + static_cast<uint32_t>(client);  // {"client": name}
      }
    }
    out_ops[i] = op;
  }
  return static_cast<int64_t>(t);
}

}  // extern "C"
