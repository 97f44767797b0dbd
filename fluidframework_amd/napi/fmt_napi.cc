// fmt_napi.cc — N-API addon exposing libfmt.so (include/fmt.h) to Node.js.
//
// This is the thin native layer between the reference's JavaScript runtime and the HIP engine.
// The reference applies one sequenced message per call, on the JS thread:
//   SharedObjectCore.processMessagesCore   packages/dds/shared-object-base/src/sharedObject.ts:415
//   SharedMap.processMessagesCore          packages/dds/map/src/map.ts:288-311
//   SharedSegmentSequence.processMessagesCore  packages/dds/sequence/src/sequence.ts:873-919
// Here one call replays a whole packed batch of many documents (fluidframework_amd/js/fmt.js packs
// it), and the load + replay + header fetch run on a libuv worker thread through napi_async_work so
// the JS event loop is never blocked. Errors reject the promise with an Error whose `code` is the
// FMT_E_* name (FMT_E_DATA is the DataProcessingError analogue, mergeTree.ts:1629-1638).
//
// Exports:
//   open(device) -> ctx                        fmt_open
//   close(ctx)                                 fmt_close (contexts still open at exit: an env cleanup hook)
//   openContexts() -> number                   contexts open in this process
//   deviceInfo(ctx) -> string                  fmt_device_info
//   capacity() -> {leaves, chars, props}       fmt_mt_capacity
//   replayMergeTree(ctx, batch) -> Promise<ArrayBuffer headers>     fmt_mt_load + fmt_mt_run + fetch
//   fetchDoc(ctx, doc, nLeaves, nChars, nProps) -> {leaves, chars, props}   fmt_mt_fetch_doc
//   fetchCatchup(ctx, doc, n) -> ArrayBuffer                         fmt_mt_fetch_catchup
//   fetchCatchupAll(ctx, nDocs) -> {offsets, ranges}                 fmt_mt_fetch_catchup_all
//   fetchRemoveOrder(ctx, doc, n) -> ArrayBuffer                     fmt_mt_fetch_remove_order
//   fetchNumbers(ctx, doc) -> Float64Array                           fmt_mt_fetch_numbers
//   fetchLegacyProps(ctx, doc, nLeaves) -> Uint16Array               fmt_mt_fetch_legacy_props
//   fetchRmClientsHi(ctx, doc, nLeaves) -> BigUint64Array            fmt_mt_fetch_rm_clients_hi (ids 64..127)
//   fetchRegen(ctx, doc) -> {ops: ArrayBuffer, text: Uint16Array}     fmt_mt_fetch_regen (f4 reconnects)
//   replayMap(ctx, batch) -> Promise<ArrayBuffer slots>              fmt_map_load + run + fetch
//   replayMapSparse(ctx, batch) -> Promise<{counts, entries}>        fmt_map_load_sparse + run + fetch
//   summarizeLegacy(ctx, quotedKeys, values, chunk, threads) -> Promise<timing>   fmt_mt_summarize_legacy
//   summaryBlobs(ctx, doc) -> {header, body?}                        fmt_mt_summary_blobs
//   stats(ctx) -> {kernelMs, totalMs, ops, docs, bytesRead, bytesWritten, launches}
//   sizes: {mtOp, mapOp, leaf, docResult, propset, mapSlot}          struct sizes for the JS views
#include <node_api.h>

#include <execinfo.h>
#include <unistd.h>

#include <csignal>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "fmt.h"

namespace {

#define CHECK_NAPI(env, call)                                                      \
  do {                                                                             \
    if ((call) != napi_ok) {                                                       \
      napi_throw_error((env), "FMT_E_USAGE", "N-API call failed: " #call);         \
      return nullptr;                                                              \
    }                                                                              \
  } while (0)

const char* status_name(int rc) {
  switch (rc) {
    case FMT_OK: return "FMT_OK";
    case FMT_E_USAGE: return "FMT_E_USAGE";
    case FMT_E_DATA: return "FMT_E_DATA";
    case FMT_E_CAPACITY: return "FMT_E_CAPACITY";
    case FMT_E_DEVICE: return "FMT_E_DEVICE";
    case FMT_E_UNSUPPORTED: return "FMT_E_UNSUPPORTED";
    default: return "FMT_E_UNKNOWN";
  }
}

struct Ctx {
  fmt_ctx* ctx = nullptr;
  bool busy = false;  // one async replay at a time per ctx (the C ABI is one-thread-per-ctx)
};

// Context lifetime without N-API weak references. node v12 (this image's) frees every weak
// v8impl::Reference when the environment is torn down even if GC already ran its first weak pass,
// and the queued second pass then calls through the freed object: the SIGSEGV at exit (libnode.so.72
// +0x878a80, the second-pass callback loading the vtable of a freed Reference, reached from
// InvokeSecondPassPhantomCallbacks during FreeEnvironment's CleanupHandles). node v12's
// napi_create_external makes such a Reference for every External, finalizer or not (round 5's
// Externals without finalizers still crashed the same way, profiles/r5/last/), so a context handle
// is a plain JS number: slot + 1 + (generation mod 2^20) * 2^32 into this table. close() frees the slot and its device context at
// once; a stale handle (closed, or from a reused slot) is detected, never dereferenced. Contexts
// still open when the environment is torn down are closed by an env cleanup hook, before node
// deletes the napi_env and while the HIP runtime is alive. Open contexts are capped
// (FMT_NAPI_MAX_CONTEXTS, default 64): a caller that drops contexts without close() gets
// FMT_E_CAPACITY instead of device memory that grows without bound.
// The table is process-wide (a handle is only a number), but every slot belongs to the napi_env
// (main thread or worker_thread) that opened it: only that env can use or close it, and its env
// cleanup hook closes only its own slots, so one worker's teardown never closes another thread's
// contexts. Slots are reached under one mutex (a worker's open() may grow the vector while another
// thread looks a handle up); a Ctx itself is only ever touched by its owner's thread.
struct Slot {
  Ctx* c = nullptr;
  napi_env env = nullptr;  // the owner
  uint32_t gen = 0;
};
std::vector<Slot>& slots() {
  static std::vector<Slot>* s = new std::vector<Slot>();
  return *s;
}
std::mutex& slots_mu() {
  static std::mutex* m = new std::mutex();
  return *m;
}
uint32_t max_contexts() {
  const char* e = std::getenv("FMT_NAPI_MAX_CONTEXTS");
  const long v = e ? std::strtol(e, nullptr, 10) : 0;
  return v > 0 ? static_cast<uint32_t>(v) : 64u;
}
uint32_t live_contexts() {  // (caller holds slots_mu)
  uint32_t n = 0;
  for (const Slot& s : slots()) n += s.c != nullptr;
  return n;
}

// env cleanup hook (arg: the env it was registered for): closes that env's contexts only
void close_env_at_teardown(void* arg) {
  const napi_env env = static_cast<napi_env>(arg);
  std::vector<Ctx*> mine;
  {
    std::lock_guard<std::mutex> lk(slots_mu());
    for (Slot& s : slots()) {
      if (s.c == nullptr || s.env != env || s.c->busy) continue;  // (a replay still on a worker: left to process exit)
      mine.push_back(s.c);
      s.c = nullptr;
      s.env = nullptr;
      s.gen++;
    }
  }
  for (Ctx* c : mine) {
    if (c->ctx) fmt_close(c->ctx);
    delete c;
  }
}

// A handle is a plain JS number, slot + 1 + (generation mod 2^20) * 2^32 (exact in a double).
constexpr uint32_t kGenMask = 0xFFFFFu;
enum class Lookup { kOk, kStale, kForeign };
// The open context handle h names, if it belongs to env (kForeign: another thread's context).
Ctx* ctx_of_handle(napi_env env, uint64_t h, Lookup* why = nullptr) {
  const uint32_t slot = static_cast<uint32_t>(h & 0xffffffffu), gen = static_cast<uint32_t>(h >> 32);
  std::lock_guard<std::mutex> lk(slots_mu());
  Lookup w = Lookup::kStale;
  Ctx* c = nullptr;
  if (slot != 0 && slot <= slots().size()) {
    const Slot& s = slots()[slot - 1];
    if ((s.gen & kGenMask) == gen && s.c != nullptr) {
      w = s.env == env ? Lookup::kOk : Lookup::kForeign;
      c = w == Lookup::kOk ? s.c : nullptr;
    }
  }
  if (why) *why = w;
  return c;
}
// The handle in v (false: v is not a number an open() returned).
bool handle_of(napi_env env, napi_value v, uint64_t* h) {
  double d = 0;
  if (napi_get_value_double(env, v, &d) != napi_ok || !(d >= 1.0) || d > 9007199254740991.0) return false;
  *h = static_cast<uint64_t>(d);
  return static_cast<double>(*h) == d;
}

napi_value make_error(napi_env env, int rc, const std::string& msg) {
  napi_value code, text, err;
  napi_create_string_utf8(env, status_name(rc), NAPI_AUTO_LENGTH, &code);
  napi_create_string_utf8(env, msg.c_str(), msg.size(), &text);
  napi_create_error(env, code, text, &err);
  napi_value status;
  napi_create_int32(env, rc, &status);
  napi_set_named_property(env, err, "status", status);
  return err;
}

bool throw_fmt(napi_env env, int rc, const std::string& msg) {
  napi_throw(env, make_error(env, rc, msg));
  return false;
}

bool get_ctx(napi_env env, napi_value v, Ctx** out) {
  uint64_t h = 0;
  if (!handle_of(env, v, &h)) return throw_fmt(env, FMT_E_USAGE, "expected an engine context from open()");
  Lookup why;
  *out = ctx_of_handle(env, h, &why);
  if (why == Lookup::kForeign)
    return throw_fmt(env, FMT_E_USAGE, "engine context belongs to another thread (open one per worker)");
  if (*out == nullptr || (*out)->ctx == nullptr) return throw_fmt(env, FMT_E_USAGE, "engine context is closed");
  return true;
}

// Bytes of an ArrayBuffer, TypedArray or DataView (nullptr/0 for undefined or null).
bool get_bytes(napi_env env, napi_value v, const char* what, void** data, size_t* len) {
  *data = nullptr;
  *len = 0;
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_undefined || t == napi_null) return true;
  bool is;
  if (napi_is_typedarray(env, v, &is) == napi_ok && is) {
    napi_typedarray_type tt;
    size_t n, off;
    napi_value ab;
    napi_get_typedarray_info(env, v, &tt, &n, data, &ab, &off);
    size_t elt = 1;
    switch (tt) {
      case napi_int16_array: case napi_uint16_array: elt = 2; break;
      case napi_int32_array: case napi_uint32_array: case napi_float32_array: elt = 4; break;
      case napi_float64_array: case napi_bigint64_array: case napi_biguint64_array: elt = 8; break;
      default: elt = 1;
    }
    *len = n * elt;
    return true;
  }
  if (napi_is_arraybuffer(env, v, &is) == napi_ok && is) {
    napi_get_arraybuffer_info(env, v, data, len);
    return true;
  }
  if (napi_is_dataview(env, v, &is) == napi_ok && is) {
    napi_value ab;
    size_t off;
    napi_get_dataview_info(env, v, len, data, &ab, &off);
    return true;
  }
  return throw_fmt(env, FMT_E_USAGE, std::string(what) + ": expected an ArrayBuffer or TypedArray");
}

napi_value prop(napi_env env, napi_value obj, const char* name) {
  napi_value v = nullptr;
  napi_get_named_property(env, obj, name, &v);
  return v;
}

bool get_u32(napi_env env, napi_value v, const char* what, uint32_t* out) {
  if (napi_get_value_uint32(env, v, out) != napi_ok)
    return throw_fmt(env, FMT_E_USAGE, std::string(what) + ": expected a number");
  return true;
}

// ------------------------------------------------------------------------------------- open/close
napi_value Open(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  int32_t device = 0;
  if (argc >= 1) napi_get_value_int32(env, argv[0], &device);
  {
    std::lock_guard<std::mutex> lk(slots_mu());
    if (live_contexts() >= max_contexts()) {
      throw_fmt(env, FMT_E_CAPACITY,
                "open: " + std::to_string(max_contexts()) + " engine contexts are open (close() the ones no longer used)");
      return nullptr;
    }
  }
  fmt_config cfg;
  std::memset(&cfg, 0, sizeof cfg);
  cfg.device = device;
  fmt_ctx* ctx = nullptr;
  int rc = fmt_open(&cfg, &ctx);
  if (rc != FMT_OK) {
    std::string msg = ctx ? fmt_last_error(ctx) : "fmt_open failed";
    if (ctx) fmt_close(ctx);
    throw_fmt(env, rc, msg);
    return nullptr;
  }
  auto* c = new Ctx;
  c->ctx = ctx;
  uint64_t h;
  {
    std::lock_guard<std::mutex> lk(slots_mu());
    std::vector<Slot>& t = slots();
    size_t k = 0;
    while (k < t.size() && t[k].c != nullptr) k++;
    if (k == t.size()) t.emplace_back();
    t[k].c = c;
    t[k].env = env;
    h = static_cast<uint64_t>(k + 1) | (static_cast<uint64_t>(t[k].gen & kGenMask) << 32);
  }
  napi_value num;
  CHECK_NAPI(env, napi_create_double(env, static_cast<double>(h), &num));
  return num;
}

napi_value Close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  uint64_t h = 0;
  if (argc < 1 || !handle_of(env, argv[0], &h)) {
    throw_fmt(env, FMT_E_USAGE, "close: expected an engine context");
    return nullptr;
  }
  Lookup why;
  Ctx* c = ctx_of_handle(env, h, &why);
  if (why == Lookup::kForeign) {
    throw_fmt(env, FMT_E_USAGE, "close: engine context belongs to another thread");
    return nullptr;
  }
  if (c == nullptr) return nullptr;  // already closed: a no-op, as before
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "close: a replay is still running on this context");
    return nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(slots_mu());
    Slot& s = slots()[static_cast<uint32_t>(h & 0xffffffffu) - 1];
    s.c = nullptr;
    s.env = nullptr;
    s.gen++;
  }
  if (c->ctx) fmt_close(c->ctx);
  delete c;
  return nullptr;
}

// openContexts() -> number of engine contexts open in this process (diagnostics and tests)
napi_value OpenContexts(napi_env env, napi_callback_info) {
  napi_value v;
  uint32_t n;
  {
    std::lock_guard<std::mutex> lk(slots_mu());
    n = live_contexts();
  }
  CHECK_NAPI(env, napi_create_uint32(env, n, &v));
  return v;
}

napi_value DeviceInfo(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 1 || !get_ctx(env, argv[0], &c)) return nullptr;
  char buf[256];
  int rc = fmt_device_info(c->ctx, buf, sizeof buf);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  napi_value s;
  CHECK_NAPI(env, napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &s));
  return s;
}

napi_value Capacity(napi_env env, napi_callback_info) {
  uint32_t l = 0, ch = 0, p = 0;
  fmt_mt_capacity(&l, &ch, &p);
  napi_value o, v;
  napi_create_object(env, &o);
  napi_create_uint32(env, l, &v);
  napi_set_named_property(env, o, "leaves", v);
  napi_create_uint32(env, ch, &v);
  napi_set_named_property(env, o, "chars", v);
  napi_create_uint32(env, p, &v);
  napi_set_named_property(env, o, "props", v);
  return o;
}

napi_value Stats(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 1 || !get_ctx(env, argv[0], &c)) return nullptr;
  fmt_stats s;
  int rc = fmt_get_stats(c->ctx, &s);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  napi_value o, v;
  napi_create_object(env, &o);
  auto num = [&](const char* k, double x) {
    napi_create_double(env, x, &v);
    napi_set_named_property(env, o, k, v);
  };
  num("kernelMs", s.kernel_ms);
  num("totalMs", s.total_ms);
  num("ops", double(s.ops));
  num("docs", double(s.docs));
  num("bytesRead", double(s.bytes_read));
  num("bytesWritten", double(s.bytes_written));
  num("launches", double(s.launches));
  return o;
}

// ------------------------------------------------------------------------------- async replays
struct Job {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  Ctx* c = nullptr;
  std::vector<napi_ref> keep;  // input arrays stay alive (and unmoved) until Complete
  enum Kind { kMergeTree, kMap, kMapSparse, kSummarize } kind = kMergeTree;
  fmt_mt_batch mt;
  const fmt_map_op* map_ops = nullptr;
  uint64_t map_n_ops = 0;
  const uint64_t* map_offs = nullptr;
  uint32_t n_docs = 0, key_bound = 0;
  std::vector<uint8_t> out;  // headers, map slots, sparse counts
  std::vector<uint8_t> out2; // sparse entries
  // sparse map with the local client's events (fmt_map_pending_*): events, offsets, results
  const fmt_map_local_op* ev = nullptr;
  uint64_t n_ev = 0;
  const uint64_t* ev_offs = nullptr;
  std::vector<uint8_t> pcounts, pstatus, pentries;
  // summarizeLegacy: JSON-quoted keys and value texts (copied on the JS thread), chunk, threads
  std::vector<std::string> keys, values;
  uint32_t chunk = 0, threads = 0;
  fmt_summary_timing timing{};
  int rc = FMT_OK;
  std::string err;
};

void Execute(napi_env, void* p) {  // libuv worker thread: no N-API calls here
  auto* j = static_cast<Job*>(p);
  fmt_ctx* ctx = j->c->ctx;
  if (j->kind == Job::kMap) {
    j->rc = fmt_map_load(ctx, j->map_ops, j->map_n_ops, j->map_offs, j->n_docs, j->key_bound);
    if (j->rc == FMT_OK) j->rc = fmt_map_run(ctx);
    if (j->rc == FMT_OK) {
      j->out.resize(size_t(j->n_docs) * j->key_bound * sizeof(fmt_map_slot));
      j->rc = fmt_map_fetch(ctx, reinterpret_cast<fmt_map_slot*>(j->out.data()));
    }
  } else if (j->kind == Job::kMapSparse) {
    j->rc = fmt_map_load_sparse(ctx, j->map_ops, j->map_n_ops, j->map_offs, j->n_docs, j->key_bound);
    if (j->rc == FMT_OK) j->rc = fmt_map_run_sparse(ctx);
    uint64_t n = 0;
    j->out.resize(size_t(j->n_docs) * sizeof(uint32_t));
    if (j->rc == FMT_OK)  // sizes first (counts + total), then the packed entries
      j->rc = fmt_map_fetch_sparse(ctx, reinterpret_cast<uint32_t*>(j->out.data()), nullptr, 0, &n);
    if (j->rc == FMT_OK) {
      j->out2.resize(size_t(n) * sizeof(fmt_map_entry));
      j->rc = fmt_map_fetch_sparse(ctx, reinterpret_cast<uint32_t*>(j->out.data()),
                                   reinterpret_cast<fmt_map_entry*>(j->out2.data()), n, &n);
    }
    if (j->rc == FMT_OK && j->ev_offs != nullptr) {  // the local client's optimistic view
      j->rc = fmt_map_pending_run(ctx, j->ev, j->n_ev, j->ev_offs);
      uint64_t np = 0;
      j->pcounts.resize(size_t(j->n_docs) * sizeof(uint32_t));
      j->pstatus.resize(size_t(j->n_docs) * sizeof(int32_t));
      auto* pc = reinterpret_cast<uint32_t*>(j->pcounts.data());
      auto* ps = reinterpret_cast<int32_t*>(j->pstatus.data());
      if (j->rc == FMT_OK) j->rc = fmt_map_pending_fetch(ctx, pc, ps, nullptr, 0, &np);
      if (j->rc == FMT_OK) {
        j->pentries.resize(size_t(np) * sizeof(fmt_map_entry));
        j->rc = fmt_map_pending_fetch(ctx, pc, ps, reinterpret_cast<fmt_map_entry*>(j->pentries.data()), np, &np);
      }
    }
  } else if (j->kind == Job::kSummarize) {
    std::vector<const char*> k, v;
    for (const auto& x : j->keys) k.push_back(x.c_str());
    for (const auto& x : j->values) v.push_back(x.c_str());
    j->rc = fmt_mt_summarize_legacy(ctx, k.data(), uint32_t(k.size()), v.data(), uint32_t(v.size()), j->chunk,
                                    j->threads, &j->timing);
  } else {
    j->rc = fmt_mt_load(ctx, &j->mt);
    if (j->rc == FMT_OK) j->rc = fmt_mt_run(ctx);
    if (j->rc == FMT_OK) {
      j->out.resize(size_t(j->n_docs) * sizeof(fmt_mt_doc_result));
      j->rc = fmt_mt_fetch_headers(ctx, reinterpret_cast<fmt_mt_doc_result*>(j->out.data()));
    }
  }
  if (j->rc != FMT_OK) j->err = fmt_last_error(ctx);
}

void Complete(napi_env env, napi_status, void* p) {  // JS thread
  auto* j = static_cast<Job*>(p);
  j->c->busy = false;
  auto buffer = [&](const std::vector<uint8_t>& bytes) {
    void* data = nullptr;
    napi_value ab;
    napi_create_arraybuffer(env, bytes.size(), &data, &ab);
    if (!bytes.empty()) std::memcpy(data, bytes.data(), bytes.size());
    return ab;
  };
  if (j->rc != FMT_OK) {
    napi_reject_deferred(env, j->deferred, make_error(env, j->rc, j->err));
  } else if (j->kind == Job::kMapSparse) {
    napi_value o;
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "counts", buffer(j->out));
    napi_set_named_property(env, o, "entries", buffer(j->out2));
    if (j->ev_offs != nullptr) {
      napi_value p;
      napi_create_object(env, &p);
      napi_set_named_property(env, p, "counts", buffer(j->pcounts));
      napi_set_named_property(env, p, "status", buffer(j->pstatus));
      napi_set_named_property(env, p, "entries", buffer(j->pentries));
      napi_set_named_property(env, o, "pending", p);
    }
    napi_resolve_deferred(env, j->deferred, o);
  } else if (j->kind == Job::kSummarize) {
    napi_value o, v;
    napi_create_object(env, &o);
    auto num = [&](const char* k, double x) {
      napi_create_double(env, x, &v);
      napi_set_named_property(env, o, k, v);
    };
    num("kernelMs", j->timing.kernel_ms);
    num("fetchMs", j->timing.fetch_ms);
    num("formatMs", j->timing.format_ms);
    num("bytes", double(j->timing.bytes));
    num("threads", double(j->timing.threads));
    napi_resolve_deferred(env, j->deferred, o);
  } else {
    napi_resolve_deferred(env, j->deferred, buffer(j->out));
  }
  for (napi_ref r : j->keep) napi_delete_reference(env, r);
  napi_delete_async_work(env, j->work);
  delete j;
}

bool keep_array(napi_env env, Job* j, napi_value v) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t != napi_object) return true;
  napi_ref r;
  if (napi_create_reference(env, v, 1, &r) != napi_ok) return false;
  j->keep.push_back(r);
  return true;
}

napi_value queue(napi_env env, Job* j, napi_value /*ctx: a number handle, kept alive by the slot table*/, const char* name) {
  napi_value promise, res_name;
  napi_create_promise(env, &j->deferred, &promise);
  napi_create_string_utf8(env, name, NAPI_AUTO_LENGTH, &res_name);
  napi_create_async_work(env, nullptr, res_name, Execute, Complete, j, &j->work);
  j->c->busy = true;
  napi_queue_async_work(env, j->work);
  return promise;
}

// replayMergeTree(ctx, {ops, docOpOffsets, text, docInit, propsOff, propsKv, snapshots?, snapshotSegs?})
napi_value ReplayMergeTree(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 2 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "replayMergeTree: a replay is already running on this context");
    return nullptr;
  }
  napi_value b = argv[1];
  const char* names[] = {"ops", "docOpOffsets", "text", "docInit", "propsOff", "propsKv"};
  void* d[6];
  size_t n[6];
  for (int i = 0; i < 6; ++i)
    if (!get_bytes(env, prop(env, b, names[i]), names[i], &d[i], &n[i])) return nullptr;
  if (n[0] % sizeof(fmt_mt_op) || n[1] < 8 || n[1] % 8 || n[4] < 4 || n[4] % 4 || n[5] % 4 || n[2] % 2) {
    throw_fmt(env, FMT_E_USAGE, "replayMergeTree: buffer sizes do not match the fmt_mt_* record layouts");
    return nullptr;
  }
  uint32_t n_docs = uint32_t(n[1] / 8 - 1);
  if (d[3] && n[3] != size_t(n_docs) * 8) {
    throw_fmt(env, FMT_E_USAGE, "replayMergeTree: docInit must hold (offset, len) per document");
    return nullptr;
  }
  auto* j = new Job;
  j->c = c;
  j->n_docs = n_docs;
  std::memset(&j->mt, 0, sizeof j->mt);
  j->mt.ops = static_cast<const fmt_mt_op*>(d[0]);
  j->mt.n_ops = n[0] / sizeof(fmt_mt_op);
  j->mt.doc_op_offsets = static_cast<const uint64_t*>(d[1]);
  j->mt.n_docs = n_docs;
  j->mt.text = static_cast<const uint16_t*>(d[2]);
  j->mt.text_len = n[2] / 2;
  j->mt.doc_init = static_cast<const uint32_t*>(d[3]);
  j->mt.props_off = static_cast<const uint32_t*>(d[4]);
  j->mt.n_props_ops = uint32_t(n[4] / 4 - 1);
  j->mt.props_kv = static_cast<const uint32_t*>(d[5]);
  // optional summary loads (f3): snapshots (fmt_mt_snapshot_doc per doc) + snapshotSegs
  void *sd, *ss;
  size_t nsd, nss;
  if (!get_bytes(env, prop(env, b, "snapshots"), "snapshots", &sd, &nsd) ||
      !get_bytes(env, prop(env, b, "snapshotSegs"), "snapshotSegs", &ss, &nss)) {
    delete j;
    return nullptr;
  }
  if (sd != nullptr) {
    if (nsd != size_t(n_docs) * sizeof(fmt_mt_snapshot_doc) || nss % sizeof(fmt_mt_snapshot_seg)) {
      delete j;
      throw_fmt(env, FMT_E_USAGE, "replayMergeTree: snapshots must hold one fmt_mt_snapshot_doc per document");
      return nullptr;
    }
    j->mt.snapshots = static_cast<const fmt_mt_snapshot_doc*>(sd);
    j->mt.snapshot_segs = static_cast<const fmt_mt_snapshot_seg*>(ss);
    j->mt.n_snapshot_segs = nss / sizeof(fmt_mt_snapshot_seg);
    keep_array(env, j, prop(env, b, "snapshots"));
    keep_array(env, j, prop(env, b, "snapshotSegs"));
    // optional SnapshotV1 merge info: snapshotInfo (fmt_mt_snapshot_info per segment) + snapshotStamps
    void *si, *st;
    size_t nsi, nst;
    if (!get_bytes(env, prop(env, b, "snapshotInfo"), "snapshotInfo", &si, &nsi) ||
        !get_bytes(env, prop(env, b, "snapshotStamps"), "snapshotStamps", &st, &nst)) {
      delete j;
      return nullptr;
    }
    if (si != nullptr) {
      if (nsi != j->mt.n_snapshot_segs * sizeof(fmt_mt_snapshot_info) || nst % sizeof(fmt_mt_stamp)) {
        delete j;
        throw_fmt(env, FMT_E_USAGE, "replayMergeTree: snapshotInfo must hold one fmt_mt_snapshot_info per segment");
        return nullptr;
      }
      j->mt.snapshot_info = static_cast<const fmt_mt_snapshot_info*>(si);
      j->mt.snapshot_stamps = static_cast<const fmt_mt_stamp*>(st);
      j->mt.n_snapshot_stamps = nst / sizeof(fmt_mt_stamp);
      keep_array(env, j, prop(env, b, "snapshotInfo"));
      if (st != nullptr) keep_array(env, j, prop(env, b, "snapshotStamps"));
    }
  }
  // optional annotate-adjust: adjusts (fmt_mt_adjust rows) + valueNum (one double per value id)
  void *adj, *vn;
  size_t nadj, nvn;
  if (!get_bytes(env, prop(env, b, "adjusts"), "adjusts", &adj, &nadj) ||
      !get_bytes(env, prop(env, b, "valueNum"), "valueNum", &vn, &nvn)) {
    delete j;
    return nullptr;
  }
  if (adj != nullptr) {
    if (nadj % sizeof(fmt_mt_adjust) || vn == nullptr || nvn % sizeof(double)) {
      delete j;
      throw_fmt(env, FMT_E_USAGE, "replayMergeTree: adjusts must hold fmt_mt_adjust rows, valueNum one double per value");
      return nullptr;
    }
    j->mt.adjusts = static_cast<const fmt_mt_adjust*>(adj);
    j->mt.n_adjusts = uint32_t(nadj / sizeof(fmt_mt_adjust));
    j->mt.value_num = static_cast<const double*>(vn);
    j->mt.n_values = uint32_t(nvn / sizeof(double));
    keep_array(env, j, prop(env, b, "adjusts"));
    keep_array(env, j, prop(env, b, "valueNum"));
  }
  // optional document-local value ids: docValueBase (n_docs + 1 uint32, fmt.h doc_value_base)
  void* vb;
  size_t nvb;
  if (!get_bytes(env, prop(env, b, "docValueBase"), "docValueBase", &vb, &nvb)) {
    delete j;
    return nullptr;
  }
  if (vb != nullptr) {
    if (nvb != (static_cast<size_t>(j->mt.n_docs) + 1) * sizeof(uint32_t)) {
      delete j;
      throw_fmt(env, FMT_E_USAGE, "replayMergeTree: docValueBase must hold n_docs + 1 uint32 entries");
      return nullptr;
    }
    j->mt.doc_value_base = static_cast<const uint32_t*>(vb);
    keep_array(env, j, prop(env, b, "docValueBase"));
  }
  // optional legacy relative positions: relpos (fmt_mt_relpos rows) + markerIdKey
  void* rp;
  size_t nrp;
  if (!get_bytes(env, prop(env, b, "relpos"), "relpos", &rp, &nrp)) {
    delete j;
    return nullptr;
  }
  j->mt.marker_id_key = FMT_MT_NO_MARKER;
  if (rp != nullptr) {
    if (nrp % sizeof(fmt_mt_relpos)) {
      delete j;
      throw_fmt(env, FMT_E_USAGE, "replayMergeTree: relpos must hold whole fmt_mt_relpos rows");
      return nullptr;
    }
    j->mt.relpos = static_cast<const fmt_mt_relpos*>(rp);
    j->mt.n_relpos = uint32_t(nrp / sizeof(fmt_mt_relpos));
    if (!get_u32(env, prop(env, b, "markerIdKey"), "markerIdKey", &j->mt.marker_id_key)) {
      delete j;
      return nullptr;
    }
    keep_array(env, j, prop(env, b, "relpos"));
  }
  for (int i = 0; i < 6; ++i) keep_array(env, j, prop(env, b, names[i]));
  return queue(env, j, argv[0], "fmtReplayMergeTree");
}

// replayMap(ctx, {ops, docOpOffsets, keyBound})
napi_value ReplayMap(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 2 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "replayMap: a replay is already running on this context");
    return nullptr;
  }
  napi_value b = argv[1];
  void *ops, *offs;
  size_t n_ops_b, n_offs_b;
  uint32_t key_bound;
  if (!get_bytes(env, prop(env, b, "ops"), "ops", &ops, &n_ops_b)) return nullptr;
  if (!get_bytes(env, prop(env, b, "docOpOffsets"), "docOpOffsets", &offs, &n_offs_b)) return nullptr;
  if (!get_u32(env, prop(env, b, "keyBound"), "keyBound", &key_bound)) return nullptr;
  if (n_ops_b % sizeof(fmt_map_op) || n_offs_b < 8 || n_offs_b % 8 || key_bound == 0) {
    throw_fmt(env, FMT_E_USAGE, "replayMap: buffer sizes do not match the fmt_map_* record layouts");
    return nullptr;
  }
  auto* j = new Job;
  j->c = c;
  j->kind = Job::kMap;
  j->map_ops = static_cast<const fmt_map_op*>(ops);
  j->map_n_ops = n_ops_b / sizeof(fmt_map_op);
  j->map_offs = static_cast<const uint64_t*>(offs);
  j->n_docs = uint32_t(n_offs_b / 8 - 1);
  j->key_bound = key_bound;
  keep_array(env, j, prop(env, b, "ops"));
  keep_array(env, j, prop(env, b, "docOpOffsets"));
  return queue(env, j, argv[0], "fmtReplayMap");
}

// replayMapSparse(ctx, {ops, docOpOffsets, keyBound, localOps?, localOffsets?}) -> Promise<{counts,
// entries, pending?}>: the sparse LWW path (key pools of any size): counts = n_docs u32 live-entry
// counts, entries = fmt_map_entry records of all documents packed in document order, each
// document's in JS Map insertion order; with the local client's events, pending = {counts, status,
// entries} of the optimistic view (fmt_map_pending_run / fetch).
napi_value ReplayMapSparse(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 2 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "replayMapSparse: a replay is already running on this context");
    return nullptr;
  }
  napi_value b = argv[1];
  void *ops, *offs;
  size_t n_ops_b, n_offs_b;
  uint32_t key_bound;
  if (!get_bytes(env, prop(env, b, "ops"), "ops", &ops, &n_ops_b)) return nullptr;
  if (!get_bytes(env, prop(env, b, "docOpOffsets"), "docOpOffsets", &offs, &n_offs_b)) return nullptr;
  if (!get_u32(env, prop(env, b, "keyBound"), "keyBound", &key_bound)) return nullptr;
  if (n_ops_b % sizeof(fmt_map_op) || n_offs_b < 8 || n_offs_b % 8 || key_bound == 0) {
    throw_fmt(env, FMT_E_USAGE, "replayMapSparse: buffer sizes do not match the fmt_map_* record layouts");
    return nullptr;
  }
  auto* j = new Job;
  j->c = c;
  j->kind = Job::kMapSparse;
  j->map_ops = static_cast<const fmt_map_op*>(ops);
  j->map_n_ops = n_ops_b / sizeof(fmt_map_op);
  j->map_offs = static_cast<const uint64_t*>(offs);
  j->n_docs = uint32_t(n_offs_b / 8 - 1);
  j->key_bound = key_bound;
  // optional: the local client's events (localOps: fmt_map_local_op records, localOffsets: n_docs + 1)
  void *ev, *eo;
  size_t n_ev_b, n_eo_b;
  if (!get_bytes(env, prop(env, b, "localOps"), "localOps", &ev, &n_ev_b) ||
      !get_bytes(env, prop(env, b, "localOffsets"), "localOffsets", &eo, &n_eo_b)) {
    delete j;
    return nullptr;
  }
  if (eo != nullptr) {
    if (n_ev_b % sizeof(fmt_map_local_op) || n_eo_b != (size_t(j->n_docs) + 1) * 8) {
      delete j;
      throw_fmt(env, FMT_E_USAGE, "replayMapSparse: localOps / localOffsets do not match the fmt_map_local_op layout");
      return nullptr;
    }
    j->ev = static_cast<const fmt_map_local_op*>(ev);
    j->n_ev = n_ev_b / sizeof(fmt_map_local_op);
    j->ev_offs = static_cast<const uint64_t*>(eo);
    keep_array(env, j, prop(env, b, "localOps"));
    keep_array(env, j, prop(env, b, "localOffsets"));
  }
  keep_array(env, j, prop(env, b, "ops"));
  keep_array(env, j, prop(env, b, "docOpOffsets"));
  return queue(env, j, argv[0], "fmtReplayMapSparse");
}

bool get_strings(napi_env env, napi_value arr, const char* what, std::vector<std::string>* out) {
  bool is = false;
  uint32_t n = 0;
  if (napi_is_array(env, arr, &is) != napi_ok || !is || napi_get_array_length(env, arr, &n) != napi_ok)
    return throw_fmt(env, FMT_E_USAGE, std::string(what) + ": expected an array of strings");
  out->resize(n);
  for (uint32_t i = 0; i < n; i++) {
    napi_value v;
    size_t len = 0;
    napi_get_element(env, arr, i, &v);
    if (napi_get_value_string_utf8(env, v, nullptr, 0, &len) != napi_ok)
      return throw_fmt(env, FMT_E_USAGE, std::string(what) + ": expected an array of strings");
    (*out)[i].resize(len + 1);
    napi_get_value_string_utf8(env, v, &(*out)[i][0], len + 1, &len);
    (*out)[i].resize(len);
  }
  return true;
}

// summarizeLegacy(ctx, quotedKeys, values, chunk, threads) -> Promise<timing>: legacy summaries of every
// document of the last merge-tree replay (fmt_mt_summarize_legacy: device merge, host JSON threads);
// read them with summaryBlobs.
napi_value SummarizeLegacy(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 5 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "summarizeLegacy: a replay is running on this context");
    return nullptr;
  }
  auto* j = new Job;
  j->c = c;
  j->kind = Job::kSummarize;
  if (!get_strings(env, argv[1], "keys", &j->keys) || !get_strings(env, argv[2], "values", &j->values) ||
      !get_u32(env, argv[3], "chunk", &j->chunk) || !get_u32(env, argv[4], "threads", &j->threads)) {
    delete j;
    return nullptr;
  }
  return queue(env, j, argv[0], "fmtSummarizeLegacy");
}

// summaryBlobs(ctx, doc) -> {header, body?}: document doc's blobs of the last summarizeLegacy
// (throws with the document's replay status, or FMT_E_UNSUPPORTED, when it has none).
napi_value SummaryBlobs(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 2 || !get_ctx(env, argv[0], &c)) return nullptr;
  uint32_t doc;
  if (!get_u32(env, argv[1], "doc", &doc)) return nullptr;
  const char *h = nullptr, *b = nullptr;
  size_t hl = 0, bl = 0;
  int rc = fmt_mt_summary_blobs(c->ctx, doc, &h, &hl, &b, &bl);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  napi_value o, v;
  napi_create_object(env, &o);
  CHECK_NAPI(env, napi_create_string_utf8(env, h, hl, &v));
  napi_set_named_property(env, o, "header", v);
  if (bl) {
    CHECK_NAPI(env, napi_create_string_utf8(env, b, bl, &v));
    napi_set_named_property(env, o, "body", v);
  }
  return o;
}

// fetchDoc(ctx, doc, nLeaves, nChars, nProps) -> {leaves: ArrayBuffer, chars: ArrayBuffer, props: ArrayBuffer}
napi_value FetchDoc(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 5 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchDoc: a replay is running on this context");
    return nullptr;
  }
  uint32_t doc, nl, nc, np;
  if (!get_u32(env, argv[1], "doc", &doc) || !get_u32(env, argv[2], "nLeaves", &nl) ||
      !get_u32(env, argv[3], "nChars", &nc) || !get_u32(env, argv[4], "nProps", &np))
    return nullptr;
  void *l, *ch, *pr;
  napi_value lv, cv, pv, o;
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(nl) * sizeof(fmt_mt_leaf), &l, &lv));
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(nc) * 2, &ch, &cv));
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(np) * sizeof(fmt_mt_propset), &pr, &pv));
  int rc = fmt_mt_fetch_doc(c->ctx, doc, static_cast<fmt_mt_leaf*>(l), nl, static_cast<uint16_t*>(ch), nc,
                            static_cast<fmt_mt_propset*>(pr), np);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  napi_create_object(env, &o);
  napi_set_named_property(env, o, "leaves", lv);
  napi_set_named_property(env, o, "chars", cv);
  napi_set_named_property(env, o, "props", pv);
  return o;
}

// fetchCatchup(ctx, doc, n) -> ArrayBuffer of n fmt_mt_catchup_range records
napi_value FetchCatchup(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 3 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchCatchup: a replay is running on this context");
    return nullptr;
  }
  uint32_t doc, n;
  if (!get_u32(env, argv[1], "doc", &doc) || !get_u32(env, argv[2], "n", &n)) return nullptr;
  void* p;
  napi_value ab;
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(n) * sizeof(fmt_mt_catchup_range), &p, &ab));
  int rc = fmt_mt_fetch_catchup(c->ctx, doc, static_cast<fmt_mt_catchup_range*>(p), n);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  return ab;
}

// fetchCatchupAll(ctx, nDocs) -> {offsets: Float64Array(nDocs + 1), ranges: ArrayBuffer}
// (fmt_mt_fetch_catchup_all; nDocs = the loaded batch's document count)
napi_value FetchCatchupAll(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  uint32_t nd;
  if (argc < 2 || !get_ctx(env, argv[0], &c) || !get_u32(env, argv[1], "nDocs", &nd)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchCatchupAll: a replay is running on this context");
    return nullptr;
  }
  std::vector<uint64_t> offs(size_t(nd) + 1);
  int rc = fmt_mt_fetch_catchup_all(c->ctx, offs.data(), nullptr, 0);
  void* p = nullptr;
  napi_value ab;
  if (rc == FMT_OK) {
    CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(offs[nd]) * sizeof(fmt_mt_catchup_range), &p, &ab));
    rc = fmt_mt_fetch_catchup_all(c->ctx, offs.data(), static_cast<fmt_mt_catchup_range*>(p), offs[nd]);
  }
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  void* q;
  napi_value ob, oa;
  CHECK_NAPI(env, napi_create_arraybuffer(env, (size_t(nd) + 1) * sizeof(double), &q, &ob));
  for (size_t d = 0; d <= nd; d++) static_cast<double*>(q)[d] = static_cast<double>(offs[d]);
  CHECK_NAPI(env, napi_create_typedarray(env, napi_float64_array, size_t(nd) + 1, ob, 0, &oa));
  napi_value o;
  napi_create_object(env, &o);
  napi_set_named_property(env, o, "offsets", oa);
  napi_set_named_property(env, o, "ranges", ab);
  return o;
}

// fetchRemoveOrder(ctx, doc, n) -> ArrayBuffer of n fmt_mt_remove_order records (SnapshotV1)
napi_value FetchRemoveOrder(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 3 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchRemoveOrder: a replay is running on this context");
    return nullptr;
  }
  uint32_t doc, n;
  if (!get_u32(env, argv[1], "doc", &doc) || !get_u32(env, argv[2], "n", &n)) return nullptr;
  void* p;
  napi_value ab;
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(n) * sizeof(fmt_mt_remove_order), &p, &ab));
  int rc = fmt_mt_fetch_remove_order(c->ctx, doc, static_cast<fmt_mt_remove_order*>(p), n);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  return ab;
}

// fetchNumbers(ctx, doc) -> Float64Array of the document's computed annotate-adjust numbers
// (value ids FMT_MT_VALUE_COMPUTED + index)
napi_value FetchNumbers(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 2 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchNumbers: a replay is running on this context");
    return nullptr;
  }
  uint32_t doc, n = 0;
  if (!get_u32(env, argv[1], "doc", &doc)) return nullptr;
  int rc = fmt_mt_fetch_numbers(c->ctx, doc, nullptr, 0, &n);
  void* p;
  napi_value ab, arr;
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(n) * sizeof(double), &p, &ab));
  if (rc == FMT_OK && n) rc = fmt_mt_fetch_numbers(c->ctx, doc, static_cast<double*>(p), n, &n);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  CHECK_NAPI(env, napi_create_typedarray(env, napi_float64_array, n, ab, 0, &arr));
  return arr;
}

// fetchLegacyProps(ctx, doc, nLeaves) -> Uint16Array: per leaf, the prop-set id of getAtSeq(minSeq)
napi_value FetchLegacyProps(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 3 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchLegacyProps: a replay is running on this context");
    return nullptr;
  }
  uint32_t doc, n;
  if (!get_u32(env, argv[1], "doc", &doc) || !get_u32(env, argv[2], "nLeaves", &n)) return nullptr;
  void* p;
  napi_value ab, arr;
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(n) * sizeof(uint16_t), &p, &ab));
  const int rc = n ? fmt_mt_fetch_legacy_props(c->ctx, doc, static_cast<uint16_t*>(p), n) : FMT_OK;
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  CHECK_NAPI(env, napi_create_typedarray(env, napi_uint16_array, n, ab, 0, &arr));
  return arr;
}

// fetchRmClientsHi(ctx, doc, nLeaves) -> BigUint64Array: per leaf, its remove clients 64..127 (bit c - 64)
napi_value FetchRmClientsHi(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 3 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchRmClientsHi: a replay is running on this context");
    return nullptr;
  }
  uint32_t doc, n;
  if (!get_u32(env, argv[1], "doc", &doc) || !get_u32(env, argv[2], "nLeaves", &n)) return nullptr;
  void* p;
  napi_value ab, arr;
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(n) * sizeof(uint64_t), &p, &ab));
  const int rc = n ? fmt_mt_fetch_rm_clients_hi(c->ctx, doc, static_cast<uint64_t*>(p), n) : FMT_OK;
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  CHECK_NAPI(env, napi_create_typedarray(env, napi_biguint64_array, n, ab, 0, &arr));
  return arr;
}

napi_value FetchRegen(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK_NAPI(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  Ctx* c;
  if (argc < 2 || !get_ctx(env, argv[0], &c)) return nullptr;
  if (c->busy) {
    throw_fmt(env, FMT_E_USAGE, "fetchRegen: a replay is running on this context");
    return nullptr;
  }
  uint32_t doc;
  if (!get_u32(env, argv[1], "doc", &doc)) return nullptr;
  uint32_t n = 0, nt = 0;
  int rc = fmt_mt_fetch_regen(c->ctx, doc, nullptr, 0, nullptr, 0, &n, &nt);
  void *po, *pt;
  napi_value abo, abt, arr, out;
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(n) * sizeof(fmt_mt_op), &po, &abo));
  CHECK_NAPI(env, napi_create_arraybuffer(env, size_t(nt) * sizeof(uint16_t), &pt, &abt));
  if (rc == FMT_OK && (n || nt))
    rc = fmt_mt_fetch_regen(c->ctx, doc, static_cast<fmt_mt_op*>(po), n, static_cast<uint16_t*>(pt), nt, &n, &nt);
  if (rc != FMT_OK) {
    throw_fmt(env, rc, fmt_last_error(c->ctx));
    return nullptr;
  }
  CHECK_NAPI(env, napi_create_typedarray(env, napi_uint16_array, nt, abt, 0, &arr));
  CHECK_NAPI(env, napi_create_object(env, &out));
  CHECK_NAPI(env, napi_set_named_property(env, out, "ops", abo));
  CHECK_NAPI(env, napi_set_named_property(env, out, "text", arr));
  return out;
}

// FMT_NAPI_BACKTRACE=1: a SIGSEGV prints the native stack to stderr before the default action
// (diagnostics for crashes inside the addon or the HIP runtime under node). backtrace() is called
// once before the handler is installed (it loads libgcc's unwinder, which allocates), the handler
// runs on its own stack (a fault from a stack overflow still reports) and is reset on entry.
void segvTrace(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  raise(sig);  // SA_RESETHAND: the default action now
}

void install_segv_trace() {
  void* warm[2];
  backtrace(warm, 2);
  static std::vector<char>* alt = new std::vector<char>(1 << 16);
  stack_t ss;
  std::memset(&ss, 0, sizeof ss);
  ss.ss_sp = alt->data();
  ss.ss_size = alt->size();
  sigaltstack(&ss, nullptr);
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_handler = segvTrace;
  sa.sa_flags = SA_RESETHAND | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, nullptr);
}

napi_value Init(napi_env env, napi_value exports) {
  if (std::getenv("FMT_NAPI_BACKTRACE") != nullptr) install_segv_trace();
  napi_add_env_cleanup_hook(env, close_env_at_teardown, env);
  napi_property_descriptor fns[] = {
      {"open", nullptr, Open, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"close", nullptr, Close, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"openContexts", nullptr, OpenContexts, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"deviceInfo", nullptr, DeviceInfo, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"capacity", nullptr, Capacity, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"stats", nullptr, Stats, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"replayMergeTree", nullptr, ReplayMergeTree, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"replayMap", nullptr, ReplayMap, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchDoc", nullptr, FetchDoc, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchCatchup", nullptr, FetchCatchup, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchCatchupAll", nullptr, FetchCatchupAll, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchRemoveOrder", nullptr, FetchRemoveOrder, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchNumbers", nullptr, FetchNumbers, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchLegacyProps", nullptr, FetchLegacyProps, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchRmClientsHi", nullptr, FetchRmClientsHi, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"fetchRegen", nullptr, FetchRegen, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"replayMapSparse", nullptr, ReplayMapSparse, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"summarizeLegacy", nullptr, SummarizeLegacy, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"summaryBlobs", nullptr, SummaryBlobs, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
  };
  napi_define_properties(env, exports, sizeof fns / sizeof fns[0], fns);
  napi_value sizes, v;
  napi_create_object(env, &sizes);
  auto sz = [&](const char* k, size_t x) {
    napi_create_uint32(env, uint32_t(x), &v);
    napi_set_named_property(env, sizes, k, v);
  };
  sz("mtOp", sizeof(fmt_mt_op));
  sz("mapOp", sizeof(fmt_map_op));
  sz("leaf", sizeof(fmt_mt_leaf));
  sz("docResult", sizeof(fmt_mt_doc_result));
  sz("propset", sizeof(fmt_mt_propset));
  sz("mapSlot", sizeof(fmt_map_slot));
  sz("catchupRange", sizeof(fmt_mt_catchup_range));
  sz("mapEntry", sizeof(fmt_map_entry));
  sz("adjust", sizeof(fmt_mt_adjust));
  napi_set_named_property(env, exports, "sizes", sizes);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
