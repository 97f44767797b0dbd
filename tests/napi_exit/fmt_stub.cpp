// A libfmt.so stand-in with no device (TEST INFRASTRUCTURE ONLY): it exports every entry point
// include/fmt.h declares so fmt_napi.node links and loads on a CPU-only machine, and does just
// enough for the addon's context and async-work paths (open / replay / fetch headers / close) to run
// end to end. Replays replay nothing: headers come back zeroed. Everything else returns
// FMT_E_UNSUPPORTED. Used by tests/test_napi_exit_cpu.py to exercise the addon's lifetime and exit
// paths (env cleanup hooks, worker_threads, pending promises at exit) under AddressSanitizer; it is
// never loaded by the product path.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "fmt.h"

struct fmt_ctx {
  uint32_t n_docs = 0, key_bound = 0;
  std::string err;
  uint64_t magic = 0x5354554246544dULL;
};

namespace {
int unsupported(fmt_ctx* c, const char* what) {
  if (c) c->err = std::string(what) + ": not available in the CPU stub";
  return FMT_E_UNSUPPORTED;
}
bool live(const fmt_ctx* c) { return c != nullptr && c->magic == 0x5354554246544dULL; }
}  // namespace

extern "C" {
int fmt_open(const fmt_config* cfg, fmt_ctx** out) {
  if (!cfg || !out) return FMT_E_USAGE;
  *out = new (std::nothrow) fmt_ctx;
  return *out ? FMT_OK : FMT_E_DEVICE;
}
void fmt_close(fmt_ctx* ctx) {
  if (!ctx) return;
  if (!live(ctx)) std::abort();  // a double close or a stale pointer: fail loudly
  ctx->magic = 0;
  delete ctx;
}
const char* fmt_last_error(const fmt_ctx* ctx) { return live(ctx) ? ctx->err.c_str() : "no context"; }
int fmt_sync(fmt_ctx* ctx) { return live(ctx) ? FMT_OK : FMT_E_USAGE; }
int fmt_get_stats(const fmt_ctx* ctx, fmt_stats* out) {
  if (!live(ctx) || !out) return FMT_E_USAGE;
  std::memset(out, 0, sizeof *out);
  out->docs = ctx->n_docs;
  return FMT_OK;
}
int fmt_device_info(fmt_ctx* ctx, char* buf, size_t cap) {
  if (!live(ctx) || !buf || cap == 0) return FMT_E_USAGE;
  std::strncpy(buf, "cpu-stub (no device)", cap - 1);
  buf[cap - 1] = 0;
  return FMT_OK;
}
int fmt_mt_summarize_legacy(fmt_ctx* ctx, const char* const*, uint32_t, const char* const*, uint32_t, uint32_t, uint32_t,
                            fmt_summary_timing*) {
  return unsupported(ctx, "fmt_mt_summarize_legacy");
}
int fmt_mt_summary_blobs(fmt_ctx* ctx, uint32_t, const char**, size_t*, const char**, size_t*) {
  return unsupported(ctx, "fmt_mt_summary_blobs");
}
int fmt_map_load(fmt_ctx* ctx, const fmt_map_op*, uint64_t, const uint64_t*, uint32_t n_docs, uint32_t key_bound) {
  if (!live(ctx)) return FMT_E_USAGE;
  ctx->n_docs = n_docs;
  ctx->key_bound = key_bound;
  return FMT_OK;
}
int fmt_map_run(fmt_ctx* ctx) { return live(ctx) ? FMT_OK : FMT_E_USAGE; }
int fmt_map_fetch(fmt_ctx* ctx, fmt_map_slot* out) {
  if (!live(ctx)) return FMT_E_USAGE;
  for (uint64_t i = 0; i < uint64_t(ctx->n_docs) * ctx->key_bound; i++) out[i] = fmt_map_slot{FMT_MAP_ABSENT, 0};
  return FMT_OK;
}
int fmt_map_replay_device(fmt_ctx* ctx, const fmt_map_op*, const uint64_t*, uint32_t, uint32_t, fmt_map_slot*) {
  return unsupported(ctx, "fmt_map_replay_device");
}
int fmt_map_check(fmt_ctx* ctx) { return live(ctx) ? FMT_OK : FMT_E_USAGE; }
int fmt_map_load_sparse(fmt_ctx* ctx, const fmt_map_op*, uint64_t, const uint64_t*, uint32_t, uint32_t) {
  return unsupported(ctx, "fmt_map_load_sparse");
}
int fmt_map_run_sparse(fmt_ctx* ctx) { return unsupported(ctx, "fmt_map_run_sparse"); }
int fmt_map_fetch_sparse(fmt_ctx* ctx, uint32_t*, fmt_map_entry*, uint64_t, uint64_t*) {
  return unsupported(ctx, "fmt_map_fetch_sparse");
}
int fmt_map_pending_run(fmt_ctx* ctx, const fmt_map_local_op*, uint64_t, const uint64_t*) {
  return unsupported(ctx, "fmt_map_pending_run");
}
int fmt_map_pending_fetch(fmt_ctx* ctx, uint32_t*, int32_t*, fmt_map_entry*, uint64_t, uint64_t*) {
  return unsupported(ctx, "fmt_map_pending_fetch");
}
int fmt_mt_load(fmt_ctx* ctx, const fmt_mt_batch* batch) {
  if (!live(ctx) || !batch) return FMT_E_USAGE;
  ctx->n_docs = batch->n_docs;
  return FMT_OK;
}
int fmt_mt_run(fmt_ctx* ctx) { return live(ctx) ? FMT_OK : FMT_E_USAGE; }
int fmt_mt_fetch_headers(fmt_ctx* ctx, fmt_mt_doc_result* out) {
  if (!live(ctx)) return FMT_E_USAGE;
  std::memset(out, 0, sizeof(fmt_mt_doc_result) * ctx->n_docs);
  return FMT_OK;
}
int fmt_mt_fetch_doc(fmt_ctx* ctx, uint32_t, fmt_mt_leaf*, uint32_t, uint16_t*, uint32_t, fmt_mt_propset*, uint32_t) {
  return unsupported(ctx, "fmt_mt_fetch_doc");
}
int fmt_mt_fetch_catchup(fmt_ctx* ctx, uint32_t, fmt_mt_catchup_range*, uint32_t) {
  return unsupported(ctx, "fmt_mt_fetch_catchup");
}
int fmt_mt_fetch_catchup_all(fmt_ctx* ctx, uint64_t*, fmt_mt_catchup_range*, uint64_t) {
  return unsupported(ctx, "fmt_mt_fetch_catchup_all");
}
int fmt_mt_fetch_remove_order(fmt_ctx* ctx, uint32_t, fmt_mt_remove_order*, uint32_t) {
  return unsupported(ctx, "fmt_mt_fetch_remove_order");
}
int fmt_mt_fetch_numbers(fmt_ctx* ctx, uint32_t, double*, uint32_t, uint32_t*) {
  return unsupported(ctx, "fmt_mt_fetch_numbers");
}
int fmt_mt_fetch_legacy_props(fmt_ctx* ctx, uint32_t, uint16_t*, uint32_t) {
  return unsupported(ctx, "fmt_mt_fetch_legacy_props");
}
int fmt_mt_fetch_rm_clients_hi(fmt_ctx* ctx, uint32_t, uint64_t*, uint32_t) {
  return unsupported(ctx, "fmt_mt_fetch_rm_clients_hi");
}
int fmt_mt_fetch_rm_clients_hi2(fmt_ctx* ctx, uint32_t, uint64_t*, uint32_t) {
  return unsupported(ctx, "fmt_mt_fetch_rm_clients_hi2");
}
int fmt_mt_fetch_regen(fmt_ctx* ctx, uint32_t, fmt_mt_op*, uint32_t, uint16_t*, uint32_t, uint32_t*, uint32_t*) {
  return unsupported(ctx, "fmt_mt_fetch_regen");
}
int fmt_mt_state_digest(fmt_ctx* ctx, uint64_t*) { return unsupported(ctx, "fmt_mt_state_digest"); }
int fmt_mt_capacity(uint32_t* max_leaves, uint32_t* max_chars, uint32_t* max_props) {
  if (max_leaves) *max_leaves = 2048;
  if (max_chars) *max_chars = 131071;
  if (max_props) *max_props = 1024;
  return FMT_OK;
}
}
