// kg_abi.cpp -- the extern "C" boundary of libketogpu.so (declared in include/ketogpu.h).
// No exception crosses the ABI; every failure returns non-zero and sets kg_last_error().
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "kg_snapshot.h"

namespace kg {
static thread_local std::string g_err;

int set_error(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
void clear_error() { g_err.clear(); }
}  // namespace kg

using kg::Snapshot;
using kg::set_error;

#define KG_GUARD_BEGIN try {
#define KG_GUARD_END                                          \
  }                                                           \
  catch (const std::bad_alloc&) {                             \
    return set_error(-4, "host allocation failed");           \
  }                                                           \
  catch (const std::exception& ex) {                          \
    return set_error(-5, "internal error: %s", ex.what());    \
  }                                                           \
  catch (...) {                                               \
    return set_error(-5, "internal error");                   \
  }

extern "C" {

const char* kg_version(void) { return "ketogpu 0.1 (gfx950)"; }

size_t kg_last_error(char* buf, size_t len) {
  const std::string& e = kg::g_err;
  if (buf && len) {
    size_t n = e.size() < len - 1 ? e.size() : len - 1;
    memcpy(buf, e.data(), n);
    buf[n] = 0;
  }
  return e.size();
}

int kg_snapshot_create(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog, int device,
                       kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (!out) return set_error(-2, "out is NULL");
  *out = nullptr;
  if (n && !rows) return set_error(-2, "rows is NULL");
  Snapshot* s = new Snapshot();
  int rc = s->init_device(device);
  if (!rc) rc = s->create_from_tuples(rows, n, dict, prog);
  if (rc) {
    delete s;
    return rc;
  }
  *out = reinterpret_cast<kg_snapshot*>(s);
  kg::clear_error();
  return 0;
  KG_GUARD_END
}

int kg_snapshot_synthetic(const kg_synth_params* params, const kg_rewrite_prog* prog, int device,
                          kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (!out || !params) return set_error(-2, "NULL argument");
  *out = nullptr;
  Snapshot* s = new Snapshot();
  int rc = s->init_device(device);
  if (!rc) rc = s->create_synthetic(params, prog);
  if (rc) {
    delete s;
    return rc;
  }
  *out = reinterpret_cast<kg_snapshot*>(s);
  return 0;
  KG_GUARD_END
}

void kg_snapshot_destroy(kg_snapshot* s) { delete reinterpret_cast<Snapshot*>(s); }

uint32_t kg_shard_owner(uint32_t ns, uint32_t obj, uint32_t nranks) { return kg::shard_owner(ns, obj, nranks); }

int kg_snapshot_create_shard(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog,
                             int device, uint32_t rank, uint32_t nranks, kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (!out) return set_error(-2, "out is NULL");
  *out = nullptr;
  if (n && !rows) return set_error(-2, "rows is NULL");
  if (nranks < 1 || nranks > KG_SHARD_MAX_RANKS || rank >= nranks) return set_error(-2, "bad shard %u/%u", rank, nranks);
  Snapshot* s = new Snapshot();
  s->shard_rank = rank;
  s->shard_n = nranks;
  int rc = s->init_device(device);
  if (!rc) rc = s->create_from_tuples(rows, n, dict, prog);
  if (rc) {
    delete s;
    return rc;
  }
  *out = reinterpret_cast<kg_snapshot*>(s);
  kg::clear_error();
  return 0;
  KG_GUARD_END
}

int kg_snapshot_synthetic_shard(const kg_synth_params* params, const kg_rewrite_prog* prog, int device, uint32_t rank,
                                uint32_t nranks, kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (!out || !params) return set_error(-2, "NULL argument");
  *out = nullptr;
  if (nranks < 1 || nranks > KG_SHARD_MAX_RANKS || rank >= nranks) return set_error(-2, "bad shard %u/%u", rank, nranks);
  Snapshot* s = new Snapshot();
  s->shard_rank = rank;
  s->shard_n = nranks;
  int rc = s->init_device(device);
  if (!rc) rc = s->create_synthetic(params, prog);
  if (rc) {
    delete s;
    return rc;
  }
  *out = reinterpret_cast<kg_snapshot*>(s);
  return 0;
  KG_GUARD_END
}

int kg_shard_seed(kg_snapshot* sp, const kg_query* d_q, size_t n, int32_t global_max_depth, kg_frec* d_out, size_t cap,
                  uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || !d_res || !d_err || (n && (!d_q || !d_out))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_seed(s, d_q, n, global_max_depth, d_out, cap, d_counts, d_res, d_err, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_level(kg_snapshot* sp, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out,
                   size_t cap, uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || !d_res || !d_err || (n_in && (!d_in || !d_out))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->shard_vis) return set_error(-2, "kg_shard_level before kg_shard_seed");
  return kg::shard_level(s, d_in, n_in, d_n_in, d_out, cap, d_counts, d_res, d_err, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_finish(kg_snapshot* sp, size_t n, uint8_t* d_res, const uint32_t* d_err, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || (n && (!d_res || !d_err))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_finish(s, n, d_res, d_err, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_snapshot_info(const kg_snapshot* sp, uint64_t* info4) {
  if (!sp || !info4) return set_error(-2, "NULL argument");
  const Snapshot* s = reinterpret_cast<const Snapshot*>(sp);
  info4[0] = s->ds.n_nodes;
  info4[1] = s->h_row_off_last;
  info4[2] = s->n_set_edges;
  info4[3] = s->device_bytes;
  return 0;
}

int kg_snapshot_tune(kg_snapshot* sp, const char* key, int64_t value) {
  if (!sp || !key) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  if (strcmp(key, "tiers") == 0) {
    if (value < 0 || value > 2) return set_error(-2, "tiers must be 0, 1 or 2");
    s->tiers = (int)value;
    return 0;
  }
  if (strcmp(key, "wide") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "wide must be 0 or 1");
    s->wide_tier = (int)value;
    return 0;
  }
  if (strcmp(key, "shard_vis") == 0) {
    if (value < 10 || value > 34) return set_error(-2, "shard_vis must be in [10, 34]");
    s->shard_vis_log2 = (int)value;
    return 0;
  }
  if (strcmp(key, "stream") == 0) {
    if (value < 0 || value > 8) return set_error(-2, "stream must be in [0, 8]");
    s->stream_variant = (int)value;
    return 0;
  }
  if (strcmp(key, "stream_ecap") == 0) {
    if (value < 0 || value > 0xFFFFFFFFll) return set_error(-2, "stream_ecap must be in [0, 2^32)");
    s->stream_ecap = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "stream_wgs") == 0) {
    if (value < 0 || value > 8) return set_error(-2, "stream_wgs must be in [0, 8]");
    s->stream_wgs = (int)value;
    return 0;
  }
  if (strcmp(key, "grid_wgs") == 0) {
    if (value < 1 || value > 64) return set_error(-2, "grid_wgs must be in [1, 64]");
    s->grid_wgs = (int)value;
    return 0;
  }
  if (strcmp(key, "interp_wgs") == 0) {
    if (value < 1 || value > 8) return set_error(-2, "interp_wgs must be in [1, 8]");
    s->interp_wgs = (int)value;
    return 0;
  }
  if (strcmp(key, "interp_cap2") == 0) {
    if (value < 0 || value > (1 << 22)) return set_error(-2, "interp_cap2 must be in [0, 4194304]");
    s->interp_cap2 = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "back_wgs") == 0) {
    if (value < 1 || value > 3) return set_error(-2, "back_wgs must be in [1, 3]");
    s->back_wgs = (int)value;
    return 0;
  }
  if (strcmp(key, "back") == 0) {
    if (value < 0 || value > 2) return set_error(-2, "back must be 0, 1 or 2");
    s->back_tier = (int)value;
    return 0;
  }
  if (strcmp(key, "light") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "light must be 0 or 1");
    s->light_tier = (int)value;
    return 0;
  }
  return set_error(-2, "unknown knob '%s'", key);
}

int kg_synth_ids(const kg_snapshot* sp, uint32_t* ids6) {
  if (!sp || !ids6) return set_error(-2, "NULL argument");
  const Snapshot* s = reinterpret_cast<const Snapshot*>(sp);
  if (!s->is_synth) return set_error(-2, "not a synthetic snapshot");
  const kg::SynthLayout& L = s->synth;
  ids6[0] = L.n_docs;
  ids6[1] = L.n_groups;
  ids6[2] = L.n_users;
  ids6[3] = L.n_folders;
  ids6[4] = L.user_obj0;
  ids6[5] = L.folder_obj0;
  return 0;
}

int64_t kg_snapshot_export(const kg_snapshot* sp, kg_tuple* rows, uint64_t cap) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  Snapshot* s = const_cast<Snapshot*>(reinterpret_cast<const Snapshot*>(sp));
  std::lock_guard<std::mutex> lk(s->mu);
  hipSetDevice(s->device);
  return s->export_rows(rows, cap);
  KG_GUARD_END
}

int kg_snapshot_export_csr(const kg_snapshot* sp, uint64_t* row_off, uint32_t* row_subj, uint32_t* nd_ns,
                           uint32_t* nd_obj, uint32_t* nd_rel) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  Snapshot* s = const_cast<Snapshot*>(reinterpret_cast<const Snapshot*>(sp));
  std::lock_guard<std::mutex> lk(s->mu);
  HIPC(hipSetDevice(s->device));
  size_t nn = s->ds.n_nodes;
  if (row_off) HIPC(hipMemcpy(row_off, s->ds.row_off, (nn + 1) * 8, hipMemcpyDeviceToHost));
  if (row_subj && s->h_row_off_last)
    HIPC(hipMemcpy(row_subj, s->ds.row_subj, s->h_row_off_last * 4, hipMemcpyDeviceToHost));
  if (nn && nd_ns) HIPC(hipMemcpy(nd_ns, s->ds.nd_ns, nn * 4, hipMemcpyDeviceToHost));
  if (nn && nd_obj) HIPC(hipMemcpy(nd_obj, s->ds.nd_obj, nn * 4, hipMemcpyDeviceToHost));
  if (nn && nd_rel) HIPC(hipMemcpy(nd_rel, s->ds.nd_rel, nn * 4, hipMemcpyDeviceToHost));
  return 0;
  KG_GUARD_END
}

int kg_check_batch_device(kg_snapshot* sp, const kg_query* d_q, size_t n, int32_t global_max_depth, uint8_t* d_out,
                          uint32_t* d_err, kg_stats* stats, void* stream) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  if (s->shard_n > 1) return set_error(-2, "sharded snapshot: checks run through kg_shard_seed / kg_shard_level");
  kg::Workspace* w = s->workspace((hipStream_t)stream);  // one per stream: batches on other streams overlap
  std::lock_guard<std::mutex> lk(w->mu);
  return kg::check_batch_device(s, w, d_q, n, global_max_depth, d_out, d_err, stats);
  KG_GUARD_END
}

int kg_check_batch(kg_snapshot* sp, const kg_query* q, size_t n, int32_t global_max_depth, uint8_t* out,
                   uint32_t* err_code, kg_stats* stats) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  if (n && (!q || !out)) return set_error(-2, "NULL buffer");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  if (s->shard_n > 1) return set_error(-2, "sharded snapshot: checks run through kg_shard_seed / kg_shard_level");
  kg::Workspace* w = s->workspace(nullptr);
  std::lock_guard<std::mutex> lk(w->mu);
  HIPC(hipSetDevice(s->device));
  if (n == 0) {
    if (stats) memset(stats, 0, sizeof *stats);
    return 0;
  }
  kg_query* d_q = nullptr;
  uint8_t* d_out = nullptr;
  uint32_t* d_err = nullptr;
  HIPC(hipMalloc(&d_q, n * sizeof(kg_query)));
  HIPC(hipMalloc(&d_out, n));
  HIPC(hipMalloc(&d_err, n * 4));
  int rc = 0;
  if (hipMemcpyAsync(d_q, q, n * sizeof(kg_query), hipMemcpyHostToDevice, s->stream) != hipSuccess)
    rc = set_error(-1, "H2D copy failed");
  if (!rc) rc = kg::check_batch_device(s, w, d_q, n, global_max_depth, d_out, d_err, stats);
  if (!rc && hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
    rc = set_error(-1, "D2H copy failed");
  if (!rc && err_code && hipMemcpyAsync(err_code, d_err, n * 4, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
    rc = set_error(-1, "D2H copy failed");
  if (!rc) {
    hipError_t e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) rc = set_error(-1, "batch failed: %s", hipGetErrorString(e));
  }
  hipFree(d_q);
  hipFree(d_out);
  hipFree(d_err);
  return rc;
  KG_GUARD_END
}

int kg_synth_queries(kg_snapshot* sp, uint64_t seed, size_t n, kg_query* d_q) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::synth_queries(s, seed, n, d_q);
  KG_GUARD_END
}

int kg_expand_batch(kg_snapshot* sp, const kg_set* roots, size_t n, int32_t global_max_depth, kg_tree_buf* out) {
  KG_GUARD_BEGIN
  if (!sp || !out) return set_error(-2, "NULL argument");
  if (n && !roots) return set_error(-2, "roots is NULL");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::expand_batch(s, roots, n, global_max_depth, out);
  KG_GUARD_END
}

void kg_tree_free(kg_tree_buf* t) {
  if (!t) return;
  free(t->nodes);
  free(t->root_off);
  memset(t, 0, sizeof *t);
}

}  // extern "C"
