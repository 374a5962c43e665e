// kg_abi.cpp -- the extern "C" boundary of libketogpu.so (declared in include/ketogpu.h).
// No exception crosses the ABI; every failure returns non-zero and sets kg_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <new>
#include <string>
#include <thread>
#include <vector>

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

}  // extern "C"

namespace {
std::vector<int> mask_devices(int device_mask) {
  std::vector<int> d;
  for (int b = 0; b < 31; b++)
    if (device_mask & (1 << b)) d.push_back(b);
  if (d.empty()) d.push_back(0);
  return d;
}

// Builds one replica per entry of devs (entries may repeat: several replicas on one device),
// concurrently, one host thread per replica; replica 0 owns the others.
int build_replicas(const int* devs, int n_dev, const std::function<int(Snapshot*, int)>& build, kg_snapshot** out) {
  if (!out) return set_error(-2, "out is NULL");
  *out = nullptr;
  if (!devs || n_dev < 1 || n_dev > 64) return set_error(-2, "between 1 and 64 devices");
  std::vector<Snapshot*> reps(n_dev, nullptr);
  std::vector<int> rcs(n_dev, 0);
  std::vector<std::string> msgs(n_dev);
  auto one = [&](int i) {
    try {
      Snapshot* s = new Snapshot();
      reps[i] = s;
      int rc = s->init_device(devs[i]);
      if (!rc) rc = build(s, i);
      rcs[i] = rc;
      if (rc) {
        char buf[1024];
        kg_last_error(buf, sizeof buf);
        msgs[i] = buf;
      }
    } catch (const std::exception& ex) {
      rcs[i] = -5;
      msgs[i] = ex.what();
    }
  };
  std::vector<std::thread> th;
  for (int i = 1; i < n_dev; i++) th.emplace_back(one, i);
  one(0);
  for (auto& t : th) t.join();
  int bad = -1;
  for (int i = 0; i < n_dev; i++)
    if (rcs[i] && bad < 0) bad = i;
  if (bad >= 0) {
    for (Snapshot* s : reps) delete s;
    return set_error(rcs[bad], "replica %d (device %d): %s", bad, devs[bad], msgs[bad].c_str());
  }
  for (int i = 1; i < n_dev; i++) reps[0]->peers.push_back(reps[i]);
  *out = reinterpret_cast<kg_snapshot*>(reps[0]);
  kg::clear_error();
  return 0;
}
}  // namespace

extern "C" {

int kg_snapshot_create_on(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog,
                          const int* devices, int n_devices, kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (n && !rows) return set_error(-2, "rows is NULL");
  return build_replicas(devices, n_devices, [&](Snapshot* s, int) { return s->create_from_tuples(rows, n, dict, prog); },
                        out);
  KG_GUARD_END
}

int kg_snapshot_create_ordered(const kg_tuple* rows, const uint64_t* keys, size_t n, const kg_dict* dict,
                               const kg_rewrite_prog* prog, const int* devices, int n_devices, kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (n && (!rows || !keys)) return set_error(-2, "rows / keys is NULL");
  for (size_t i = 1; i < n; i++)
    if (keys[i] < keys[i - 1]) return set_error(-2, "kg_snapshot_create_ordered: keys not ascending at row %zu", i);
  return build_replicas(devices, n_devices,
                        [&](Snapshot* s, int) { return s->create_from_tuples(rows, n, dict, prog, keys); }, out);
  KG_GUARD_END
}

int kg_snapshot_apply(kg_snapshot* bp, const kg_tuple* ins, const uint64_t* ins_keys, size_t n_ins, const kg_tuple* del,
                      size_t n_del, const kg_dict* dict, const kg_rewrite_prog* prog, kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (!bp || !out) return set_error(-2, "NULL argument");
  if ((n_ins && !ins) || (n_del && !del)) return set_error(-2, "ins / del is NULL");
  Snapshot* base = reinterpret_cast<Snapshot*>(bp);
  std::vector<int> devs;
  for (size_t i = 0; i < base->n_replicas(); i++) devs.push_back(base->replica(i)->device);
  return build_replicas(devs.data(), (int)devs.size(), [&](Snapshot* s, int i) {
    return s->create_from_delta(base->replica((size_t)i), ins, ins_keys, n_ins, del, n_del, dict, prog);
  }, out);
  KG_GUARD_END
}

int kg_snapshot_create(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog, int device_mask,
                       kg_snapshot** out) {
  const std::vector<int> d = mask_devices(device_mask);
  return kg_snapshot_create_on(rows, n, dict, prog, d.data(), (int)d.size(), out);
}

int kg_snapshot_synthetic_on(const kg_synth_params* params, const kg_rewrite_prog* prog, const int* devices,
                             int n_devices, kg_snapshot** out) {
  KG_GUARD_BEGIN
  if (!params) return set_error(-2, "NULL argument");
  return build_replicas(devices, n_devices, [&](Snapshot* s, int) { return s->create_synthetic(params, prog); }, out);
  KG_GUARD_END
}

int kg_snapshot_synthetic(const kg_synth_params* params, const kg_rewrite_prog* prog, int device_mask,
                          kg_snapshot** out) {
  const std::vector<int> d = mask_devices(device_mask);
  return kg_snapshot_synthetic_on(params, prog, d.data(), (int)d.size(), out);
}

int kg_snapshot_replicas(const kg_snapshot* sp, int* devices, int cap) {
  if (!sp) return set_error(-2, "NULL snapshot");
  Snapshot* s = const_cast<Snapshot*>(reinterpret_cast<const Snapshot*>(sp));
  const int n = (int)s->n_replicas();
  for (int i = 0; devices && i < n && i < cap; i++) devices[i] = s->replica(i)->device;
  return n;
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
                   size_t cap, uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done,
                   uint32_t done_words, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || !d_res || !d_err || (n_in && (!d_in || !d_out))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  {
    kg::ShardCtx* c = s->shard_ctx((hipStream_t)stream, false);
    if (!c || !c->vis) return set_error(-2, "kg_shard_level before kg_shard_seed (on this stream)");
  }
  return kg::shard_level(s, d_in, n_in, d_n_in, d_out, cap, d_counts, d_res, d_err, d_done, done_words,
                         (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_level_seg(kg_snapshot* sp, const kg_frec* d_in, uint32_t n_seg, size_t seg_cap,
                       const uint32_t* d_seg_counts, kg_frec* d_out, size_t cap, uint32_t* d_counts, uint8_t* d_res,
                       uint32_t* d_err, const uint32_t* d_done, uint32_t done_words, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || !d_res || !d_err || !d_seg_counts || (n_seg && (!d_in || !d_out)))
    return set_error(-2, "NULL argument");
  if (n_seg < 1 || n_seg > KG_SHARD_MAX_RANKS || seg_cap == 0) return set_error(-2, "n_seg in [1, %d], seg_cap > 0", KG_SHARD_MAX_RANKS);
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  {
    kg::ShardCtx* c = s->shard_ctx((hipStream_t)stream, false);
    if (!c || !c->vis) return set_error(-2, "kg_shard_level_seg before kg_shard_seed (on this stream)");
  }
  return kg::shard_level(s, d_in, (size_t)n_seg * seg_cap, d_seg_counts, d_out, cap, d_counts, d_res, d_err, d_done,
                         done_words, (hipStream_t)stream, n_seg, seg_cap);
  KG_GUARD_END
}

int kg_shard_levels(kg_snapshot* sp, int32_t levels, kg_frec* d_buf0, kg_frec* d_buf1, size_t cap, uint32_t* d_counts0,
                    uint32_t* d_counts1, int32_t start, uint8_t* d_res, uint32_t* d_err, size_t n_slots,
                    int32_t with_escalated, int32_t* end, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_buf0 || !d_buf1 || !d_counts0 || !d_counts1 || !d_res || !d_err) return set_error(-2, "NULL argument");
  if (levels < 0 || levels > 1024 || (start != 0 && start != 1) || with_escalated < 0 || with_escalated > 2 || cap == 0)
    return set_error(-2, "kg_shard_levels: levels in [0, 1024], start 0 / 1, with_escalated 0..2, cap > 0");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  kg_frec* bufs[2] = {d_buf0, d_buf1};
  uint32_t* counts[2] = {d_counts0, d_counts1};
  int e = start;
  const int rc = kg::shard_levels(s, levels, bufs, cap, counts, start, d_res, d_err, n_slots, with_escalated, &e,
                                  (hipStream_t)stream);
  if (end) *end = e;
  return rc;
  KG_GUARD_END
}

int kg_shard_done(kg_snapshot* sp, size_t n, const uint8_t* d_res, const uint32_t* d_err, int with_escalated,
                  uint32_t* d_bits, uint32_t words, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || (n && (!d_res || !d_bits))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_done(s, n, d_res, d_err, with_escalated, d_bits, words, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_back_list(kg_snapshot* sp, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_list,
                       size_t cap, uint32_t* d_counts, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || (n && (!d_res || !d_err || !d_list))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_back_list(s, n, d_res, d_err, d_list, cap, d_counts, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_back_seed(kg_snapshot* sp, const kg_frec* d_list, size_t m, const uint32_t* d_m, kg_frec* d_out,
                       size_t cap, uint32_t* d_counts, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || (m && (!d_list || !d_out))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_back_seed(s, d_list, m, d_m, d_out, cap, d_counts, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_back_level(kg_snapshot* sp, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out,
                        size_t cap, uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done,
                        uint32_t done_words, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || !d_res || !d_err || (n_in && (!d_in || !d_out))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  {
    kg::ShardCtx* c = s->shard_ctx((hipStream_t)stream, false);
    if (!c || !c->vis) return set_error(-2, "kg_shard_back_level before kg_shard_seed (on this stream)");
  }
  return kg::shard_back_level(s, d_in, n_in, d_n_in, d_out, cap, d_counts, d_res, d_err, d_done, done_words,
                              (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_refwd_seed(kg_snapshot* sp, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_out,
                        size_t cap, uint32_t* d_counts, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !d_counts || (n && (!d_res || !d_err || !d_out))) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_refwd_seed(s, n, d_res, d_err, d_out, cap, d_counts, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_held(kg_snapshot* sp, uint32_t* d_bits, size_t words, int import, void* stream) {
  KG_GUARD_BEGIN
  if (!sp || (words && !d_bits)) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_held(s, d_bits, words, import, (hipStream_t)stream);
  KG_GUARD_END
}

int kg_shard_held_words(const kg_snapshot* sp, size_t* words) {
  if (!sp || !words) return set_error(-2, "NULL argument");
  const Snapshot* s = reinterpret_cast<const Snapshot*>(sp);
  *words = ((size_t)s->ds.hbits_n + 31) / 32;
  return 0;
}

int kg_shard_bad_nodes(const kg_snapshot* sp, uint64_t* count) {
  KG_GUARD_BEGIN
  if (!sp || !count) return set_error(-2, "NULL argument");
  Snapshot* s = const_cast<Snapshot*>(reinterpret_cast<const Snapshot*>(sp));
  std::lock_guard<std::mutex> lk(s->mu);
  return kg::shard_bad_nodes(s, count);
  KG_GUARD_END
}

size_t kg_shard_result_slots(const kg_snapshot* sp, size_t n) {
  return sp ? kg::shard_result_slots(reinterpret_cast<const Snapshot*>(sp), n) : n;
}

int kg_shard_finish(kg_snapshot* sp, size_t n, uint8_t* d_res, uint32_t* d_err, void* stream) {
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

int kg_snapshot_materialized(const kg_snapshot* sp, uint64_t* out3) {
  if (!sp || !out3) return set_error(-2, "NULL argument");
  const Snapshot* s = reinterpret_cast<const Snapshot*>(sp);
  out3[0] = s->n_virtual;
  out3[1] = s->n_virtual_new;
  out3[2] = s->n_check_rows;
  return 0;
}

static int tune_one(Snapshot* s, const char* key, int64_t value) {
  std::lock_guard<std::mutex> lk(s->mu);


  if (strcmp(key, "shard_vis") == 0) {
    if (value < 10 || value > 34) return set_error(-2, "shard_vis must be in [10, 34]");
    s->shard_vis_log2 = (int)value;
    return 0;
  }
  if (strcmp(key, "shard_bucket") == 0) {
    if (value < 0 || value > (1ll << 26)) return set_error(-2, "shard_bucket must be in [0, 2^26]");
    s->shard_bucket0 = (uint32_t)value;
    return 0;
  }

  if (strcmp(key, "shard_force_exchange") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "shard_force_exchange must be 0 or 1");
    s->shard_force_exchange = (int)value;
    return 0;
  }
  if (strcmp(key, "shard_local") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "shard_local must be 0 or 1");
    s->shard_local = (int)value;
    return 0;
  }
  if (strcmp(key, "shard_remote_meta") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "shard_remote_meta must be 0 or 1");
    s->shard_remote_meta = (int)value;
    return 0;
  }
  if (strcmp(key, "shard_max_reruns") == 0) {
    if (value < 0 || value > 64) return set_error(-2, "shard_max_reruns must be in [0, 64]");
    s->shard_max_reruns = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "shard_max_bytes") == 0) {
    if (value < 0) return set_error(-2, "shard_max_bytes must be >= 0 (0: a quarter of the free HBM)");
    s->shard_max_bytes = (uint64_t)value;
    return 0;
  }
  if (strcmp(key, "shard_force_overflow") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "shard_force_overflow must be 0 or 1");
    s->shard_force_overflow = (int)value;
    return 0;
  }

  if (strcmp(key, "stream_ecap") == 0) {
    if (value < 0 || value > 0xFFFFFFFFll) return set_error(-2, "stream_ecap must be in [0, 2^32)");
    s->stream_ecap = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "shard_budget") == 0) {
    if (value < 0 || value > 0xFFFFFFFFll) return set_error(-2, "shard_budget must be in [0, 2^32)");
    s->shard_budget = (uint32_t)value;
    return 0;
  }

  if (strcmp(key, "shard_heavy") == 0) {
    if (value < 0 || value > 0xFFFFFFFFll) return set_error(-2, "shard_heavy must be in [0, 2^32)");
    s->shard_heavy = (uint32_t)value;
    return 0;
  }



  if (strcmp(key, "shard_back_budget") == 0) {
    if (value < 0 || value > 0xFFFFFFFFll) return set_error(-2, "shard_back_budget must be in [0, 2^32)");
    s->shard_back_budget = (uint32_t)value;
    return 0;
  }

  if (strcmp(key, "stream_steal") == 0) {
    if (value < 1 || value > 8) return set_error(-2, "stream_steal must be in [1, 8]");
    s->stream_steal = (uint32_t)value;
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

  if (strcmp(key, "interp_cap2") == 0) {
    if (value < 0 || value > (1 << 22)) return set_error(-2, "interp_cap2 must be in [0, 4194304]");
    s->interp_cap2 = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "grid_reserve") == 0) return kg::grid_reserve(s);  // the shared full-size grid pool, now
  if (strcmp(key, "grid_cap") == 0) {
    if (value < 0 || value > (1ll << 34)) return set_error(-2, "grid_cap must be in [0, 2^34]");
    s->grid_small_cap = (uint64_t)value;
    return 0;
  }
  if (strcmp(key, "expand_gw") == 0 || strcmp(key, "expand_skip_lds") == 0) {
    if (value < 0 || value > (strcmp(key, "expand_gw") == 0 ? 1 : 2))
      return set_error(-2, "%s must be 0 or 1 (expand_skip_lds: 0, 1 or 2)", key);
    (strcmp(key, "expand_gw") == 0 ? s->expand_gw : s->expand_skip_lds) = (int)value;
    return 0;
  }
  if (strcmp(key, "level_events") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "level_events must be 0 or 1");
    s->level_events = (int)value;
    return 0;
  }
  if (strcmp(key, "expand_gw_wait_us") == 0) {
    if (value < 0 || value > 10000000) return set_error(-2, "expand_gw_wait_us must be in [0, 10^7]");
    s->expand_gw_wait_us = (uint32_t)value;
    return 0;
  }

  if (strcmp(key, "grid_ms") == 0) {
    if (value < 0 || value > 1) return set_error(-2, "grid_ms must be 0 or 1");
    s->grid_ms = (int)value;
    return 0;
  }
  if (strcmp(key, "grid_ms_bytes") == 0) {
    if (value < (1 << 20) || value > (1ll << 40)) return set_error(-2, "grid_ms_bytes must be in [2^20, 2^40]");
    s->grid_ms_bytes = (size_t)value;
    return 0;
  }
  if (strcmp(key, "grid_ms_words") == 0) {
    if (value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
      return set_error(-2, "grid_ms_words must be 1, 2, 4, 8 or 16");
    s->grid_ms_words = (int)value;
    return 0;
  }
  if (strcmp(key, "grid_ms_tg_cap") == 0) {
    if (value < 0 || value > 0x7FFFFFFF) return set_error(-2, "grid_ms_tg_cap must be in [0, 2^31)");
    s->grid_ms_tg_cap = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "grid_ms_cap") == 0) {
    if (value < 0 || value > (1ll << 28)) return set_error(-2, "grid_ms_cap must be in [0, 2^28]");
    s->grid_ms_cap = (uint64_t)value;
    return 0;
  }

  if (strcmp(key, "max_lanes") == 0) {
    if (value < 1 || value > 1024) return set_error(-2, "max_lanes in [1, 1024]");
    {
      std::lock_guard<std::mutex> lk(s->lane_mu);
      s->lane_cap = (size_t)value;  // sets already created stay in the pool
    }
    s->lane_cv.notify_all();
    return 0;
  }
  if (strcmp(key, "back_edges") == 0) {
    if (value < 0 || value > (1 << 20)) return set_error(-2, "back_edges must be in [0, 2^20]");
    s->back_edges = (uint32_t)value;
    return 0;
  }
  if (strcmp(key, "back_wgs") == 0) {
    if (value < 1 || value > 3) return set_error(-2, "back_wgs must be in [1, 3]");
    s->back_wgs = (int)value;
    return 0;
  }

  return set_error(-2, "unknown knob '%s'", key);
}

int kg_snapshot_tune(kg_snapshot* sp, const char* key, int64_t value) {
  if (!sp || !key) return set_error(-2, "NULL argument");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  for (size_t i = 0; i < s->n_replicas(); i++)
    if (int rc = tune_one(s->replica(i), key, value)) return rc;
  return 0;
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

int64_t kg_snapshot_rows(const kg_snapshot* sp, const kg_set* keys, size_t n, uint64_t* offsets, kg_tuple* out,
                         uint64_t cap) {
  KG_GUARD_BEGIN
  if (!sp || (n && (!keys || !offsets))) return set_error(-2, "NULL argument");
  Snapshot* s = const_cast<Snapshot*>(reinterpret_cast<const Snapshot*>(sp));
  std::lock_guard<std::mutex> lk(s->mu);
  return s->rows_of(keys, n, offsets, out, cap);
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
  // a transport bound to this stream: the whole hash-sharded batch inside the library (kg_shard_comm.hip)
  bool sharded = false;
  const int src = kg::shard_check_entry(s, (hipStream_t)stream, d_q, n, global_max_depth, d_out, d_err, stats, &sharded);
  if (sharded) return src;
  if (s->shard_n > 1)
    return set_error(-2, "sharded snapshot: bind a transport to this stream (kg_shard_comm_init) or drive "
                         "kg_shard_seed / kg_shard_level");
  kg::Workspace* w = s->workspace((hipStream_t)stream);  // one per stream: batches on other streams overlap
  std::lock_guard<std::mutex> lk(w->mu);
  return kg::check_batch_device(s, w, d_q, n, global_max_depth, d_out, d_err, stats);
  KG_GUARD_END
}

int kg_check_batch_packed_device(kg_snapshot* sp, const kg_query_packed* d_q, size_t n, int32_t global_max_depth,
                                 uint8_t* d_out, uint32_t* d_err, kg_stats* stats, void* stream) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  if (n && !d_q) return set_error(-2, "d_q is NULL");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  if (s->shard_n > 1 || kg::shard_comm_of(s, (hipStream_t)stream)) {
    // hash-sharded: the seed reads kg_query records -- unpacked into a buffer of this call, then the
    // usual sharded batch (completed before the buffer is freed)
    HIPC(hipSetDevice(s->device));
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    kg_query* dq = nullptr;
    if (n) HIPC(hipMalloc(&dq, n * sizeof(kg_query)));
    int rc = n ? kg::unpack_queries(d_q, n, dq, st) : 0;
    if (!rc) rc = kg_check_batch_device(sp, dq, n, global_max_depth, d_out, d_err, stats, stream);
    if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = set_error(-1, "packed sharded batch");
    hipFree(dq);
    return rc;
  }
  kg::Workspace* w = s->workspace((hipStream_t)stream);
  std::lock_guard<std::mutex> lk(w->mu);
  return kg::check_batch_device(s, w, nullptr, n, global_max_depth, d_out, d_err, stats, d_q);
  KG_GUARD_END
}

int kg_pack_queries_device(kg_snapshot* sp, const kg_query* d_q, size_t n, kg_query_packed* d_pk, void* stream) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  if (n && (!d_q || !d_pk)) return set_error(-2, "NULL buffer");
  if (n > 0x7FFFFFFFull) return set_error(-2, "batch too large");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  HIPC(hipSetDevice(s->device));
  hipStream_t st = stream ? (hipStream_t)stream : s->stream;
  uint32_t* d_bad = nullptr;
  HIPC(hipMalloc(&d_bad, 4));
  uint32_t bad = 0;
  int rc = hipMemsetAsync(d_bad, 0, 4, st) != hipSuccess ? set_error(-1, "pack: memset") : 0;
  if (!rc) rc = kg::pack_queries(d_q, n, d_pk, d_bad, st);
  if (!rc && (hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipStreamSynchronize(st) != hipSuccess))
    rc = set_error(-1, "pack: readback");
  hipFree(d_bad);
  if (!rc && bad) rc = set_error(-2, "an id does not fit kg_query_packed (use kg_check_batch_device)");
  return rc;
  KG_GUARD_END
}

// A checked-out lane set goes back to the snapshot's pool when the call returns (any path).
struct LaneLease {
  Snapshot* s;
  std::vector<kg::Lane*>* v;
  ~LaneLease() { s->lanes_release(v); }
};

// The sparse error output of kg_check_batch_packed.
struct SparseErr {
  uint32_t* idx;
  uint32_t* code;
  size_t cap;
  size_t* n;
};

// Host buffers in and out: the batch is split over the snapshot's replicas (one contiguous chunk
// each, none smaller than MIN_PER_REPLICA queries), every chunk on this thread's lane of its
// replica.  All chunks are staged and enqueued before the first wait, so the devices run
// concurrently; queries are staged through pinned memory in slices so the H2D copy of one slice
// overlaps the staging of the next.  Packed queries (pq) cross PCIe as 16 B and are unpacked on the
// device; with `sp` only the answers cross back, plus the (index, code) pairs of the KG_ERROR ones.
static int check_host(Snapshot* s, const kg_query* q, const kg_query_packed* pq, size_t n, int32_t global_max_depth,
                      uint8_t* out, uint32_t* err_code, SparseErr* sp, kg_stats* stats) {
  constexpr size_t MIN_PER_REPLICA = 16384, SLICE = 65536;
  if (stats) memset(stats, 0, sizeof *stats);
  if (sp) *sp->n = 0;
  if (n == 0) return 0;
  if (n > 0x7FFFFFFFull) return set_error(-2, "batch too large");
  std::vector<kg::Lane*>* lanes = s->lanes_acquire();
  if (!lanes) return -1;
  LaneLease lease{s, lanes};
  const size_t R = std::max<size_t>(1, std::min(lanes->size(), (n + MIN_PER_REPLICA - 1) / MIN_PER_REPLICA));
  // batches that use fewer replicas than exist rotate over them (a batcher's small batches spread
  // over every GPU instead of all landing on replica 0)
  const size_t r0 = R < lanes->size() ? (size_t)(s->rr_next.fetch_add(1, std::memory_order_relaxed) % lanes->size()) : 0;
  auto lane = [&](size_t i) { return (*lanes)[(r0 + i) % lanes->size()]; };
  std::vector<kg::BatchPending> bp(R);
  std::vector<kg_stats> st(R);
  std::vector<size_t> b(R + 1);
  for (size_t i = 0; i <= R; i++) b[i] = n * i / R;
  size_t begun = 0;
  int rc = 0;
  for (size_t i = 0; i < R && !rc; i++) {
    kg::Lane* L = lane(i);
    const size_t m = b[i + 1] - b[i];
    if ((rc = pq ? L->reserve_packed(m) : L->reserve(m))) break;
    HIPC(hipSetDevice(L->device));
    const size_t rec = pq ? sizeof(kg_query_packed) : sizeof(kg_query);
    char* hs = reinterpret_cast<char*>(L->h_q);
    char* ds = pq ? reinterpret_cast<char*>(L->d_pk) : reinterpret_cast<char*>(L->d_q);
    const char* src = pq ? reinterpret_cast<const char*>(pq + b[i]) : reinterpret_cast<const char*>(q + b[i]);
    for (size_t o = 0; o < m; o += SLICE) {
      const size_t k = std::min(SLICE, m - o);
      memcpy(hs + o * rec, src + o * rec, k * rec);
      if (hipMemcpyAsync(ds + o * rec, hs + o * rec, k * rec, hipMemcpyHostToDevice, L->stream) != hipSuccess) {
        rc = set_error(-1, "H2D copy failed");
        break;
      }
    }
    if (!rc && pq) rc = kg::unpack_queries(L->d_pk, m, L->d_q, L->stream);
    if (rc) break;
    L->w->mu.lock();
    rc = kg::check_batch_begin(L->rep, L->w, L->d_q, m, global_max_depth, L->d_out, L->d_err, stats ? &st[i] : nullptr,
                               &bp[i]);
    begun++;
    if (!rc && (hipMemcpyAsync(L->h_out, L->d_out, m, hipMemcpyDeviceToHost, L->stream) != hipSuccess ||
                (!sp && hipMemcpyAsync(L->h_err, L->d_err, m * 4, hipMemcpyDeviceToHost, L->stream) != hipSuccess)))
      rc = set_error(-1, "D2H copy failed");
  }
  std::vector<std::pair<uint32_t, uint32_t>> errs;  // sparse: (index, code) over every chunk
  for (size_t i = 0; i < begun; i++) {
    kg::Lane* L = lane(i);
    const size_t m = b[i + 1] - b[i];
    if (!rc) {
      hipSetDevice(L->device);
      bool reran = false;
      // asleep on a blocking-sync event, not spinning (round 2: one spinning core per in-flight batch
      // competed with the server's threads; the "host_sync" knob was removed in round 6)
      int r2 = kg::check_batch_end(L->rep, L->w, &bp[i], &reran, true);
      if (!r2 && reran &&  // the grid tier rewrote results after the first copy: copy them again
          (hipMemcpyAsync(L->h_out, L->d_out, m, hipMemcpyDeviceToHost, L->stream) != hipSuccess ||
           (!sp && hipMemcpyAsync(L->h_err, L->d_err, m * 4, hipMemcpyDeviceToHost, L->stream) != hipSuccess)))
        r2 = set_error(-1, "D2H copy failed");
      const size_t pre = std::min(m, kg::Lane::EL_PREFETCH);
      if (!r2 && sp) {  // the error list of the final answers, its count and first pairs read back with them
        r2 = kg::error_list(L->d_out, L->d_err, m, (uint32_t)b[i], L->d_el, m, L->stream);
        if (!r2 && hipMemcpyAsync(L->h_el, L->d_el, (2 + 2 * pre) * 4, hipMemcpyDeviceToHost, L->stream) != hipSuccess)
          r2 = set_error(-1, "D2H copy failed");
      }
      if (!r2) r2 = L->w->wait(L->stream, true);  // the error text is set by wait()
      if (!r2) {
        memcpy(out + b[i], L->h_out, m);
        if (err_code && !sp) memcpy(err_code + b[i], L->h_err, m * 4);
      }
      if (!r2 && sp) {
        const size_t cnt = std::min<size_t>(L->h_el[0], m);
        std::vector<uint32_t> more;
        const uint32_t* pairs = L->h_el + 2;
        if (cnt > pre) {  // rare: more errors than the prefetch held
          more.resize(2 * cnt);
          if (hipMemcpy(more.data(), L->d_el + 2, 2 * cnt * 4, hipMemcpyDeviceToHost) != hipSuccess)
            r2 = set_error(-1, "D2H copy failed");
          pairs = more.data();
        }
        for (size_t k = 0; !r2 && k < cnt; k++) errs.emplace_back(pairs[2 * k], pairs[2 * k + 1]);
      }
      rc = r2;
    } else {
      hipSetDevice(L->device);
      (void)hipStreamSynchronize(L->stream);
    }
    L->w->mu.unlock();
  }
  if (!rc && sp) {
    std::sort(errs.begin(), errs.end());
    *sp->n = errs.size();
    for (size_t k = 0; k < errs.size() && k < sp->cap; k++) {
      if (sp->idx) sp->idx[k] = errs[k].first;
      if (sp->code) sp->code[k] = errs[k].second;
    }
  }
  if (!rc && stats) {  // counters add up over replicas; device time is the slowest replica's
    for (size_t i = 0; i < R; i++) {
      const kg_stats& x = st[i];
      uint64_t* d = reinterpret_cast<uint64_t*>(stats);
      const uint64_t* y = reinterpret_cast<const uint64_t*>(&x);
      for (size_t f = 0; f < sizeof(kg_stats) / 8; f++) d[f] += y[f];
    }
    double km = 0, lm = 0, tm = 0, sm = 0;
    uint64_t tk = 0;
    for (size_t i = 0; i < R; i++) {
      km = std::max(km, st[i].kernel_ms);
      lm = std::max(lm, st[i].light_ms);
      tm = std::max(tm, st[i].tail_ms);
      sm = std::max(sm, st[i].split_ms);
      tk = std::max(tk, st[i].tail_kind);  // a kind, not a count
    }
    stats->tail_kind = tk;
    stats->kernel_ms = km;
    stats->light_ms = lm;
    stats->tail_ms = tm;
    stats->split_ms = sm;
  }
  return rc;
}

int kg_check_batch(kg_snapshot* sp, const kg_query* q, size_t n, int32_t global_max_depth, uint8_t* out,
                   uint32_t* err_code, kg_stats* stats) {
  KG_GUARD_BEGIN
  if (!sp) return set_error(-2, "NULL snapshot");
  if (n && (!q || !out)) return set_error(-2, "NULL buffer");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  if (s->shard_n > 1 || kg::shard_comm_of(s, nullptr))  // hash-sharded: the whole batch in kg_shard_comm.hip
    return kg::shard_check_host_entry(s, q, n, global_max_depth, out, err_code, stats);
  return check_host(s, q, nullptr, n, global_max_depth, out, err_code, nullptr, stats);
  KG_GUARD_END
}

int kg_check_batch_packed(kg_snapshot* sp, const kg_query_packed* q, size_t n, int32_t global_max_depth, uint8_t* out,
                          uint32_t* err_index, uint32_t* err_code, size_t err_cap, size_t* n_err, kg_stats* stats) {
  KG_GUARD_BEGIN
  if (!sp || !n_err) return set_error(-2, "NULL argument");
  *n_err = 0;  // defined on every return, failures included
  if (n && (!q || !out)) return set_error(-2, "NULL buffer");
  if (err_cap && (!err_index || !err_code)) return set_error(-2, "err_cap > 0 needs err_index and err_code");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  SparseErr spe{err_index, err_code, err_cap, n_err};
  if (s->shard_n > 1 || kg::shard_comm_of(s, nullptr)) {
    // hash-sharded: unpacked on the host, the whole batch in kg_shard_comm.hip (not the narrow path)
    std::vector<kg_query> w(n);
    for (size_t i = 0; i < n; i++) {
      const kg_query_packed& p = q[i];
      const uint32_t sns = (p.w2 >> 24) | ((p.w3 & 0xFu) << 8);
      w[i].t = kg_tuple{p.w2 & 0xFFFu, p.obj, (p.w2 >> 12) & 0xFFFu, sns == KG_PACK_SUBJECT_ID ? KG_SUBJECT_ID : sns,
                        p.sobj, (p.w3 >> 4) & 0xFFFu};
      w[i].max_depth = (int32_t)(p.w3 >> 16);
    }
    std::vector<uint32_t> e(n);
    if (int rc = kg::shard_check_host_entry(s, w.data(), n, global_max_depth, out, e.data(), stats)) return rc;
    *n_err = 0;
    for (size_t i = 0; i < n; i++)
      if (out[i] == KG_ERROR) {
        if (*n_err < err_cap) {
          err_index[*n_err] = (uint32_t)i;
          err_code[*n_err] = e[i];
        }
        ++*n_err;
      }
    return 0;
  }
  return check_host(s, nullptr, q, n, global_max_depth, out, nullptr, &spe, stats);
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

// Roots are split over the replicas (contiguous chunks, one host thread per replica: an expand
// call waits for its device) and the per-replica trees concatenated in root order.
int kg_expand_batch(kg_snapshot* sp, const kg_set* roots, size_t n, int32_t global_max_depth, kg_tree_buf* out) {
  KG_GUARD_BEGIN
  constexpr size_t MIN_PER_REPLICA = 1024;
  if (!sp || !out) return set_error(-2, "NULL argument");
  if (n && !roots) return set_error(-2, "roots is NULL");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  // hash-sharded: the rows the roots can reach are gathered to this rank first (collective)
  if (s->shard_n > 1 || kg::shard_comm_of(s, nullptr)) return kg::shard_expand(s, roots, n, global_max_depth, out);
  // a lane set from the pool: one stream + cached buffers per replica, so concurrent callers overlap
  std::vector<kg::Lane*>* lanes = s->lanes_acquire();
  if (!lanes) return -1;
  LaneLease lease{s, lanes};
  const size_t R = std::max<size_t>(1, std::min(s->n_replicas(), (n + MIN_PER_REPLICA - 1) / MIN_PER_REPLICA));
  const size_t r0 = R < lanes->size() ? (size_t)(s->rr_next.fetch_add(1, std::memory_order_relaxed) % lanes->size()) : 0;
  auto lane = [&](size_t i) { return (*lanes)[(r0 + i) % lanes->size()]; };
  if (R == 1) {
    kg::Lane* L = lane(0);
    return kg::expand_batch(L->rep, L->stream, &L->exp, roots, n, global_max_depth, out);
  }
  std::vector<kg_tree_buf> parts(R);
  std::vector<int> rcs(R, 0);
  std::vector<std::string> msgs(R);
  std::vector<size_t> b(R + 1);
  for (size_t i = 0; i <= R; i++) b[i] = n * i / R;
  auto one = [&](size_t i) {
    try {
      kg::Lane* L = lane(i);
      rcs[i] = kg::expand_batch(L->rep, L->stream, &L->exp, roots + b[i], b[i + 1] - b[i], global_max_depth, &parts[i]);
      if (rcs[i]) {
        char buf[1024];
        kg_last_error(buf, sizeof buf);
        msgs[i] = buf;
      }
    } catch (const std::exception& ex) {
      rcs[i] = -5;
      msgs[i] = ex.what();
    }
  };
  std::vector<std::thread> th;
  for (size_t i = 1; i < R; i++) th.emplace_back(one, i);
  one(0);
  for (auto& t : th) t.join();
  memset(out, 0, sizeof *out);
  int rc = 0;
  for (size_t i = 0; i < R && !rc; i++)
    if (rcs[i]) rc = set_error(rcs[i], "replica %zu: %s", i, msgs[i].c_str());
  uint64_t total = 0;
  for (size_t i = 0; i < R; i++) total += parts[i].n_nodes;
  if (!rc) {
    out->root_off = (uint64_t*)calloc(n + 1, 8);
    out->nodes = (kg_tree_node*)malloc(std::max<uint64_t>(total, 1) * sizeof(kg_tree_node));
    if (!out->root_off || !out->nodes) rc = set_error(-4, "host allocation failed");
  }
  if (!rc) {
    uint64_t at = 0;
    for (size_t i = 0; i < R; i++) {
      const size_t m = b[i + 1] - b[i];
      for (size_t r = 0; r < m; r++) out->root_off[b[i] + r + 1] = at + parts[i].root_off[r + 1];
      if (parts[i].n_nodes) memcpy(out->nodes + at, parts[i].nodes, parts[i].n_nodes * sizeof(kg_tree_node));
      at += parts[i].n_nodes;
      out->kernel_ms = std::max(out->kernel_ms, parts[i].kernel_ms);
    }
    out->n_nodes = total;
    out->n_roots = n;
  } else {
    free(out->root_off);
    free(out->nodes);
    memset(out, 0, sizeof *out);
  }
  for (auto& p : parts) kg_tree_free(&p);
  return rc;
  KG_GUARD_END
}

// Device-resident roots and trees (the C5 path without PCIe): one lane per stream (the stream's
// workspace keeps the expand buffers), single GPU.
int kg_expand_batch_device(kg_snapshot* sp, const kg_set* d_roots, size_t n, int32_t global_max_depth, kg_tree_buf* out,
                           void* stream) {
  KG_GUARD_BEGIN
  if (!sp || !out) return set_error(-2, "NULL argument");
  if (n && !d_roots) return set_error(-2, "d_roots is NULL");
  if (n > 0x7FFFFFFFull) return set_error(-2, "batch too large");
  Snapshot* s = reinterpret_cast<Snapshot*>(sp);
  if (s->shard_n > 1 || kg::shard_comm_of(s, (hipStream_t)stream))
    return set_error(-2, "kg_expand_batch_device: hash-sharded snapshots expand through kg_expand_batch");
  kg::Workspace* w = s->workspace((hipStream_t)stream);
  std::lock_guard<std::mutex> lk(w->mu);
  return kg::expand_batch(s, w->stream, &w->exp, d_roots, n, global_max_depth, out, true);
  KG_GUARD_END
}

void kg_tree_free(kg_tree_buf* t) {
  if (!t) return;
  if (t->pinned & kg::KG_TREE_DEVICE) {  // device-resident (kg_expand_batch_device)
    const int dev = (int)(t->pinned & 0xFF);
    kg::tree_dev_put(dev, t->nodes, t->n_nodes * sizeof(kg_tree_node));
    kg::tree_dev_put(dev, t->root_off, (t->n_roots + 1) * 8);
    memset(t, 0, sizeof *t);
    return;
  }
  if (t->pinned) kg::tree_pool_put(t->nodes, t->n_nodes * sizeof(kg_tree_node));
  else free(t->nodes);
  free(t->root_off);
  memset(t, 0, sizeof *t);
}

}  // extern "C"
