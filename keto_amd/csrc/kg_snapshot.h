// kg_snapshot.h -- host-side snapshot object and error plumbing (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <list>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/ketogpu.h"
#include "kg_grid.h"
#include "kg_internal.h"
#include "kg_synth.h"

namespace kg {

constexpr int KG_ERR_RESOURCE_CODE = -4;

// Thread-local last error (kg_last_error).  Returns `code` so callers can `return set_error(...)`.
int set_error(int code, const char* fmt, ...);
void clear_error();

#define HIPC(expr)                                                                               \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess) return ::kg::set_error(-1, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                                 __FILE__, __LINE__);                            \
  } while (0)

// Grid-tier memory (kg_grid.hip): visited hash | entry log | tile maps | slots | control block.
struct GridPool {
  void* mem = nullptr;
  size_t bytes = 0;
  uint64_t cap = 0;    // log entries the pool is laid out for (0: not yet)
  uint32_t epoch = 0;  // visited-table epoch of the last round
  void release();
};

// Everything one in-flight check batch mutates: scratch lists, tier pools, the grid tier's epoch,
// timing events and the pinned readback buffer.  One per HIP stream, so batches on different
// streams overlap on the device (the tail tiers of one batch run beside the next batch's
// k_resolve / k_stream); batches on the same stream are serialised by `mu`.
struct Workspace {
  int device = -1;
  hipStream_t stream = nullptr;
  std::mutex mu;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  size_t scratch_n = 0;  // queries the scratch was last sized for
  GridPool grid;  // grid tier, sized for the queries that reach it (16 Mi log entries)
  GridPool ms;    // the grid tier's MS-BFS path (kg_msbfs.hip): dense masks of its query groups
  bool grid_reran = false;  // the last batch's grid tier ran rounds after the first (results rewritten)
  void* split = nullptr;  // formula split (kg_formula.hip): leaf queries, their results, per-query plan refs
  size_t split_bytes = 0;
  void* interp_pool = nullptr;
  size_t interp_pool_bytes = 0;
  uint64_t interp_layout = 0;  // (pass-2 slots, pass-1 slots, list cap) the pool was last laid out for
  hipEvent_t ev[6] = {};  // batch timing events (created on first use)
  // tail-tier level launches (k_grid_level / k_ms_level) of a batch with stats: one event pair each,
  // summed in check_batch_end (kg_stats::tail_ms); launches past LEV_EV are counted, not timed
  static constexpr int LEV_EV = 64;
  hipEvent_t lev_ev[2 * LEV_EV] = {};
  int lev_n = 0, lev_kind = 0;
  uint64_t lev_launches = 0;
  bool lev_on = false;
  // record the start (end = false) or end (end = true) of one level launch
  void lev_mark(hipStream_t st, bool end, int kind) {
    if (!lev_on) return;
    if (!end) {
      lev_kind = kind;
      lev_launches++;
    }
    if (lev_n >= LEV_EV) return;
    hipEvent_t& e = lev_ev[2 * lev_n + (end ? 1 : 0)];
    if (!e && hipEventCreate(&e) != hipSuccess) {
      (void)hipGetLastError();
      e = nullptr;
    }
    if (e) (void)hipEventRecord(e, st);
    if (end) lev_n++;
  }
  hipEvent_t sync_ev = nullptr;  // blocking-sync event (host-buffer batches wait on it asleep)
  int wait(hipStream_t st, bool blocking);  // waits for st: spin (hipStreamSynchronize) or asleep
  void* exp = nullptr;  // expand buffers of kg_expand_batch_device calls on this stream (kg_expand.hip)
  void* pinned = nullptr;  // 64 KiB of pinned host memory for small device->host readbacks
  kg_query* unpacked = nullptr;  // packed device batches that need the original queries (a program)
  size_t unpacked_n = 0;
  void* host_buf(size_t bytes);
  ~Workspace();
};

// One in-flight batch between check_batch_begin and check_batch_end (kg_check.hip).
struct BatchPending {
  kg_stats* stats = nullptr;
  uint8_t* d_out = nullptr;
  uint32_t* d_err = nullptr;
  bool grid_pending = false;
  const uint32_t *grid_list = nullptr, *grid_count = nullptr;
  const RQuery* rq = nullptr;
  int32_t gdepth = 5;
  size_t n = 0;
  // formula split: the batch ran as the originals + leaf sub-checks into split buffers; the
  // requested results are combined into f_out / f_err at the end
  bool split = false;
  size_t f_n = 0;
  uint8_t* f_out = nullptr;
  uint32_t* f_err = nullptr;
  const uint2* f_ref = nullptr;
  void* ctl_host = nullptr;
  GridStats gs;
};

// Host interning map (u64 key (ns, rel, obj) -> node id), open addressing.  Kept by tuple-built
// snapshots so kg_snapshot_apply can intern a delta's new nodes without rebuilding it.
struct HostMap {
  std::vector<uint64_t> k;
  std::vector<uint32_t> v;
  uint64_t mask = 0, n = 0;
  void init(uint64_t cap) {
    uint64_t c = 16;
    while (c < cap * 2) c <<= 1;
    k.assign(c, EMPTY64);
    v.assign(c, 0);
    mask = c - 1;
    n = 0;
  }
  void grow() {
    std::vector<uint64_t> ok;
    std::vector<uint32_t> ov;
    ok.swap(k);
    ov.swap(v);
    init(ok.size());
    for (size_t i = 0; i < ok.size(); i++)
      if (ok[i] != EMPTY64) put(ok[i], ov[i]);
  }
  // returns the existing value or inserts val
  uint32_t put(uint64_t key, uint32_t val) {
    if ((n + 1) * 2 > k.size()) grow();
    uint64_t i = mix64(key) & mask;
    while (k[i] != EMPTY64) {
      if (k[i] == key) return v[i];
      i = (i + 1) & mask;
    }
    k[i] = key;
    v[i] = val;
    n++;
    return val;
  }
  uint32_t get(uint64_t key) const {
    if (k.empty()) return NONE;
    uint64_t i = mix64(key) & mask;
    while (k[i] != EMPTY64) {
      if (k[i] == key) return v[i];
      i = (i + 1) & mask;
    }
    return NONE;
  }
};

// One stream's hash-sharded batch state (kg_shard.hip).
struct ShardCtx {
  hipStream_t stream = nullptr;
  int device = -1;
  void* vis = nullptr;  // per-batch visited table of (query, node)
  uint64_t vis_slots = 0;
  void* heavy = nullptr;  // hub rows a level hands to k_shard_heavy (+ count)
  void* qcnt = nullptr;   // per-batch escalation counters (hashed by query)
  void* qinfo = nullptr;  // per query slot (root, subject, depth, seeded)
  size_t qinfo_n = 0;
  bool final = false;      // the batch's final forward phase (kg_shard_refwd_seed): no escalation
  uint32_t* ref = nullptr;  // formula split: plan of every query of the batch
  size_t ref_n = 0;
  uint32_t* bits = nullptr;  // kg_shard_levels: the batch's done bitmap
  size_t bits_n = 0;
  uint32_t* cnt8 = nullptr;  // kg_shard_levels: per-XCD sub-bucket counters of the two level buffers (+ flags)
  int32_t gdepth = 0;        // the batch's global depth (kg_shard_seed): packed records need depths < 256
  ~ShardCtx();
};

struct Snapshot;
struct ShardComm;  // kg_shard_comm.hip: a transport bound to one stream's sharded batches

// A deep copy of the kg_dict + kg_rewrite_prog a snapshot was built with (the sharded general phase
// builds a snapshot of gathered rows with the same program).
struct ProgCopy {
  bool have = false;
  kg_dict dict{};
  std::vector<uint8_t> ns_has_rel;
  std::vector<uint32_t> rel_ns, rel_rel;
  std::vector<int32_t> rel_root;
  std::vector<kg_rw_node> rw;
  std::vector<int32_t> child;
  kg_rewrite_prog view() const {
    kg_rewrite_prog p{};
    p.n_ns = (uint32_t)ns_has_rel.size();
    p.ns_has_rel = ns_has_rel.data();
    p.n_rel = (uint32_t)rel_ns.size();
    p.rel_ns = rel_ns.data();
    p.rel_rel = rel_rel.data();
    p.rel_root = rel_root.data();
    p.n_rw = (uint32_t)rw.size();
    p.rw = rw.data();
    p.n_child = (uint32_t)child.size();
    p.child = child.data();
    return p;
  }
};

// Host-buffer batches (kg_check_batch, kg_expand_batch): a call checks out one lane set (one lane per
// replica -- its own HIP stream, hence its own batch workspace, pinned staging for queries and
// results, and device buffers, all grown on demand) from the snapshot's bounded pool and returns it
// when done, so thread churn (a Go server's cgo calls each pin an OS thread) never grows streams or
// HBM past the pool's cap; at the cap a call waits for a set to come back.
struct Lane {
  Snapshot* rep = nullptr;
  int device = -1;
  hipStream_t stream = nullptr;
  Workspace* w = nullptr;
  kg_query* h_q = nullptr;
  uint8_t* h_out = nullptr;
  uint32_t* h_err = nullptr;
  kg_query* d_q = nullptr;
  uint8_t* d_out = nullptr;
  uint32_t* d_err = nullptr;
  size_t cap = 0;
  void* exp = nullptr;  // expand buffers of this lane (kg_expand.hip)
  // kg_check_batch_packed: packed queries on the device (staged through h_q) and the error list
  kg_query_packed* d_pk = nullptr;
  uint32_t* d_el = nullptr;  // count word, pad, then (index, code) pairs: room for every query of the chunk
  uint32_t* h_el = nullptr;  // pinned: the count and the first EL_PREFETCH pairs, read back with the answers
  size_t pk_cap = 0;
  static constexpr size_t EL_PREFETCH = 4096;
  int reserve(size_t n);
  int reserve_packed(size_t n);
  ~Lane();
};

struct Snapshot {
  int device = -1;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  std::mutex mu;  // expand / hash-sharded calls and tuning (they run on the snapshot's own stream)
  DevSnap ds{};
  uint32_t wildcard_rel = NONE;
  bool has_program = false;
  bool is_synth = false;
  SynthLayout synth{};
  uint64_t h_row_off_last = 0, n_set_edges = 0, device_bytes = 0;
  uint64_t n_check_rows = 0;  // entries of the check rows (crow; == h_row_off_last without materialisation)
  uint64_t n_virtual = 0, n_virtual_new = 0;  // materialised rewrite nodes (kg_augment.hip), of them new ids
  int materialize = 1;  // rewrite materialisation at build (KG_MATERIALIZE=0 turns it off)
  std::vector<uint8_t> h_virt;  // [n_ns * n_rel] materialised union relations (kg_augment.hip)
  uint8_t* d_virt = nullptr;    // the same on the device (hash-sharded seed)
  // boolean rewrites over union / plain relations (kg_formula.hip): per (ns, rel) plan index or -1
  int32_t* d_fidx = nullptr;
  void* d_fplans = nullptr;
  uint32_t n_fplans = 0, fp_leaves = 0;  // plans, most leaves of one plan
  std::vector<std::pair<void*, size_t>> allocs;
  // host mirrors (host-tuple path); hmap + h_nd_* are handed on to a snapshot kg_snapshot_apply
  // builds from this one
  HostMap hmap;
  uint64_t* d_row_key = nullptr;  // per row entry order key (kg_snapshot_create_ordered), or null
  std::vector<uint32_t> h_nd_ns, h_nd_obj, h_nd_rel, h_row_subj;
  std::vector<uint64_t> h_row_off, h_adj_off;
  std::vector<uint8_t> h_relflags;
  std::vector<int32_t> h_relroot;
  std::vector<RwNode> h_rw;
  std::vector<int32_t> h_rwchild;
  // per-stream batch workspaces (check batches on different streams run concurrently)
  std::mutex ws_mu;
  std::vector<Workspace*> wss;
  Workspace* workspace(hipStream_t st);  // finds or creates the workspace of stream st (NULL = stream)
  uint64_t batch_seq = 0;
  uint32_t shard_rank = 0, shard_n = 1;  // hash-sharded mode (set before create)
  // per-stream batch state of the hash-sharded mode (kg_shard.hip), so batches on different streams
  // can be in flight at once; created by the first kg_shard_seed on a stream
  std::vector<ShardCtx*> shard_ctxs;
  ShardCtx* shard_ctx(hipStream_t st, bool create = true);  // st == NULL: the snapshot's stream
  // sharded batches inside the library (kg_shard_comm.hip): a transport per stream, reference-counted
  // (a caller inside a batch keeps its binding alive across kg_shard_comm_release / a re-bind)
  std::mutex comm_mu;
  std::vector<std::shared_ptr<ShardComm>> comms;
  std::atomic<int> n_comms{0};  // comms.size(): the replicated path's lock-free "nothing bound" test
  int shard_force_exchange = 0;  // kg_snapshot_tune("shard_force_exchange"): one rank runs the N > 1 protocol
  int shard_local = 1;           // kg_snapshot_tune("shard_local"): one rank runs the replica tier chain
  int shard_remote_meta = 1;     // kg_snapshot_tune("shard_remote_meta"): bind-time remote child metadata (DevSnap)
  uint32_t shard_max_reruns = 0;  // kg_snapshot_tune("shard_max_reruns"): overflow reruns per batch (0: max(4, exchanges))
  uint64_t shard_max_bytes = 0;   // kg_snapshot_tune("shard_max_bytes"): bucket buffers cap (0: 1/4 of free HBM)
  int shard_force_overflow = 0;   // kg_snapshot_tune("shard_force_overflow"): tests -- every run overflows
  uint32_t rel_span = 0;          // 1 + the largest relation id of any node (0: not yet computed)
  ProgCopy prog_copy;  // the program the snapshot was built with (the general phase's region snapshots)
  uint32_t* shard_held = nullptr;  // holder bitmap OR-ed over every rank (kg_shard_held), or null
  uint32_t shard_held_n = 0;
  int shard_vis_log2 = 23;
  uint32_t shard_bucket0 = 0;  // kg_snapshot_tune("shard_bucket"): first bucket size of new in-library bindings (0: by batch)
  uint32_t shard_wgs = 8;  // k_shard_level workgroups per CU
  uint32_t shard_heavy = 64;  // kg_snapshot_tune("shard_heavy"): set rows longer than this go to k_shard_heavy (r3p A/B)
  uint32_t shard_budget = 0;       // kg_snapshot_tune("shard_budget"): forward set edges per query and rank (0 = off)
  uint32_t shard_back_budget = 1u << 14;  // kg_snapshot_tune("shard_back_budget"): reverse edges per query and rank
  uint32_t stream_ecap = 512;  // kg_snapshot_tune("stream_ecap"): stream-tier edge budget per query (0 = none)
  // kg_snapshot_tune("expand_gw"): pass-1 overflows of kg_expand_batch run gather-then-walk (1) or the
  // hash pass directly (0); "expand_skip_lds" (tests): 1 = every root skips the LDS passes, 2 = the
  // 16-lane walkers (pass 0) are skipped and the 64-lane pass takes every root
  int expand_gw = 1;
  int expand_skip_lds = 0;
  // kg_snapshot_tune("level_events"): batches with stats time every tail-tier level launch with a HIP
  // event pair (kg_stats tail_ms); off by default -- the records leave gaps between the launches
  int level_events = 0;
  // k_expand_gw: longest wait (us) of a large slot for a small slot's hand-on before it gives its ticket up
  uint32_t expand_gw_wait_us = 100000;
  uint32_t stream_steal = 4;   // kg_snapshot_tune("stream_steal"): XCD ranges a k_stream4 wave dequeues from (1..8)
  // Occupancy defaults (library-wide, measured with several batches in flight, the way a server keeps
  // them: C2 and C3 A/Bs in profiles/r2gw_tier_wgs_sweep.jsonl, r2v_occupancy_sweep.jsonl,
  // r2bw_back_wgs_ab.jsonl; a one-batch-at-a-time caller loses < 5 % with them)
  // C2 (round 4, profiles/r4w_grid_stream_wgs_ab.jsonl): k_grid_level 2 and k_stream4 2 workgroups per CU
  // (the LDS a third stream workgroup held now serves the other batches' tail tiers): 7.00 -> 7.20 x 10^9;
  // C3 keeps 4 / 3 through bench.py
  int grid_wgs = 2;          // kg_snapshot_tune("grid_wgs"): k_grid_level workgroups per CU
  int stream_wgs = 2;        // kg_snapshot_tune("stream_wgs"): k_stream4 workgroups per CU (LDS left to other batches)
  int interp_wgs = 6;        // k_interp_lds workgroups (4 waves) per CU (6 fit the LDS)
  uint32_t interp_cap2 = 0;  // kg_snapshot_tune("interp_cap2"): pass-2 BFS list cap of the rewrite path (0 = 256 Ki)
  // k_back workgroups per CU (1..3, LDS allows 3; C3 prefers 1).  3: one wave per query for up to 3 Ki
  // hand-ons (C2 hands on ~2.2 k per 1 M batch: at 2, ~170 of them waited for a second pass on a
  // freed wave; 6.3 -> 6.8 x 10^9 checks/s, profiles/r4s_back_wgs_ab.jsonl)
  int back_wgs = 3;          // kg_snapshot_tune("back_wgs")
  uint32_t back_edges = 0;   // kg_snapshot_tune("back_edges"): k_back<64>'s reverse-edge budget per query (0 = 2^12)
  uint64_t grid_small_cap = 0;  // kg_snapshot_tune("grid_cap"): workspace grid-log entries (0 = 16 Mi; tests)
  int grid_ms = 1;  // kg_snapshot_tune("grid_ms"): grid-tier queries as MS-BFS when the dense masks fit (0: off)
  size_t grid_ms_bytes = 1ull << 30;  // kg_snapshot_tune("grid_ms_bytes"): MS-BFS mask budget per workspace
  int grid_ms_words = 8;     // kg_snapshot_tune("grid_ms_words"): 64-bit words per MS-BFS mask (64 queries each)
  uint32_t grid_ms_tg_cap = 256;  // kg_snapshot_tune("grid_ms_tg_cap"): holders above which MS-BFS probes dset instead
  uint64_t grid_ms_cap = 0;  // kg_snapshot_tune("grid_ms_cap"): MS-BFS entries per level buffer (0 = 16 Mi; tests)
  // replicas: the same snapshot on more devices (kg_snapshot_create's device mask); this object is
  // replica 0 and owns the others.  Host-buffer batches and expands are split over all of them.
  std::vector<Snapshot*> peers;
  Snapshot* replica(size_t i) { return i == 0 ? this : peers[i - 1]; }
  size_t n_replicas() const { return 1 + peers.size(); }
  std::mutex lane_mu;
  std::condition_variable lane_cv;
  std::list<std::vector<Lane*>> lane_sets;     // every set created (list: stable addresses)
  std::vector<std::vector<Lane*>*> lane_free;  // sets not checked out (LIFO: the warmest first)
  size_t lane_cap = 32;                        // kg_snapshot_tune("max_lanes"): concurrent host-buffer calls
  std::vector<Lane*>* lanes_acquire();         // a free lane set (created up to lane_cap; waits at the cap)
  void lanes_release(std::vector<Lane*>* v);
  std::atomic<uint64_t> rr_next{0};      // replica rotation of batches smaller than one chunk per replica
  // The grid tier's full-size pool (a log that holds every node): shared by the workspaces, used
  // one query at a time by a round whose single query overflowed its workspace's pool.
  std::mutex giant_mu;
  GridPool giant;

  ~Snapshot();
  int init_device(int dev);
  int alloc(void** p, size_t bytes);
  void free_alloc(const void* p);
  int create_from_tuples(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog,
                         const uint64_t* keys = nullptr);
  // kg_delta.hip: this snapshot = base's rows + inserted - deleted, built on the device
  int create_from_delta(Snapshot* base, const kg_tuple* ins, const uint64_t* ins_keys, size_t n_ins,
                        const kg_tuple* del, size_t n_del, const kg_dict* dict, const kg_rewrite_prog* prog);
  int device_flags();  // purity closure on the device (rewrite / undeclared relations reachable)
  int create_synthetic(const kg_synth_params* p, const kg_rewrite_prog* prog);
  int upload_program(const kg_dict* dict, const kg_rewrite_prog* prog);
  int augment_rewrites();  // kg_augment.hip: monotone rewrites -> plain union nodes
  int build_formulas();    // kg_formula.hip: boolean rewrites -> leaf sub-checks
  int build_hash_tables();
  int build_reverse();
  uint8_t host_relflag(uint32_t ns, uint32_t rel) const;
  int64_t export_rows(kg_tuple* out, uint64_t cap);
  int64_t rows_of(const kg_set* keys, size_t n, uint64_t* offsets, kg_tuple* out, uint64_t cap);  // kg_rows.hip
};

// kg_check.hip
// d_pk (packed queries, d_q unused): read by k_resolve itself when nothing else of the batch needs the
// original queries (no namespace program), else unpacked into the workspace first
int check_batch_device(Snapshot* s, Workspace* w, const kg_query* d_q, size_t n, int32_t global_max_depth,
                       uint8_t* d_out, uint32_t* d_err, kg_stats* stats, const kg_query_packed* d_pk = nullptr);
int check_batch_begin(Snapshot* s, Workspace* w, const kg_query* d_q, size_t n, int32_t global_max_depth,
                      uint8_t* d_out, uint32_t* d_err, kg_stats* stats, BatchPending* bp,
                      const kg_query_packed* d_pk = nullptr);
int check_batch_end(Snapshot* s, Workspace* w, BatchPending* bp, bool* reran, bool blocking = false);
int synth_queries(Snapshot* s, uint64_t seed, size_t n, kg_query* d_q);
// kg_check_batch_packed: packed queries -> kg_query on the device; the KG_ERROR answers of [0, n) as
// (base + index, code) pairs after a count word (d_list: 2 + 2 * cap words)
int unpack_queries(const kg_query_packed* d_pk, size_t n, kg_query* d_q, hipStream_t stream);
int pack_queries(const kg_query* d_q, size_t n, kg_query_packed* d_pk, uint32_t* d_bad, hipStream_t stream);
int error_list(const uint8_t* d_out, const uint32_t* d_err, size_t n, uint32_t base, uint32_t* d_list, size_t cap,
               hipStream_t stream);
// kg_formula.hip: split a batch's decomposable queries into leaf checks / combine their results
int formula_split(Snapshot* s, Workspace* w, const kg_query* d_q, size_t n, int32_t gdepth, const kg_query** q2,
                  size_t* n2, const uint32_t** n_extra, uint8_t** out2, uint32_t** err2, const uint2** ref);
int formula_combine(Snapshot* s, Workspace* w, size_t n, const uint2* ref, const uint8_t* out2, const uint32_t* err2,
                    uint8_t* d_out, uint32_t* d_err);
// kg_shard.hip
int shard_seed(Snapshot* s, const kg_query* d_q, size_t n, int32_t gdepth, kg_frec* d_out, size_t cap,
               uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, hipStream_t stream);
int shard_level(Snapshot* s, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out, size_t cap,
                uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done, uint32_t done_words,
                hipStream_t stream, uint32_t n_seg = 1, size_t seg_cap = 0, bool prezeroed = false);
// the stream's hub-row list head (zeroed before each level; kg_shard_comm's fused pre-level kernel)
unsigned long long* shard_heavy_head(Snapshot* s, hipStream_t stream);
// the exchange protocol's fused pre-exchange kernel (accumulators, next counters, hub head, done bitmap)
int shard_pre_level(Snapshot* s, hipStream_t stream, const uint32_t* d_cur, uint32_t N, uint32_t B, uint32_t me,
                    unsigned long long* acc, unsigned long long* lvl, uint32_t* d_next_counts, size_t n,
                    const uint8_t* d_res, const uint32_t* d_err, int with_esc, uint32_t* d_bits, uint32_t words);
int shard_done(Snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, int with_esc, uint32_t* d_bits,
               uint32_t words, hipStream_t stream);
int shard_levels(Snapshot* s, int levels, kg_frec* d_buf[2], size_t cap, uint32_t* d_counts[2], int start,
                 uint8_t* d_res, uint32_t* d_err, size_t slots, int esc_mode, int* end, hipStream_t stream,
                 unsigned long long* need = nullptr);  // *need: the bucket size the levels needed
int shard_back_list(Snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_list, size_t cap,
                    uint32_t* d_counts, hipStream_t stream);
int shard_back_seed(Snapshot* s, const kg_frec* d_list, size_t m, const uint32_t* d_m, kg_frec* d_out, size_t cap,
                    uint32_t* d_counts, hipStream_t stream, uint32_t n_seg = 1, size_t seg_cap = 0);
int shard_back_level(Snapshot* s, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out, size_t cap,
                     uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done, uint32_t done_words,
                     hipStream_t stream, uint32_t n_seg = 1, size_t seg_cap = 0);
bool shard_escalates(const Snapshot* s);  // the escalation phases run (shard_budget, no program, reverse index)
int shard_refwd_seed(Snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_out, size_t cap,
                     uint32_t* d_counts, hipStream_t stream);
int shard_held(Snapshot* s, uint32_t* d_bits, size_t words, int import, hipStream_t stream);
// remote child metadata (DevSnap::remote_meta): this rank's per-node (row length, signature) words,
// then -- after the caller's max all-reduce -- the owners' values written into adjx
int shard_meta_local(Snapshot* s, uint64_t* d_meta, hipStream_t st);
int shard_meta_apply(Snapshot* s, const uint64_t* d_meta, hipStream_t st);
int shard_finish(Snapshot* s, size_t n, uint8_t* d_res, uint32_t* d_err, hipStream_t stream);
size_t shard_result_slots(const Snapshot* s, size_t n);
size_t shard_slot_limit();  // result slots one sharded batch can address (query index bits of kg_frec.q)
int shard_bad_nodes(Snapshot* s, uint64_t* count);
// kg_shard_comm.hip: sharded batches inside the library
void shard_comms_free(Snapshot* s);
std::shared_ptr<ShardComm> shard_comm_of(Snapshot* s, hipStream_t st);  // the transport bound to st, or null
int shard_check(Snapshot* s, ShardComm* c, const kg_query* d_q, size_t n, int32_t gdepth, uint8_t* d_out,
                uint32_t* d_err, kg_stats* stats);
int shard_check_entry(Snapshot* s, hipStream_t st, const kg_query* d_q, size_t n, int32_t gdepth, uint8_t* d_out,
                      uint32_t* d_err, kg_stats* stats, bool* handled);  // kg_check_batch_device on a bound stream
int shard_expand(Snapshot* s, const kg_set* roots, size_t n, int32_t gdepth, kg_tree_buf* out);  // collective
int shard_check_host_entry(Snapshot* s, const kg_query* q, size_t n, int32_t gdepth, uint8_t* out, uint32_t* err,
                           kg_stats* stats);  // kg_check_batch on a sharded snapshot (its own stream's binding)
// kg_grid.hip
int grid_reserve(Snapshot* s);  // allocates the shared full-size grid pool now (kg_snapshot_tune "grid_reserve")
// kg_expand.hip
// runs on `stream` with the lane's cached device buffers (*bufs, created on first use)
// dev_io: roots is a device pointer and the trees stay in HBM (kg_expand_batch_device: out->nodes /
// out->root_off device buffers of the per-device output pool, out->pinned = KG_TREE_DEVICE | device)
int expand_batch(Snapshot* s, hipStream_t stream, void** bufs, const kg_set* roots, size_t n, int32_t global,
                 kg_tree_buf* out, bool dev_io = false);
void expand_bufs_free(void* bufs);
void* tree_pool_get(size_t bytes);  // pinned host memory for tree outputs (kg_tree_free returns it)
void tree_pool_put(void* p, size_t bytes);
constexpr uint64_t KG_TREE_DEVICE = 0x100;  // kg_tree_buf.pinned: device-resident trees (low byte: the device)
void* tree_dev_get(int device, size_t bytes);  // device memory for device-resident tree outputs
void tree_dev_put(int device, void* p, size_t bytes);

}  // namespace kg
