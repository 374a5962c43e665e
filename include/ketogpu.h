/*
 * ketogpu.h -- C ABI of libketogpu.so, the MI355X (gfx950) batched permission-check engine.
 *
 * This is the drop-in boundary for Ory Keto's check / expand hot path.  A Go host binds it
 * through cgo; the Python host in keto_amd/ binds it through ctypes.
 * Plain C types only: dense u32 ids, POD structs, caller-owned input/output buffers.
 *
 * Every entry point names the reference interface it replaces (paths relative to the
 * reference checkout, ryukinix/keto @ 2025-01-31):
 *
 *   kg_snapshot_create   relationtuple.Manager.GetRelationTuples  internal/relationtuple/definitions.go:19-25
 *                        + Persister.GetRelationTuples           internal/persistence/sql/relationtuples.go:203-244
 *                        + namespace AST / config                internal/namespace/ast/ast_definitions.go:5-68,
 *                                                                internal/check/engine.go:209-229 (astRelationFor)
 *   kg_check_batch       check.Engine.CheckIsMember (looped)      internal/check/engine.go:54-60
 *                        check.Engine.CheckRelationTuple          internal/check/engine.go:65-80
 *                        (new BatchCheck, SURVEY.md 8b: equals a loop of CheckIsMember)
 *   kg_expand_batch      expand.Engine.BuildTree                  internal/expand/engine.go:35-104
 *   kg_last_error        herodot / errors.WithStack message text  internal/check/engine.go:228, rewrites.go:15-17
 *
 * Id spaces (the caller interns strings; the reference maps strings to UUIDv5 first,
 * internal/persistence/sql/uuid_mapping.go:31-66 -- a dense id per UUID is equivalent):
 *   namespace ids  < 65535, relation ids < 65535 (global over namespaces),
 *   object ids     < 2^31-1, one space for objects AND subject ids (both are UUIDs upstream).
 * Rows must be passed in shard_id order (the order GetRelationTuples returns them).
 */
#ifndef KETOGPU_H
#define KETOGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KG_SUBJECT_ID 0xFFFFFFFFu /* kg_tuple.sns value marking a SubjectID subject (id in sobj) */

/* One relation tuple ns:obj#rel@subject (internal/relationtuple/definitions.go:46-57). */
typedef struct {
  uint32_t ns, obj, rel;    /* namespace, object, relation                         */
  uint32_t sns, sobj, srel; /* subject set (sns,sobj,srel), or sns = KG_SUBJECT_ID */
} kg_tuple;

/* A check request: the tuple to test plus the request max-depth (<= 0 means "use global"),
 * exactly the arguments of CheckIsMember(ctx, tuple, restDepth). */
typedef struct {
  kg_tuple t;
  int32_t max_depth;
} kg_query;

/* The same request in 16 bytes (kg_check_batch_packed: the host boundary moves 16 B per check in
 * instead of 28).  Namespace and relation ids < 4095 (KG_PACK_ID_MAX), the subject-id marker
 * KG_PACK_SUBJECT_ID in the subject namespace field, request max-depth 0..65535 (0: use global; the
 * configured max_read_depth's own range, embedx/config.schema.json:308-315; a negative depth is 0):
 *   obj, sobj  as in kg_tuple
 *   w2         ns (bits 0-11) | rel (bits 12-23) | sns bits 0-7 (bits 24-31)
 *   w3         sns bits 8-11 (bits 0-3) | srel (bits 4-15) | max_depth (bits 16-31) */
typedef struct {
  uint32_t obj, sobj, w2, w3;
} kg_query_packed;
#define KG_PACK_ID_MAX 4094u
#define KG_PACK_SUBJECT_ID 4095u
/* Returns 0, or -2 when an id does not fit (use kg_check_batch). */
static inline int kg_pack_query(const kg_query* q, kg_query_packed* p) {
  const uint32_t sns = q->t.sns == 0xFFFFFFFFu ? KG_PACK_SUBJECT_ID : q->t.sns;
  const uint32_t srel = q->t.sns == 0xFFFFFFFFu ? 0u : q->t.srel;
  const uint32_t d = q->max_depth <= 0 ? 0u : (q->max_depth > 65535 ? 65535u : (uint32_t)q->max_depth);
  if (q->t.ns > KG_PACK_ID_MAX || q->t.rel > KG_PACK_ID_MAX || (sns != KG_PACK_SUBJECT_ID && sns > KG_PACK_ID_MAX) ||
      srel > KG_PACK_ID_MAX)
    return -2;
  p->obj = q->t.obj;
  p->sobj = q->t.sobj;
  p->w2 = q->t.ns | (q->t.rel << 12) | ((sns & 0xFFu) << 24);
  p->w3 = (sns >> 8) | (srel << 4) | (d << 16);
  return 0;
}

/* An expand root: a subject set, or a subject id (sns = KG_SUBJECT_ID) -- BuildTree's Subject. */
typedef struct {
  uint32_t sns, sobj, srel;
  int32_t max_depth;
} kg_set;

/* Interning metadata. */
typedef struct {
  uint32_t n_namespaces;
  uint32_t n_relations;
  uint32_t wildcard_rel; /* id of the "..." relation (engine.go:40), or 0xFFFFFFFF */
} kg_dict;

/* Compiled namespace configuration (the OPL / ast.Relation rewrites).
 * rw nodes: kind 0 = or, 1 = and (SubjectSetRewrite), 2 = ComputedSubjectSet(rel),
 *           3 = TupleToSubjectSet(rel, crel), 4 = InvertResult (its one child in child[first]).
 * Children of node i are child[first .. first+count).  Relation j of namespace rel_ns[j]
 * named rel_rel[j] has rewrite root rel_root[j] (-1: declared without rewrite).
 * ns_has_rel[ns] != 0 when the namespace is configured with at least one relation
 * (engine.go:219-228: otherwise every relation is accepted without rewrite). */
typedef struct {
  int32_t kind, rel, crel, first, count;
} kg_rw_node;

typedef struct {
  uint32_t n_ns;
  const uint8_t* ns_has_rel;
  uint32_t n_rel;
  const uint32_t* rel_ns;
  const uint32_t* rel_rel;
  const int32_t* rel_root;
  uint32_t n_rw;
  const kg_rw_node* rw;
  uint32_t n_child;
  const int32_t* child;
} kg_rewrite_prog;

/* Per-batch counters; the algorithmic-byte model of SURVEY.md 8d is
 * B = 8*rows_opened + 4*edges_read + 16*direct_probes + 16*frontier_hbm. */
typedef struct {
  uint64_t rows_opened;
  uint64_t edges_read;
  uint64_t direct_probes;
  uint64_t frontier_hbm;
  uint64_t n_light, n_heavy, n_general; /* queries finished by the stream tier / reaching the grid tier / the interpreter */
  uint64_t n_medium;                    /* reserved (0) */
  uint64_t light_rows_opened, light_edges_read, light_probes; /* the stream tier's (k_stream4's) share of the counters */
  double kernel_ms;                     /* device time of the whole batch (HIP events)  */
  double light_ms;                      /* device time of the k_stream4 launch           */
  uint64_t n_wide;                      /* reserved (0) */
  uint64_t n_grid;                      /* queries resolved by the grid tier             */
  uint64_t n_back;                      /* queries resolved by the backward tier         */
  uint64_t n_no_holder;                 /* queries answered NotMember by k_resolve: no row holds the subject */
  uint64_t back_rows, back_edges;       /* backward tier: parent lists opened / parents read */
  uint64_t light_steps;                 /* k_stream4: wave steps (one HBM round trip each) */
  uint64_t light_waves;                 /* k_stream4: waves that ran                     */
  uint64_t light_wave_ticks;            /* k_stream4: sum of wave lifetimes (100 MHz ticks) */
  uint64_t light_span_ticks;            /* k_stream4: first wave start to last wave end  */
  uint64_t light_wave_max_ticks;        /* k_stream4: longest wave lifetime              */
  /* the tail tier's level kernels (round 6): the grid tier's k_grid_level or the MS-BFS k_ms_level */
  double tail_ms;                       /* summed device time of those launches (HIP events per launch; only with kg_snapshot_tune "level_events" 1) */
  uint64_t tail_launches;               /* level launches of the batch (the first 64 are timed)          */
  uint64_t tail_kind;                   /* 0 none, 1 k_grid_level, 2 k_ms_level                          */
  uint64_t tail_rows, tail_edges, tail_probes, tail_logged; /* the tail tier's share of the counters    */
  uint64_t ms_edges_loaded;             /* k_ms_level: adjx records loaded (an edge with work in any word) */
  uint64_t ms_words_active;             /* k_ms_level: (edge, 64-query word) pairs with work              */
  double split_ms;                      /* device time of the formula split (k_fsplit), 0 when none      */
} kg_stats;

/* Per-query outputs of kg_check_batch. */
#define KG_NOT_MEMBER 0
#define KG_IS_MEMBER 1
#define KG_ERROR 2

/* err_code values (mirror the reference's error sources). */
#define KG_ERR_NONE 0
#define KG_ERR_RELATION_NOT_FOUND 1 /* engine.go:228  relation %q not found            */
#define KG_ERR_NOT_IMPLEMENTED 2    /* rewrites.go:15-17 not implemented                */
#define KG_ERR_REWRITE_CYCLE 3      /* computed-subject-set cycle (reference recurses forever) */
#define KG_ERR_RESOURCE 4           /* exceeded an engine capacity                       */

/* Expand output: pre-order records.  type 1 = union, 2 = leaf (ketoapi TreeNodeUnion/Leaf).
 * Root r of the batch owns records [root_off[r], root_off[r+1]); an empty range = nil tree. */
typedef struct {
  uint8_t type;
  uint8_t is_set;  /* 1: subject set (ns,obj,rel); 0: subject id in obj */
  uint16_t pad;
  uint32_t ns, obj, rel;
  uint32_t n_children;
} kg_tree_node;

typedef struct {
  kg_tree_node* nodes;
  uint64_t n_nodes;
  uint64_t* root_off; /* n_roots + 1 entries */
  uint64_t n_roots;
  double kernel_ms;   /* device time of the expand kernels (HIP events), filled by the library */
  uint64_t pinned;    /* library use: nodes lives in the library's pinned-host pool (kg_tree_free returns it) */
} kg_tree_buf;

typedef struct kg_snapshot kg_snapshot;

/* Synthetic "Drive-like" tuple graph generated on the device.
 * Deterministic in (seed, index); kg_snapshot_export returns its rows. */
typedef struct {
  uint64_t n_tuples_target; /* ~total tuples (docs#viewer + group#member)           */
  uint64_t seed;
  uint32_t n_layers;        /* group layers (8)                                    */
  uint32_t max_degree;      /* out-degree truncation (1e5)                        */
  float set_fraction;       /* fraction of group#member subjects that are subject sets */
  float doc_set_fraction;   /* fraction of doc#viewer subjects that are L0 groups  */
  uint32_t preset;          /* 0 = C2/C4 rewrite-free; 1 = C3 (+ folders, OPL view/edit/share) */
  float doc_alpha;          /* Pareto tail index of doc#viewer out-degrees (0 = 1.3)         */
  float group_alpha;        /* Pareto tail index of group#member out-degrees (0 = 1.1); 0.5 =
                               the degree law P(k) ~ k^-1.5 (Zipf 1.5) of SURVEY.md 8d       */
} kg_synth_params;

/* ---- snapshot --------------------------------------------------------------------------- */
/* device_mask: bit d set = a replica of the snapshot on device d (0 = device 0 only).  Every
 * replica holds the whole snapshot (1 B synthetic tuples take 69 GB of a 288 GB MI355X rewrite-free,
 * 194 GB with C3's materialised rewrites); kg_check_batch and
 * kg_expand_batch split their host-buffer batches over the replicas inside the call, which is how
 * one `keto serve` process (one check.Engine, internal/driver/registry_default.go:180-185) uses
 * every GPU of the node.  Replicas are built concurrently. */
int kg_snapshot_create(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog,
                       int device_mask, kg_snapshot** out);
/* Rows with an order key each (ascending: the persister's shard ids, relationtuples.go:203-244
 * ORDER BY shard_id), kept per row so kg_snapshot_apply can place inserted rows in key order. */
int kg_snapshot_create_ordered(const kg_tuple* rows, const uint64_t* keys, size_t n, const kg_dict* dict,
                               const kg_rewrite_prog* prog, const int* devices, int n_devices, kg_snapshot** out);
/* Incremental refresh (TransactRelationTuples, internal/persistence/sql/relationtuples.go:260-270):
 * *out = base's rows, minus every row equal to a tuple in del (:164-185; deletes apply to base
 * rows), plus ins (ins_keys: their order keys, or NULL = after the node's existing rows).  Only the
 * delta is handled on the host; rows and every derived structure are rebuilt on the device, replica
 * by replica.  The base stays valid (in-flight batches keep reading it) but hands its host node map
 * on to *out: apply the next delta to *out, not to base (a second apply on the same base rebuilds
 * the map from the device).  Not concurrently on one base. */
int kg_snapshot_apply(kg_snapshot* base, const kg_tuple* ins, const uint64_t* ins_keys, size_t n_ins,
                      const kg_tuple* del, size_t n_del, const kg_dict* dict, const kg_rewrite_prog* prog,
                      kg_snapshot** out);
/* The same with an explicit device list; entries may repeat (several replicas on one device). */
int kg_snapshot_create_on(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog,
                          const int* devices, int n_devices, kg_snapshot** out);
/* prog: the namespace program compiled against the generator's ids (ns doc=0 group=1 user=2
 * folder=3; rel "..."=0 viewer=1 member=2 editor=3 owner=4 parents=5 blocked=6 view=7 edit=8
 * share=9), or NULL for none.  keto_amd/synth.py builds both. */
int kg_snapshot_synthetic(const kg_synth_params* params, const kg_rewrite_prog* prog, int device_mask,
                          kg_snapshot** out);
int kg_snapshot_synthetic_on(const kg_synth_params* params, const kg_rewrite_prog* prog, const int* devices,
                             int n_devices, kg_snapshot** out);
/* Number of replicas; their devices go to devices[0 .. min(count, cap)) (devices may be NULL). */
int kg_snapshot_replicas(const kg_snapshot* s, int* devices, int cap);
void kg_snapshot_destroy(kg_snapshot* s);
/* sizes: [0]=nodes [1]=rows [2]=set edges [3]=device bytes */
int kg_snapshot_info(const kg_snapshot* s, uint64_t* info4);
/* Rewrite materialisation at build (no reference counterpart; keto_amd/csrc/kg_augment.hip): every
 * relation whose rewrite is a union of `this` rows, computed subject sets and tuple-to-subject-sets
 * (internal/check/rewrites.go:30-260 restricted to `or`) is answered as one plain union node per
 * object.  out3: [0] union nodes, [1] of them new node ids (objects without a row of the relation
 * itself), [2] check-row entries (the direct tuples the union nodes hold).  KG_MATERIALIZE=0 in
 * the environment at snapshot creation turns it off. */
int kg_snapshot_materialized(const kg_snapshot* s, uint64_t* out3);
/* Engine knobs (no reference counterpart; tuning and tests).  Results never depend on any of them.
 * key "back": 1 = the backward tier (reverse search from the subject's holders, one wave per query,
 * then one workgroup per query) takes the stream tier's overflow before the grid tier, and k_resolve
 * answers queries whose subject no row holds; 2 = the same with the wave width only (its overflow
 * goes straight to the grid tier; default); 0 = off.
 * key "stream_ecap": edges a query may enqueue in the stream tier before it is handed to the
 * backward / grid tiers (default 512; 0 = no budget) -- cuts the stream kernel's tail of long walks.
 * key "resolve_unheld" (0..2): without a namespace program, k_resolve reads a subject id's holder
 * bit before the node map and answers an unheld subject NotMember without the lookup (default 1);
 * 2 = the bit is read only by queries that the node map and the root probe leave for the stream
 * tier; 0 = the bit beside the node-map lookup for every query.
 * key "device_sync" (0/1): the same for kg_check_batch_device when it waits (stats or a grid-tier
 * readback; default 1: asleep -- 5.6 -> 5.8 x 10^9 checks/s with 4 batches in flight).  key "host_sync" (0/1): kg_check_batch waits for its device work asleep on a blocking-sync event
 * (1, default: no core spins per in-flight batch) or spinning in hipStreamSynchronize (0).
 * key "stream_steal" (1..8): XCD ranges of the work list a k_stream4 wave dequeues from (default 4:
 * when the list drains every wave walks them, one atomic each on a few hot words).
 * key "stream_chunk" (1..64): queries a k_stream4 wave dequeues at once (default 64).
 * key "stream_wgs": k_stream4 workgroups per CU (0 = 2; default 2); "back_wgs" (1..3, default 3), "back_edges" (reverse edges one backward-tier query may read, 0 = 2^12)
 * and "grid_wgs" (1..64, default 2): k_back / k_grid_level workgroups per CU (defaults = bench.py's C2 set).  key "shard_vis": log2 of the
 * hash-sharded mode's per-batch (query, node) visited table (default 25).  key "interp_cap2"
 * (0..4194304): BFS list cap of the rewrite interpreter's many-slot HBM pass (0 = 256 Ki nodes);
 * queries that outgrow it rerun in the single full-size slot.  key "interp_wgs" (1..8): workgroups
 * of 4 query waves per CU in the interpreter's LDS pass (default 6).  key "grid_reserve": allocate
 * now the grid tier's shared full-size pool (used by a query that overflows a workspace's pool on
 * its own; otherwise allocated on first need).  key "grid_cap": log entries of a workspace's grid
 * pool (0 = 16 Mi; small values force the overflow paths in tests).  key "max_lanes" (1..1024, default
 * 32): lane sets (a stream, staging and workspace per replica) that concurrent kg_check_batch /
 * kg_expand_batch calls check out of the snapshot's pool; at the cap a call waits for one to return.
 * key "grid_ms" (0/1, default 1): the grid tier's queries run as a multi-source bit-parallel BFS,
 * 64 x "grid_ms_words" (1..16, default 8) queries per group sharing each level's walk, when one
 * group's dense per-node masks (32 B per word per node) fit an eighth of "grid_ms_bytes" (default
 * 2^30 per in-flight batch; the width halves until they do) -- graphs of up to ~4 M nodes.  key
 * "grid_ms_tg_cap" (default 256): a query whose subject has more holders is probed in dset per
 * newly reached node instead of marking its holders in the group's target masks.  key "grid_ms_cap": entries per MS-BFS level buffer (0 = 16 Mi; small values force the
 * overflow reruns in tests).
 * key "grid_bidir" (0..2^31-1, default 0): grid-tier slots whose subject has at most this many
 * holders alternate forward and backward turns (0: forward only).  key "expand_tail" (0/1, default
 * 1): the expand walk caches a root's last frontier in LDS.  key "expand_gw" (0/1, default 1): roots
 * that outgrow the LDS pass gather their neighbourhood in parallel and walk the copy (small and large
 * workgroup slots, then the hash pass); "expand_skip_lds" (0/1, tests): every root skips the LDS pass.
 * Hash-sharded mode: key "shard_wgs"
 * (1..64, default 8) k_shard_level workgroups per CU; "shard_heavy" (default 64) set rows longer than
 * this go to k_shard_heavy, which spreads their edges over the grid (0: every row); "shard_vis_mode"
 * 0 = exact (query, node) CAS table (default), 1 = lossy direct-mapped cache; "shard_pack" (0/1,
 * default 0): kg_shard_levels sends a locally owned child as its set-row begin and length (no
 * adj_off read at the next level; no namespace program, depths < 256); "shard_budget" /
 * "shard_back_budget": see kg_shard_back_* below; "shard_bucket" (0..2^26, default 0 = sized from the
 * batch): the first bucket size (records per destination) of in-library bindings made after it. */
int kg_snapshot_tune(kg_snapshot* s, const char* key, int64_t value);
/* Synthetic layout: ids6 = {n_docs, n_groups, n_users, n_folders, user_obj0, folder_obj0}
 * (doc d = object d, group g = object n_docs+g, user u = object user_obj0+u). */
int kg_synth_ids(const kg_snapshot* s, uint32_t* ids6);
/* Copies the snapshot's rows back (shard order) as kg_tuple, for oracle cross-checks.
 * rows may be NULL to query the count. */
int64_t kg_snapshot_export(const kg_snapshot* s, kg_tuple* rows, uint64_t cap);
/* GetRelationTuples(namespace, object, relation) for n keys at once (keys[i] = (ns, obj, rel) in
 * (sns, sobj, srel); max_depth ignored): the rows of each key in shard_id order, concatenated --
 * key i's rows are out[offsets[i] .. offsets[i+1]).  offsets[n+1] is always filled; out == NULL
 * returns the total only, cap < total is an error (-3).  Raw tuples (a materialised union node's
 * merged rows are not returned).  A sharded snapshot returns its own rows only.  Not a hot path:
 * the CheckRelationTuple tree walk (keto_amd/explain.py) reads rows through it.  Replaces
 * internal/persistence/sql/relationtuples.go:260-270 for the engines' reads. */
int64_t kg_snapshot_rows(const kg_snapshot* s, const kg_set* keys, size_t n, uint64_t* offsets, kg_tuple* out,
                         uint64_t cap);
/* Copies the row index back: row_off[nodes+1], row_subj[rows] (tagged: bit31 = subject set ->
 * node id, else subject id), node triples nd_ns/nd_obj/nd_rel[nodes].  For the CPU baseline. */
int kg_snapshot_export_csr(const kg_snapshot* s, uint64_t* row_off, uint32_t* row_subj, uint32_t* nd_ns,
                           uint32_t* nd_obj, uint32_t* nd_rel);

/* ---- check ------------------------------------------------------------------------------ */
/* Host buffers: q[n] in, out[n] (KG_NOT_MEMBER / KG_IS_MEMBER / KG_ERROR), err_code[n] (may be
 * NULL), stats (may be NULL; counters summed over replicas, kernel_ms = the slowest replica's).
 * Synchronous.  Thread-safe: every calling thread gets its own stream and pinned staging per
 * replica (kept for its later calls), so concurrent callers' batches overlap on the devices.
 * The batch is split over the replicas in contiguous chunks of >= 16384 queries. */
int kg_check_batch(kg_snapshot* s, const kg_query* q, size_t n, int32_t global_max_depth, uint8_t* out,
                   uint32_t* err_code, kg_stats* stats);
/* kg_check_batch with the narrow boundary (round 5): 16-B packed queries in (kg_query_packed, unpacked
 * on the device), 1 B per answer out, and the error codes only of the checks answered KG_ERROR, as a
 * sparse list: *n_err = how many there are; the first min(n_err, err_cap) of them, by ascending index,
 * in err_index[] / err_code[] (both may be NULL when err_cap is 0).  Same engine, answers and
 * threading as kg_check_batch: the reference's BatchCheck (one CheckIsMember per request,
 * internal/check/engine.go:54-60; error codes as kg_check_batch's err_code). */
int kg_check_batch_packed(kg_snapshot* s, const kg_query_packed* q, size_t n, int32_t global_max_depth, uint8_t* out,
                          uint32_t* err_index, uint32_t* err_code, size_t err_cap, size_t* n_err, kg_stats* stats);
/* Device-resident variant (replica 0 only: the pointers belong to its device): d_q / d_out / d_err are device pointers (HBM), stream is a
 * hipStream_t (NULL = the snapshot's stream).  Returns once the batch is enqueued; when queries
 * reach the grid tier the call waits for the wave tiers (the grid tier's size is read back), and
 * with stats != NULL it waits for the whole batch.  Every stream gets its own batch workspace
 * (scratch lists, tier pools, pinned readback), so calls on different streams -- e.g. one host
 * thread per stream -- keep several batches in flight on the device at once; calls on the same
 * stream are serialised.  kg_check_batch uses the snapshot's own stream. */
int kg_check_batch_device(kg_snapshot* s, const kg_query* d_q, size_t n, int32_t global_max_depth,
                          uint8_t* d_out, uint32_t* d_err, kg_stats* stats, void* stream);
/* kg_check_batch_device with 16-B packed queries in HBM (round 5): without a namespace program the
 * request-mapping kernel reads them itself (16 B per check instead of 28: the batch's only coalesced
 * stream of the first tier); with one they are unpacked on the device first.  Same answers, error
 * codes, streams and waiting as kg_check_batch_device; on a hash-sharded snapshot the call unpacks
 * into a buffer of its own and completes before it returns. */
int kg_check_batch_packed_device(kg_snapshot* s, const kg_query_packed* d_q, size_t n, int32_t global_max_depth,
                                 uint8_t* d_out, uint32_t* d_err, kg_stats* stats, void* stream);
/* kg_pack_query over device-resident queries (d_q[n] -> d_pk[n]) on `stream` (NULL: the snapshot's);
 * returns once done, -2 when an id does not fit. */
int kg_pack_queries_device(kg_snapshot* s, const kg_query* d_q, size_t n, kg_query_packed* d_pk, void* stream);
/* Device-side synthetic check batch for a synthetic snapshot: 50% positive (reverse walks) and
 * 50% uniform doc#viewer@user queries, max_depth in {0,1..10}.  d_q is a device buffer. */
int kg_synth_queries(kg_snapshot* s, uint64_t seed, size_t n, kg_query* d_q);

/* ---- request batcher -----------------------------------------------
 * Replaces one goroutine per Check RPC (internal/check/handler.go:248 -> CheckIsMember,
 * internal/check/engine.go:54-60) with one BLOCKING call per request: concurrent callers' queries
 * are coalesced into kg_check_batch batches (closed at max_batch queries or when the oldest has
 * waited max_wait_us) run by `dispatchers` threads, so consecutive batches overlap on the devices.
 * Each caller gets exactly its own answers (allowed = a loop of CheckIsMember). */
typedef struct kg_batcher kg_batcher;
typedef struct {
  uint64_t batches, checks;          /* since creation / the last reset                         */
  double batch_p50_ms, batch_p99_ms; /* oldest submission of a batch -> its answers delivered    */
  double call_p50_ms, call_p99_ms;   /* one kg_batcher_check call, submit -> return               */
} kg_batcher_stats_t;
int kg_batcher_create(kg_snapshot* s, int32_t global_max_depth, size_t max_batch, uint32_t max_wait_us,
                      int dispatchers, kg_batcher** out);
/* n queries of one caller (usually 1); out[n] / err_code[n] as in kg_check_batch.  Thread-safe. */
int kg_batcher_check(kg_batcher* b, const kg_query* q, size_t n, uint8_t* out, uint32_t* err_code);
int kg_batcher_stats(kg_batcher* b, kg_batcher_stats_t* st);
void kg_batcher_reset_stats(kg_batcher* b);
/* Answers what is pending, stops the dispatchers, frees the batcher (the snapshot stays). */
void kg_batcher_destroy(kg_batcher* b);

/* ---- hash-sharded mode --------------------------------------------------------
 * For graphs larger than one GPU: rank r of N holds the rows of the nodes (ns, obj, rel) with
 * kg_shard_owner(ns, obj, N) == r (all relations of an object on one rank).  A batch is a
 * level-synchronous BFS across ranks: every level each rank processes the frontier records it
 * received (nodes it owns, or hit / error reports for queries it is home of) and writes the next
 * level's records into one bucket per destination rank; the caller exchanges the buckets
 * (all-to-all, RCCL over xGMI) and calls kg_shard_level again until no rank sends anything, then
 * kg_shard_finish.  Replaces the single-GPU kg_check_batch for such snapshots.  Rewrites: union
 * rewrites are materialised into plain union nodes as in the single-GPU engine and boolean ones
 * over plain / union leaves are split into parts (kg_shard_result_slots); a query that reaches any
 * other rewrite (or an undeclared relation) ends here as KG_ERROR / KG_ERR_NOT_IMPLEMENTED, and the
 * driver's general phase answers it: the rows of every object within gdepth + 1 subject-set hops of
 * its root are gathered to its home rank (kg_snapshot_rows at each owner, all-to-all) and a
 * single-GPU snapshot of them (kg_snapshot_create + kg_check_batch: the rewrite interpreter) gives
 * the reference's answer and error.  keto_amd/sharded.py is the driver. */
typedef struct {
  uint32_t q;     /* home rank << 26 | index in the home rank's batch                         */
  uint32_t node;  /* node to check (checkIsAllowed(node, depth)), KG_FREC_HIT or KG_FREC_ERR  */
  uint32_t subj;  /* tagged subject: bit31 set = subject-set node id, else subject id;
                     the err code of a KG_FREC_ERR record                                     */
  int32_t depth;  /* rest depth (>= 1)                                                        */
} kg_frec;
#define KG_FREC_HIT 0xFFFFFFFFu /* kg_frec.node of a record reporting IsMember to the query's home */
#define KG_FREC_ERR 0xFFFFFFFEu /* kg_frec.node of a record reporting an error (code in subj)     */
#define KG_FREC_ESC 0xFFFFFFFDu /* kg_frec.node of a record handing the query to the backward phase */
#define KG_SHARD_MAX_RANKS 64

uint32_t kg_shard_owner(uint32_t ns, uint32_t obj, uint32_t nranks);
int kg_snapshot_create_shard(const kg_tuple* rows, size_t n, const kg_dict* dict, const kg_rewrite_prog* prog,
                             int device, uint32_t rank, uint32_t nranks, kg_snapshot** out);
int kg_snapshot_synthetic_shard(const kg_synth_params* params, const kg_rewrite_prog* prog, int device,
                                uint32_t rank, uint32_t nranks, kg_snapshot** out);
/* Device buffers: d_out = nranks buckets of `cap` records; d_counts[nranks + 1]: records written
 * per bucket (true counts: > cap means the bucket overflowed and the batch must be rerun with a
 * larger cap) and, in [nranks], overflow flags (1 bucket, 2 visited table).  kg_shard_seed zeroes
 * d_res (0 NotMember, 1 IsMember) / d_err and the counters; kg_shard_level zeroes the counters
 * before writing.  d_n_in: when non-NULL the level reads its record count from device memory
 * (n_in is then only an upper bound), so levels can be enqueued without a host round trip.
 * kg_shard_finish sets d_res[i] = KG_ERROR where d_err[i] != 0.  All of them only enqueue work
 * on `stream` (NULL = the snapshot's stream). */
int kg_shard_seed(kg_snapshot* s, const kg_query* d_q, size_t n, int32_t global_max_depth, kg_frec* d_out,
                  size_t cap, uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, void* stream);
int kg_shard_level(kg_snapshot* s, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out,
                   size_t cap, uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done,
                   uint32_t done_words, void* stream);
/* kg_shard_level over the receive buffer of a fixed-split all-to-all: segment k (k < n_seg) holds
 * d_seg_counts[k] records (device memory, clamped to seg_cap) at d_in + k * seg_cap.  With it a
 * multi-rank driver exchanges fixed-size buckets and never reads a count on the host inside a batch
 * (keto_amd/sharded.py: the level loop runs a fixed number of levels, overflow is checked once). */
int kg_shard_level_seg(kg_snapshot* s, const kg_frec* d_in, uint32_t n_seg, size_t seg_cap,
                       const uint32_t* d_seg_counts, kg_frec* d_out, size_t cap, uint32_t* d_counts, uint8_t* d_res,
                       uint32_t* d_err, const uint32_t* d_done, uint32_t done_words, void* stream);
/* Early exit across ranks: d_done (may be NULL) is the done bitmap of the batch, done_words words per
 * home rank ([rank][word], bit i = query i of that rank answered IsMember by the previous levels);
 * kg_shard_level drops the records of those queries.  kg_shard_done packs this rank's d_res into its
 * words (words >= ceil(n / 32)); with_escalated 1: queries escalated out of the forward phase count
 * as done too, 2: those escalated out of the backward phase; the driver all-gathers the words
 * before each level. */
/* One-rank snapshots (nranks 1): `levels` kg_shard_level calls enqueued back to back in ONE call,
 * ping-ponging between (d_buf0, d_counts0) and (d_buf1, d_counts1) from buffer `start` (0 / 1;
 * each buffer holds cap records, its record count in counts[0] on the device), with the done bitmap
 * of kg_shard_done (with_escalated as there) rebuilt before every level after the first.  *end
 * receives the buffer the last level wrote.  Replaces the driver's per-level loop when no exchange
 * happens between levels (keto_amd/sharded.py at world 1).  n_slots 0: no done bitmap (no query's
 * records are dropped once it is a member -- what a graph that can end a check in an error needs,
 * kg_shard_bad_nodes). */
int kg_shard_levels(kg_snapshot* s, int32_t levels, kg_frec* d_buf0, kg_frec* d_buf1, size_t cap, uint32_t* d_counts0,
                    uint32_t* d_counts1, int32_t start, uint8_t* d_res, uint32_t* d_err, size_t n_slots,
                    int32_t with_escalated, int32_t* end, void* stream);
int kg_shard_done(kg_snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, int with_escalated,
                  uint32_t* d_bits, uint32_t words, void* stream);
/* Backward phase (snapshots without a namespace program; kg_snapshot_tune "shard_budget", default
 * 0 = off).  A query whose forward records expand more than the budget of set edges on one
 * rank escalates: its forward walk stops (d_err carries a batch-internal marker until
 * kg_shard_finish) and, once no rank sends forward records, it is answered by a reverse search from
 * its subject's holders -- the single-GPU backward tier across ranks.  kg_shard_back_list writes
 * this rank's open escalated queries (q, root, subject, depth) into d_list, count in d_counts[0];
 * the driver all-gathers every rank's lists.  kg_shard_back_seed turns the global list (m entries,
 * or the count at d_m) into level-0 records: this rank's holders of each subject.
 * kg_shard_back_level processes a level's records -- ALL ranks' records, all-gathered: a node's
 * parents live in the rows of their owners, so every rank expands its own -- into one bucket
 * (d_counts[0]; d_counts[1] = overflow flags, accumulated), until no rank emits anything.  The done
 * bitmap of this phase is kg_shard_done without escalated queries. */
int kg_shard_back_list(kg_snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_list,
                       size_t cap, uint32_t* d_counts, void* stream);
int kg_shard_back_seed(kg_snapshot* s, const kg_frec* d_list, size_t m, const uint32_t* d_m, kg_frec* d_out,
                       size_t cap, uint32_t* d_counts, void* stream);
int kg_shard_back_level(kg_snapshot* s, const kg_frec* d_in, size_t n_in, const uint32_t* d_n_in, kg_frec* d_out,
                        size_t cap, uint32_t* d_counts, uint8_t* d_res, uint32_t* d_err, const uint32_t* d_done,
                        uint32_t done_words, void* stream);
/* The reverse search has its own budget (kg_snapshot_tune "shard_back_budget", reverse edges per
 * query and rank, default 2^14); a query past it is handed on once more (d_err marker; done bitmap
 * mode 2 of kg_shard_done during the backward phase) and kg_shard_refwd_seed re-seeds this rank's
 * such queries at their roots for a final forward phase: kg_shard_level without any budget until
 * the next kg_shard_seed (the single-GPU engine's stream -> backward -> grid tier chain). */
int kg_shard_refwd_seed(kg_snapshot* s, size_t n, const uint8_t* d_res, const uint32_t* d_err, kg_frec* d_out,
                        size_t cap, uint32_t* d_counts, void* stream);
/* The no-holder test across ranks (k_resolve's in the single-GPU engine): import 0 copies this
 * rank's holder bitmap (bit = a subject id some local row holds) into d_bits[words] (words >=
 * kg_shard_held_words); import 1 installs d_bits -- the OR over all ranks -- so kg_shard_seed
 * answers NotMember at once for a subject no rank holds (snapshots without a namespace program).
 * A single-rank snapshot uses its own bitmap without this. */
int kg_shard_held_words(const kg_snapshot* s, size_t* words);
int kg_shard_held(kg_snapshot* s, uint32_t* d_bits, size_t words, int import, void* stream);
int kg_shard_finish(kg_snapshot* s, size_t n, uint8_t* d_res, uint32_t* d_err, void* stream);
/* Result slots a batch of n queries needs in d_res / d_err (n, or more when the snapshot splits
 * boolean rewrites into parts: the parts' answers sit behind the n requested ones and
 * kg_shard_finish combines them into d_res[0, n) / d_err[0, n)). */
size_t kg_shard_result_slots(const kg_snapshot* s, size_t n);
/* Nodes a record can reach (a set edge of this rank's rows leads to them; an impure union counted by
 * its owner) that the level protocol cannot evaluate (a relation with a rewrite that is not
 * materialised, or undeclared): when no rank has any, no check can end in
 * an error below its root, and the driver may drop a member query's records (the done bitmap).
 * Otherwise it must not: the reference's order can make an error in an earlier branch win over a
 * member found at a shallower level in a later one (internal/check/checkgroup's first-decisive
 * rule); the walk then goes on, the error reaches the query's home and the general phase decides. */
int kg_shard_bad_nodes(const kg_snapshot* s, uint64_t* count);

/* ---- hash-sharded batches inside the library (round 4) --------------------------------------
 * The whole sharded batch -- seed, gdepth + 1 levels with their all-to-all exchanges, the done
 * bitmap, finish and the general phase -- runs inside kg_check_batch / kg_check_batch_device once a
 * transport is bound to the snapshot, so a host drives a sharded engine exactly like a replicated
 * one (internal/driver/registry_default.go:180-185 builds ONE check.Engine, engine.go:65-80): every
 * rank calls kg_check_batch(_device) with its own queries (any count, 0 included) in the same order
 * on the same stream, and gets its own answers back.  Per level: ONE grouped exchange of the
 * per-destination record counts and fixed-size buckets (B records each, the same B on every rank,
 * learned from the previous batch), one all-gather of the done bitmap, the level kernels; per
 * batch: one all-reduce that agrees on the slot count (the done bitmap's width) and one at the end
 * (overflow flags, largest bucket, records left, "a query needs the general phase") -- two host
 * round trips per batch, none per level.  A bucket or visited-table overflow on any rank reruns the
 * batch on every rank with room to spare.  Escalation (kg_snapshot_tune "shard_budget", round 5) runs
 * here too: a backward phase over all-gathered fixed buckets of the escalated queries and a final forward
 * phase for the queries past both budgets (keto_amd/sharded.py ShardedChecker is the restatement).
 *
 * kg_shard_comm_init binds an RCCL communicator (over xGMI on one node) to the batches the
 * snapshot runs on `stream` (NULL: the snapshot's own stream, which kg_check_batch uses); several
 * streams with a communicator each keep several batches in flight per rank.  All ranks call it
 * collectively with the id rank 0 got from kg_shard_unique_id (the host broadcasts the 128 bytes);
 * the snapshot must have been created for (rank, world) (kg_snapshot_create_shard / _synthetic_shard).
 * It also installs the OR of every rank's holder bitmap (kg_shard_held) and agrees whether any rank
 * can end a check in an error (kg_shard_bad_nodes).  Round 5: the first binding of a snapshot at
 * world > 1 also writes the OWNER's set-row length and row signature of every remote child into this
 * rank's adjacency records and node map (one max all-reduce of 8 B per node; kg_snapshot_tune
 * "shard_remote_meta" 0 skips it), so a remote child that can neither hit nor expand is never sent
 * and no per-edge owner lookup is made -- the same answers with fewer records (a transport's
 * allreduce_max_u64 must compare all 64 bits unsigned). */
#define KG_SHARD_UNIQUE_ID_BYTES 128
int kg_shard_unique_id(void* id);
int kg_shard_comm_init(kg_snapshot* s, const void* id, int rank, int world, void* stream);
/* Any other transport (MPI, a test harness) as callbacks, bound the same way.  Every call is
 * collective over the `world` ranks, in the same order on every rank.  host_memory 1: the library
 * hands the callbacks host buffers (it stages through pinned memory and completes its stream
 * first); 0: device buffers, the work enqueued on `stream`.
 *   alltoall2  fixed-size all-to-all of two buffers at once: block p (bytes0 / bytes1 bytes) of
 *              send0 / send1 goes to rank p, block q of recv0 / recv1 comes from rank q
 *   allgather  block r of recv (bytes each) = rank r's send
 *   allreduce_max_u64  element-wise max over ranks, in place
 * Each returns 0 on success. */
typedef struct {
  void* ctx;
  int32_t rank, world, host_memory;
  int (*alltoall2)(void* ctx, const void* send0, void* recv0, size_t bytes0, const void* send1, void* recv1,
                   size_t bytes1, void* stream);
  int (*allgather)(void* ctx, const void* send, void* recv, size_t bytes, void* stream);
  int (*allreduce_max_u64)(void* ctx, uint64_t* buf, size_t count, void* stream);
} kg_shard_transport;
int kg_shard_transport_attach(kg_snapshot* s, const kg_shard_transport* t, void* stream);
/* Unbinds (and for RCCL destroys) the communicator of `stream`; kg_snapshot_destroy does it for all. */
int kg_shard_comm_release(kg_snapshot* s, void* stream);
/* Round 5.  Local-first: a one-rank binding (world 1) runs a batch through the replica engine's tier
 * chain -- every row is that rank's, so no record would leave it (kg_snapshot_tune "shard_local" 0:
 * the one-rank device level loop instead).  kg_snapshot_tune "shard_force_exchange" 1 makes a
 * one-rank binding run the N > 1 exchange protocol over its transport (RCCL: self send / recv,
 * all-gather and all-reduce over one rank), so the transport code an N-GPU run uses can run, and be
 * tested, on one GPU.  The exchange protocol sizes the buckets of each exchange k (k = 0 .. gdepth)
 * separately, from what exchange k needed in the previous batch.  Overflow reruns are bounded
 * ("shard_max_reruns", default 4) and so are the bucket buffers ("shard_max_bytes", default a quarter
 * of the free HBM): past either, every rank returns KG_ERR_RESOURCE (-4) together, with the reason in
 * kg_last_error.  A rank that cannot run its batch (too large, out of memory) says so in the batch's
 * first all-reduce and every rank returns an error; any other failure inside the protocol (a transport
 * error, a failed kernel launch) leaves the binding unusable: release it (kg_shard_comm_release) and
 * bind a new one on every rank. */
/* Counters of the last batch on `stream`: [0] levels, [1] records sent, [2] host round trips,
 * [3] reruns after a bucket overflow, [4] after a visited-table overflow, [5] queries answered by
 * the general phase, [6] rows it gathered, [7] bucket size B (the largest B_k).
 * kg_shard_comm_stats_ex gives up to 16: [8] records this rank sent to OTHER ranks (what crosses
 * xGMI), [9] bytes it put on the wire (every other rank gets B_k records per exchange, plus counts
 * and done bitmaps), [10] path (0 local-first tier chain, 1 one-rank device loop, 2 exchange
 * protocol), [11] exchanges the last batch ran (learned: the previous batch's last non-empty exchange
 * + 2, at most gdepth + 1), [12] levels of the escalation phases (backward + final forward), [13] 1 when
 * the last batch had records left after the learned exchanges and reran with all of them. */
int kg_shard_comm_stats(const kg_snapshot* s, void* stream, uint64_t out8[8]);
int kg_shard_comm_stats_ex(const kg_snapshot* s, void* stream, uint64_t* out, size_t n);
/* Per exchange k of the last batch: out[2k] = B_k (records per destination it was sent with),
 * out[2k + 1] = its largest bucket (records).  Returns the number of exchanges (0 without one). */
int64_t kg_shard_comm_levels(const kg_snapshot* s, void* stream, uint64_t* out, size_t cap);

/* ---- check trees ----------------------------------------------------------------------------
 * CheckRelationTuple's Result.Tree (internal/check/engine.go:65-80, checkgroup/definitions.go:46-50,
 * 101-124): for a member, the tree of the branch that answered -- direct tuples, then subject-set rows
 * in row order, then the rewrite (the reference runs them concurrently; its asserted paths are
 * rewrites_test.go:186-205).  Every membership the walk relies on comes from kg_check_batch on this
 * snapshot (batched per row of candidates) and every row from the snapshot's row reads.  *result /
 * *err_code: the check's answer; the tree (pre-order kg_check_node records, n_children each) only for
 * KG_IS_MEMBER.  hidden_rels: relations a compiler introduced for tuple-to-subject-set leaves of
 * boolean rewrites (keto_amd/namespace.py lower_ttu_leaves) -- their computed edge is inlined, as the
 * reference's tree has the TTU edge there.  cap too small: returns -3 with *n_nodes = records needed.
 * Not on hash-sharded snapshots.  Not a hot path. */
#define KG_CTREE_LEAF 1
#define KG_CTREE_UNION 2
#define KG_CTREE_INTERSECTION 3 /* an `and`: has_tuple 0 (binop.go:47-50 builds it without one) */
#define KG_CTREE_COMPUTED 4
#define KG_CTREE_TTU 5
#define KG_CTREE_NOT 6
typedef struct {
  uint8_t type;      /* KG_CTREE_* */
  uint8_t has_tuple; /* 0: no tuple (an `and` node) */
  uint16_t pad;
  uint32_t n_children;
  kg_tuple t;        /* the node's tuple (its request tuple) */
} kg_check_node;
int kg_check_tree(kg_snapshot* s, const kg_query* q, int32_t global_max_depth, const uint32_t* hidden_rels,
                  size_t n_hidden, kg_check_node* out, size_t cap, size_t* n_nodes, uint8_t* result,
                  uint32_t* err_code);

/* ---- expand ----------------------------------------------------------------------------- */
/* Roots are split over the replicas (chunks of >= 1024 roots, one host thread each).  On a
 * hash-sharded snapshot with a transport bound to its own stream (kg_shard_comm_init(.., NULL)) the
 * call is collective like kg_check_batch: every rank passes its own roots (any count) and the rows
 * those roots can reach are gathered to it first (the general phase's region gather), then expanded
 * there -- the same trees as an unsharded snapshot. */
int kg_expand_batch(kg_snapshot* s, const kg_set* roots, size_t n, int32_t global_max_depth, kg_tree_buf* out);
/* kg_expand_batch with the roots and the trees in HBM (round 6; the expand analogue of
 * kg_check_batch_device, expand/engine.go:35-104 per root): d_roots[n] on the snapshot's device, work on
 * `stream` (NULL: the snapshot's).  out->nodes and out->root_off (n + 1 entries) are DEVICE pointers
 * (out->pinned = 0x100 | device), valid until kg_tree_free; the call returns with them complete.
 * Single GPU (an unsharded snapshot). */
int kg_expand_batch_device(kg_snapshot* s, const kg_set* d_roots, size_t n, int32_t global_max_depth, kg_tree_buf* out,
                           void* stream);
void kg_tree_free(kg_tree_buf* t);

/* ---- errors ----------------------------------------------------------------------------- */
/* Thread-local text of the last failing call; returns its length. */
size_t kg_last_error(char* buf, size_t len);
const char* kg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KETOGPU_H */
