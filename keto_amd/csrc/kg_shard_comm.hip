// kg_shard_comm.hip -- hash-sharded batches inside the library.
//
// kg_check_batch / kg_check_batch_device on a snapshot with a transport bound to the call's stream
// run the whole sharded batch here, so a host drives the sharded engine through the same entry
// point as the replicated one (the reference wires ONE check.Engine into the registry,
// internal/driver/registry_default.go:180-185, internal/check/engine.go:65-80):
//
//   agree    all-reduce of this rank's result-slot count (the done bitmap's width)  host round trip 1
//   seed     kg_shard_seed: this rank's queries -> one record each at its root's owner
//   level k  (k = 0 .. gdepth; a record's rest depth falls by one per level, the last level only
//            delivers hit / error reports) ONE grouped exchange of the per-destination counts and
//            the fixed-size buckets (B records per destination, the same B on every rank), the
//            done bitmap all-gathered when pruning is on, kg_shard_level over the N received
//            segments (their counts read on the device)
//   end      kg_shard_finish, then one all-reduce of (bucket overflow, visited overflow, largest
//            bucket, records left, a query needs the general phase)           host round trip 2
//   rerun    on an overflow anywhere: every rank reruns with bigger buckets / a bigger table
//   general  queries that reached a rewrite the level protocol cannot evaluate across ranks: the rows
//            of every object within gdepth + 1 subject-set hops of their roots are gathered to their
//            home rank (each owner ships an object's rows once per home) and a single-GPU snapshot of
//            them answers them with the rewrite interpreter -- the reference's answers and errors
//
// This is keto_amd/sharded.py's fixed-bucket protocol (ShardedChecker._check_fixed, _general_phase,
// still the CPU-tested restatement) moved below the C ABI.  The transport is RCCL over xGMI
// (kg_shard_comm_init) or any host callbacks (kg_shard_transport_attach).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <set>
#include <vector>

#include "kg_internal.h"
#include "kg_snapshot.h"

namespace kg {

struct ShardComm {
  hipStream_t bound = nullptr;  // as bound by the caller (NULL: the snapshot's stream)
  hipStream_t run = nullptr;    // the stream the batches run on
  int device = -1;
  int rank = 0, world = 1;
  kg_shard_transport t{};
  ncclComm_t nccl = nullptr;
  std::mutex mu;
  bool prune = false;
  // device buffers, grown on demand
  kg_frec* buf[2] = {nullptr, nullptr};
  kg_frec* recv = nullptr;
  size_t recs = 0;                  // records each of buf[0], buf[1], recv holds (N * B)
  uint32_t* cnt = nullptr;          // counts[2][N + 1] | rc[N]
  unsigned long long* acc = nullptr;  // acc[4] | tot[8] | scratch[8]
  uint32_t* bits = nullptr;
  uint32_t* bits_all = nullptr;
  size_t words_cap = 0, all_cap = 0;
  uint8_t* res = nullptr;
  uint32_t* err = nullptr;
  size_t slots_cap = 0;
  kg_query* dq = nullptr;  // kg_check_batch (host buffers): staged queries and results
  uint8_t* dout = nullptr;
  uint32_t* derr = nullptr;
  size_t dq_cap = 0;
  void* pinned = nullptr;  // host staging: host-memory transports and readbacks
  size_t pinned_bytes = 0;
  size_t bucket = 0;     // one rank's device loop: B, learned from the previous batch
  // the exchange protocol: B_k records per destination for exchange k (k = 0 .. gdepth; the seed
  // writes exchange 0's buckets, level k - 1 exchange k's), each learned from the largest bucket
  // exchange k needed in the previous batch -- levels differ by orders of magnitude, and every
  // destination of exchange k gets B_k records on the wire whatever it holds
  std::vector<size_t> lb;
  size_t bb = 0;  // escalation: records per rank of a backward-phase all-gather, learned like B_k
  unsigned long long* red = nullptr;  // [8 + levels]: the end-of-batch all-reduce (tot[5] | per-exchange largest)
  size_t red_cap = 0;
  std::vector<uint64_t> lvl_last, lb_last;  // the last batch: per exchange its largest bucket and B_k
  // exchanges a batch runs (round 6): learned from the last batch -- its last
  // non-empty exchange + 2 -- instead of always gdepth + 1 (the trailing ones carried nothing and cost
  // ~37 us each); a batch that still has records after them reruns with all of them (0: not learned yet)
  int lx = 0;
  std::mutex host_mu;    // kg_check_batch (host buffers): one batch at a time through dq / dout / derr
  uint64_t st[16] = {};  // kg_shard_comm_stats (kg_shard_comm_stats_ex: all 16)
  hipEvent_t ev[2] = {nullptr, nullptr};
  void* xbufs = nullptr;  // one rank's local-first expand: device buffers kept across calls (under mu)
  ~ShardComm();
};

ShardComm::~ShardComm() {
  if (device >= 0) hipSetDevice(device);
  if (run) hipStreamSynchronize(run);
  if (nccl) ncclCommDestroy(nccl);
  if (xbufs) expand_bufs_free(xbufs);
  hipFree(buf[0]);
  hipFree(buf[1]);
  hipFree(recv);
  hipFree(cnt);
  hipFree(acc);
  hipFree(red);
  hipFree(bits);
  hipFree(bits_all);
  hipFree(res);
  hipFree(err);
  hipFree(dq);
  hipFree(dout);
  hipFree(derr);
  if (pinned) hipHostFree(pinned);
  for (auto e : ev)
    if (e) hipEventDestroy(e);
}

void shard_comms_free(Snapshot* s) {
  std::vector<std::shared_ptr<ShardComm>> v;
  {
    std::lock_guard<std::mutex> lk(s->comm_mu);
    v.swap(s->comms);
    s->n_comms.store(0, std::memory_order_release);
  }
  v.clear();  // each binding is destroyed when its last caller lets go of it
}

// The binding of stream st (shared: kg_shard_comm_release or a re-bind on st only drops the list's
// reference, and a caller inside a batch keeps the object alive until it returns).  Snapshots with
// nothing bound -- the replicated path -- take no lock.
std::shared_ptr<ShardComm> shard_comm_of(Snapshot* s, hipStream_t st) {
  if (s->n_comms.load(std::memory_order_acquire) == 0) return nullptr;
  std::lock_guard<std::mutex> lk(s->comm_mu);
  for (const auto& c : s->comms)
    if (c->bound == st) return c;
  return nullptr;
}

// ------------------------------------------------------------------ RCCL transport
#define NCCLC(expr)                                                                                            \
  do {                                                                                                         \
    ncclResult_t _r = (expr);                                                                                  \
    if (_r != ncclSuccess) return set_error(-1, "%s: %s", #expr, ncclGetErrorString(_r));                    \
  } while (0)

static int rccl_alltoall2(void* ctx, const void* s0, void* r0, size_t b0, const void* s1, void* r1, size_t b1,
                          void* stream) {
  ShardComm* c = static_cast<ShardComm*>(ctx);
  hipStream_t st = (hipStream_t)stream;
  NCCLC(ncclGroupStart());
  for (int p = 0; p < c->world; p++) {
    if (b0) {
      NCCLC(ncclSend((const char*)s0 + p * b0, b0 / 4, ncclUint32, p, c->nccl, st));
      NCCLC(ncclRecv((char*)r0 + p * b0, b0 / 4, ncclUint32, p, c->nccl, st));
    }
    if (b1) {
      NCCLC(ncclSend((const char*)s1 + p * b1, b1 / 4, ncclUint32, p, c->nccl, st));
      NCCLC(ncclRecv((char*)r1 + p * b1, b1 / 4, ncclUint32, p, c->nccl, st));
    }
  }
  NCCLC(ncclGroupEnd());
  return 0;
}

static int rccl_allgather(void* ctx, const void* s, void* r, size_t bytes, void* stream) {
  ShardComm* c = static_cast<ShardComm*>(ctx);
  NCCLC(ncclAllGather(s, r, bytes / 4, ncclUint32, c->nccl, (hipStream_t)stream));
  return 0;
}

static int rccl_allreduce_max(void* ctx, uint64_t* buf, size_t count, void* stream) {
  ShardComm* c = static_cast<ShardComm*>(ctx);
  NCCLC(ncclAllReduce(buf, buf, count, ncclUint64, ncclMax, c->nccl, (hipStream_t)stream));
  return 0;
}

// ------------------------------------------------------------------ transport calls, staged as needed
static void* pinned_at_least(ShardComm* c, size_t bytes) {
  if (bytes > c->pinned_bytes) {
    if (c->pinned) hipHostFree(c->pinned);
    c->pinned = nullptr;
    c->pinned_bytes = 0;
    const size_t b = std::max<size_t>(bytes, 1 << 16);
    if (hipHostMalloc(&c->pinned, b) != hipSuccess) return nullptr;
    c->pinned_bytes = b;
  }
  return c->pinned;
}

static int tcall(int rc, const char* what) {
  return rc ? set_error(-1, "sharded transport: %s failed (%d)", what, rc) : 0;
}

// device buffers in, device buffers out (enqueued on c->run, or staged and completed)
static int x_alltoall2(ShardComm* c, const void* s0, void* r0, size_t b0, const void* s1, void* r1, size_t b1) {
  if (!c->t.host_memory) return tcall(c->t.alltoall2(c->t.ctx, s0, r0, b0, s1, r1, b1, c->run), "alltoall2");
  const size_t N = (size_t)c->world, a = N * b0, b = N * b1;
  char* h = (char*)pinned_at_least(c, 2 * (a + b));
  if (!h) return set_error(-1, "pinned staging");
  HIPC(hipStreamSynchronize(c->run));  // earlier H2D copies out of the staging area are done
  if (a) HIPC(hipMemcpyAsync(h, s0, a, hipMemcpyDeviceToHost, c->run));
  if (b) HIPC(hipMemcpyAsync(h + a, s1, b, hipMemcpyDeviceToHost, c->run));
  HIPC(hipStreamSynchronize(c->run));
  if (int rc = tcall(c->t.alltoall2(c->t.ctx, h, h + a + b, b0, h + a, h + 2 * a + b, b1, nullptr), "alltoall2"))
    return rc;
  if (a) HIPC(hipMemcpyAsync(r0, h + a + b, a, hipMemcpyHostToDevice, c->run));
  if (b) HIPC(hipMemcpyAsync(r1, h + 2 * a + b, b, hipMemcpyHostToDevice, c->run));
  return 0;
}

static int x_allgather(ShardComm* c, const void* s, void* r, size_t bytes) {
  if (!c->t.host_memory) return tcall(c->t.allgather(c->t.ctx, s, r, bytes, c->run), "allgather");
  const size_t N = (size_t)c->world;
  char* h = (char*)pinned_at_least(c, (N + 1) * bytes);
  if (!h) return set_error(-1, "pinned staging");
  HIPC(hipStreamSynchronize(c->run));
  HIPC(hipMemcpyAsync(h, s, bytes, hipMemcpyDeviceToHost, c->run));
  HIPC(hipStreamSynchronize(c->run));
  if (int rc = tcall(c->t.allgather(c->t.ctx, h, h + bytes, bytes, nullptr), "allgather")) return rc;
  HIPC(hipMemcpyAsync(r, h + bytes, N * bytes, hipMemcpyHostToDevice, c->run));
  return 0;
}

static int x_allreduce_max(ShardComm* c, unsigned long long* d, size_t count) {
  if (!c->t.host_memory) return tcall(c->t.allreduce_max_u64(c->t.ctx, (uint64_t*)d, count, c->run), "allreduce");
  uint64_t* h = (uint64_t*)pinned_at_least(c, count * 8);
  if (!h) return set_error(-1, "pinned staging");
  HIPC(hipStreamSynchronize(c->run));
  HIPC(hipMemcpyAsync(h, d, count * 8, hipMemcpyDeviceToHost, c->run));
  HIPC(hipStreamSynchronize(c->run));
  if (int rc = tcall(c->t.allreduce_max_u64(c->t.ctx, h, count, nullptr), "allreduce")) return rc;
  HIPC(hipMemcpyAsync(d, h, count * 8, hipMemcpyHostToDevice, c->run));
  return 0;
}

// host buffers in and out, completed on return (agreement, the general phase)
static int h_allreduce_max(ShardComm* c, uint64_t* v, size_t count) {
  if (count > 8) return set_error(-2, "h_allreduce_max: at most 8 values");
  unsigned long long* d = c->acc + 12;
  HIPC(hipMemcpyAsync(d, v, count * 8, hipMemcpyHostToDevice, c->run));
  if (int rc = x_allreduce_max(c, d, count)) return rc;
  HIPC(hipMemcpyAsync(v, d, count * 8, hipMemcpyDeviceToHost, c->run));
  HIPC(hipStreamSynchronize(c->run));
  return 0;
}

static int h_alltoall2(ShardComm* c, const void* s0, void* r0, size_t b0, const void* s1, void* r1, size_t b1) {
  if (c->t.host_memory) {
    HIPC(hipStreamSynchronize(c->run));
    return tcall(c->t.alltoall2(c->t.ctx, s0, r0, b0, s1, r1, b1, nullptr), "alltoall2");
  }
  const size_t N = (size_t)c->world, a = N * b0, b = N * b1;
  char* d = nullptr;
  HIPC(hipMalloc(&d, 2 * (a + b) + 16));
  int rc = 0;
  if (a) rc |= hipMemcpyAsync(d, s0, a, hipMemcpyHostToDevice, c->run) != hipSuccess;
  if (b) rc |= hipMemcpyAsync(d + a, s1, b, hipMemcpyHostToDevice, c->run) != hipSuccess;
  if (!rc) rc = x_alltoall2(c, d, d + a + b, b0, d + a, d + 2 * a + b, b1);
  else rc = set_error(-1, "H2D staging");
  if (!rc && a && hipMemcpyAsync(r0, d + a + b, a, hipMemcpyDeviceToHost, c->run) != hipSuccess) rc = -1;
  if (!rc && b && hipMemcpyAsync(r1, d + 2 * a + b, b, hipMemcpyDeviceToHost, c->run) != hipSuccess) rc = -1;
  if (hipStreamSynchronize(c->run) != hipSuccess && !rc) rc = set_error(-1, "D2H staging");
  hipFree(d);
  return rc;
}

// ------------------------------------------------------------------ small kernels
// acc words (32, cleared per run): [0] flags, [1] largest bucket, [2] records sent, [3] records to other
// ranks, [4..11] tot of the one-rank loop, [12..19] host all-reduce scratch, then:
constexpr int ACC_LEFT = 20;  // records left at the end of the phases before the last
constexpr int ACC_BACK = 21;  // largest backward-phase bucket
// Per exchange k before it runs (kg_shard.hip k_shard_pre; keto_amd/sharded.py _check_fixed's device
// accumulators): acc[0] |= overflow flags (c[N], or a bucket past B_k), acc[1] = largest bucket,
// acc[2] += records sent, acc[3] += records sent to other ranks (what crosses xGMI), *lvl = exchange
// k's largest bucket (the counters keep counting past B_k, so an overflowed bucket reports what it
// would have needed).
// After the last level: tot = (bucket overflow, visited overflow, largest bucket, records left, 0).
__global__ void k_sc_final(const uint32_t* __restrict__ c, uint32_t N, uint32_t B, unsigned long long* acc,
                           unsigned long long* tot) {
  const uint32_t i = threadIdx.x;
  const uint32_t v = i < N ? c[i] : 0u;
  unsigned long long fl = (i < N && v > B) ? 1ull : 0ull, sum = v;
  for (int off = 32; off; off >>= 1) {
    fl |= __shfl_xor(fl, off, 64);
    sum += __shfl_xor(sum, off, 64);
  }
  if (i == 0) {
    const unsigned long long f = acc[0] | fl | c[N];
    tot[0] = f & 1ull;
    tot[1] = (f >> 1) & 1ull;
    tot[2] = acc[1];
    tot[3] = sum + acc[ACC_LEFT];
    tot[4] = 0;
    tot[5] = acc[ACC_BACK];
  }
}

// End of a forward phase that another phase follows (escalation): its flags and the records it left
// (none, in a clean run) go to the accumulators k_sc_final reads.
__global__ void k_sc_phase_end(const uint32_t* __restrict__ c, uint32_t N, uint32_t B, unsigned long long* acc) {
  const uint32_t i = threadIdx.x;
  const uint32_t v = i < N ? c[i] : 0u;
  unsigned long long fl = (i < N && v > B) ? 1ull : 0ull, sum = v;
  for (int off = 32; off; off >>= 1) {
    fl |= __shfl_xor(fl, off, 64);
    sum += __shfl_xor(sum, off, 64);
  }
  if (i == 0) {
    acc[0] |= fl | c[N];
    acc[ACC_LEFT] += sum;
  }
}

// The one-rank device loop's version: counts (left, flags) of its two buffers, `cur` the last one.
__global__ void k_sc_loop_end(const uint32_t* __restrict__ c0, const uint32_t* __restrict__ c1, int cur,
                              unsigned long long* acc) {
  if (threadIdx.x == 0) {
    acc[0] |= c0[1] | c1[1];
    acc[ACC_LEFT] += cur ? c1[0] : c0[0];
  }
}

// A backward-phase bucket (count, flags): its overflow and its size (the largest one sizes the next
// batch's backward buckets); with `left`, the records it holds are records left (the phase's last).
__global__ void k_sc_back(const uint32_t* __restrict__ cb, uint32_t B, int left, unsigned long long* acc) {
  if (threadIdx.x == 0) {
    acc[0] |= cb[1] | (cb[0] > B ? 1u : 0u);
    acc[ACC_BACK] = max(acc[ACC_BACK], (unsigned long long)cb[0]);
    if (left) acc[ACC_LEFT] += cb[0];
  }
}

// One rank (kg_shard_levels' device loop): tot = (bucket overflow, visited overflow, -, records left, 0)
// from the flags words of both buffers and the count of the last one; tot[2] = the bucket size the
// levels needed, written by kg_shard_levels' fold.
__global__ void k_sc_final1(const uint32_t* __restrict__ c0, const uint32_t* __restrict__ c1, int end,
                            const unsigned long long* acc, unsigned long long* tot) {
  if (threadIdx.x == 0) {
    const unsigned long long f = c0[1] | c1[1] | acc[0];
    tot[0] = f & 1u;
    tot[1] = (f >> 1) & 1u;
    tot[3] = (end ? c1[0] : c0[0]) + acc[ACC_LEFT];
    tot[4] = 0;
    tot[5] = acc[ACC_BACK];
  }
}

// 1 + the largest relation id of any node (the general phase's region gather asks owners for every
// relation of an object, so every relation a row can carry must be named).
__global__ void k_sc_rel_span(const uint32_t* __restrict__ nd_rel, uint64_t n, unsigned int* out) {
  uint32_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    m = max(m, nd_rel[i] + 1u);
  for (int off = 32; off; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

// tot[4] = 1 when some query of [0, n) ended KG_ERROR / KG_ERR_NOT_IMPLEMENTED (general phase).
__global__ void k_sc_open(uint32_t n, const uint8_t* __restrict__ res, const uint32_t* __restrict__ err,
                          unsigned long long* tot) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool open = i < n && res[i] == KG_ERROR && err[i] == KG_ERR_NOT_IMPLEMENTED;
  if (__ballot(open) && (threadIdx.x & 63) == 0) tot[4] = 1ull;
}

// out[w] = OR over ranks of parts[r * words + w] (the holder bitmaps of every rank).
__global__ void k_sc_or(const uint32_t* __restrict__ parts, uint32_t N, uint64_t words, uint32_t* out) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= words) return;
  uint32_t v = 0;
  for (uint32_t r = 0; r < N; r++) v |= parts[r * words + w];
  out[w] = v;
}

// ------------------------------------------------------------------ binding
static int grow(void** p, size_t* have, size_t want, size_t unit) {
  if (want <= *have && *p) return 0;
  if (*p) hipFree(*p);
  *p = nullptr;
  *have = 0;
  const size_t n = std::max<size_t>(want, 1024);
  HIPC(hipMalloc(p, n * unit));
  *have = n;
  return 0;
}

// Collective, once per binding: the OR of every rank's holder bitmap (kg_shard_seed's no-holder test
// across ranks) and whether any rank can end a check in an error (pruning through the done bitmap).
static int comm_setup(Snapshot* s, ShardComm* c) {
  HIPC(hipMalloc((void**)&c->acc, 32 * 8));
  HIPC(hipMemsetAsync(c->acc, 0, 32 * 8, c->run));
  HIPC(hipMalloc((void**)&c->cnt, (4 * (size_t)KG_SHARD_MAX_RANKS + 8) * 4));
  uint64_t bad = 0;
  if (int rc = shard_bad_nodes(s, &bad)) return rc;
  size_t words = 0;
  if (c->world > 1) words = ((size_t)s->ds.hbits_n + 31) / 32;
  // remote child metadata (DevSnap::remote_meta) runs when every rank wants it (not yet done, knob on)
  // and every rank has the same node id space (node ids are global: kg_snapshot.hip create_from_tuples)
  const uint64_t nn = s->ds.n_nodes;
  uint64_t* dmeta = nullptr;  // allocated before the agreement: a rank without it makes every rank skip
  if (c->world > 1 && !s->ds.remote_meta && s->shard_remote_meta && nn &&
      hipMalloc((void**)&dmeta, nn * 8) != hipSuccess) {
    (void)hipGetLastError();
    dmeta = nullptr;
  }
  // a host-memory transport stages the all-reduce through pinned memory: taken now, so a rank that
  // cannot have it makes every rank skip instead of failing alone inside the collective below
  if (dmeta && c->t.host_memory && !pinned_at_least(c, nn * 8)) {
    hipFree(dmeta);
    dmeta = nullptr;
  }
  const uint64_t skip = dmeta ? 0 : 1;
  uint64_t v[4] = {bad, words, nn, 0xFFFFFFFFull - nn};
  v[3] |= skip << 40;
  if (int rc = h_allreduce_max(c, v, 4)) {
    hipFree(dmeta);
    return rc;
  }
  c->prune = v[0] == 0;
  words = (size_t)v[1];
  const bool meta = !(v[3] >> 40) && v[2] == 0xFFFFFFFFull - (v[3] & 0xFFFFFFFFull);
  if (!meta) {
    hipFree(dmeta);
    dmeta = nullptr;
  }
  if (c->world > 1 && words) {
    uint32_t *mine = nullptr, *all = nullptr;
    HIPC(hipMalloc((void**)&mine, words * 4));
    HIPC(hipMalloc((void**)&all, (size_t)c->world * words * 4));
    int rc = shard_held(s, mine, words, 0, c->run);
    if (!rc) rc = x_allgather(c, mine, all, words * 4);
    if (!rc) {
      hipLaunchKernelGGL(k_sc_or, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0, c->run, all, (uint32_t)c->world,
                         (uint64_t)words, mine);
      rc = shard_held(s, mine, words, 1, c->run);  // synchronises
    }
    hipFree(mine);
    hipFree(all);
    if (rc) {
      hipFree(dmeta);
      return rc;
    }
  }
  if (dmeta) {
    // one max all-reduce of 8 B per node: each node's (row length, signature) word is non-zero on its
    // owner only.  Every rank reaches both collectives whatever its own step did: a rank whose local
    // step failed contributes zeros and a failure flag, and the second all-reduce makes every rank skip
    // the metadata together (the nowner path: more records, the same answers).  Only a failed
    // collective (the transport itself) or a failed apply on this rank fails the bind.
    uint64_t* d = dmeta;
    const int lrc = shard_meta_local(s, d, c->run);
    if (lrc && hipMemsetAsync(d, 0, nn * 8, c->run) != hipSuccess) (void)hipGetLastError();
    int rc = x_allreduce_max(c, reinterpret_cast<unsigned long long*>(d), nn);
    uint64_t failed = lrc != 0;
    if (!rc) rc = h_allreduce_max(c, &failed, 1);
    if (!rc && !failed) rc = shard_meta_apply(s, d, c->run);  // synchronises
    else (void)hipStreamSynchronize(c->run);
    hipFree(d);
    if (rc) return rc;
  }
  return 0;
}

// Takes ownership of c (freed on failure).
static int bind(Snapshot* s, ShardComm* c, hipStream_t st) {
  std::shared_ptr<ShardComm> sp(c);
  if ((uint32_t)c->world != s->shard_n || (uint32_t)c->rank != s->shard_rank)
    return set_error(-2, "transport is rank %d of %d, the snapshot was built as shard %u of %u", c->rank, c->world,
                     s->shard_rank, s->shard_n);
  c->bound = st;
  c->run = st ? st : s->stream;
  c->bucket = s->shard_bucket0;
  c->device = s->device;
  if (int rc = comm_setup(s, c)) return rc;
  std::shared_ptr<ShardComm> old;  // a previous binding of st: destroyed outside the lock, once unused
  std::lock_guard<std::mutex> lk(s->comm_mu);
  for (auto it = s->comms.begin(); it != s->comms.end(); ++it)
    if ((*it)->bound == st) {
      old = *it;
      s->comms.erase(it);
      break;
    }
  s->comms.push_back(sp);
  s->n_comms.store((int)s->comms.size(), std::memory_order_release);
  return 0;
}

// ------------------------------------------------------------------ the general phase
// s->rel_span (1 + the largest relation id of any node; collective callers all compute their own)
static int rel_span(Snapshot* s, hipStream_t st) {
  if (s->rel_span || !s->ds.n_nodes) return 0;
  unsigned int* d = nullptr;
  HIPC(hipMalloc((void**)&d, 4));
  unsigned int h = 0;
  int rc = hipMemsetAsync(d, 0, 4, st) != hipSuccess;
  if (!rc) {
    const uint64_t nn = s->ds.n_nodes;
    hipLaunchKernelGGL(k_sc_rel_span, dim3((uint32_t)std::min<uint64_t>((nn + 255) / 256, 4096)), dim3(256), 0, st,
                       s->ds.nd_rel, nn, d);
    rc = hipGetLastError() != hipSuccess || hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
         hipStreamSynchronize(st) != hipSuccess;
  }
  hipFree(d);
  if (rc) return set_error(-1, "relation span of the snapshot's nodes");
  s->rel_span = std::max(h, 1u);
  return 0;
}

template <int W>
using Row = std::array<uint64_t, W>;

// All-to-all of host rows: rows[i] goes to rank dest[i]; returns what this rank received (collective).
template <int W>
static int a2a_rows(ShardComm* c, const std::vector<Row<W>>& rows, const std::vector<int>& dest,
                    std::vector<Row<W>>* out) {
  const size_t N = (size_t)c->world;
  out->clear();
  std::vector<uint64_t> cnt(N, 0);
  for (int d : dest) cnt[(size_t)d]++;
  uint64_t m = 0;
  for (uint64_t x : cnt) m = std::max(m, x);
  if (int rc = h_allreduce_max(c, &m, 1)) return rc;
  if (m == 0) return 0;
  std::vector<uint64_t> send(N * m * W, 0), recv(N * m * W, 0), rcnt(N, 0);
  std::vector<uint64_t> fill(N, 0);
  for (size_t i = 0; i < rows.size(); i++) {
    const size_t d = (size_t)dest[i];
    std::memcpy(&send[(d * m + fill[d]++) * W], rows[i].data(), W * 8);
  }
  if (int rc = h_alltoall2(c, cnt.data(), rcnt.data(), 8, send.data(), recv.data(), m * W * 8)) return rc;
  for (size_t q = 0; q < N; q++)
    for (uint64_t j = 0; j < rcnt[q] && j < m; j++) {
      Row<W> r;
      std::memcpy(r.data(), &recv[(q * m + j) * W], W * 8);
      out->push_back(r);
    }
  return 0;
}

// Every row of every object within gdepth + 1 subject-set hops of the open queries' root objects,
// gathered at their home rank (keto_amd/sharded.py _gather_region: expand rows and tuple-to-subject-set
// rows both lead through subject sets; computed subject sets stay on the object, all of whose
// relations live on its owner).  Collective: every rank takes part, with or without open queries.
static int gather_region(Snapshot* s, ShardComm* c, const std::vector<std::pair<uint32_t, uint32_t>>& starts,
                         int32_t gdepth, std::vector<kg_tuple>* region) {
  const uint32_t N = (uint32_t)c->world;
  std::set<Row<3>> reqset;
  for (const auto& o : starts) reqset.insert(Row<3>{(uint64_t)c->rank, o.first, o.second});
  std::vector<Row<3>> req(reqset.begin(), reqset.end());
  std::set<Row<3>> seen;  // (home, ns, obj) this owner has shipped
  // every relation a row can carry: the program's / dict's relation count does not bound the ids a
  // snapshot built without a dict (or with undeclared relations) stores
  if (int rc = rel_span(s, c->run)) return rc;
  const uint32_t nrel = std::max<uint32_t>(std::max<uint32_t>(s->ds.n_rel, s->rel_span), 1);
  for (int hop = 0; hop < gdepth + 2; hop++) {
    std::vector<int> dest(req.size());
    for (size_t i = 0; i < req.size(); i++) dest[i] = (int)shard_owner((uint32_t)req[i][1], (uint32_t)req[i][2], N);
    std::vector<Row<3>> got;
    if (int rc = a2a_rows<3>(c, req, dest, &got)) return rc;
    std::vector<Row<3>> fresh;
    for (const Row<3>& r : got)
      if (seen.insert(r).second) fresh.push_back(r);
    std::vector<kg_set> keys(fresh.size() * nrel);
    for (size_t i = 0; i < fresh.size(); i++)
      for (uint32_t r = 0; r < nrel; r++) keys[i * nrel + r] = kg_set{(uint32_t)fresh[i][1], (uint32_t)fresh[i][2], r, 0};
    std::vector<uint64_t> off(keys.size() + 1, 0);
    std::vector<kg_tuple> tup;
    if (!keys.empty()) {
      const int64_t total = s->rows_of(keys.data(), keys.size(), off.data(), nullptr, 0);
      if (total < 0) return (int)total;
      tup.resize((size_t)total);
      if (total && s->rows_of(keys.data(), keys.size(), off.data(), tup.data(), (uint64_t)total) < 0) return -1;
    }
    std::vector<Row<7>> pay;
    std::vector<int> pdest;
    for (size_t i = 0; i < fresh.size(); i++)
      for (uint64_t j = off[i * nrel]; j < off[(i + 1) * nrel]; j++) {
        const kg_tuple& t = tup[j];
        pay.push_back(Row<7>{fresh[i][0], t.ns, t.obj, t.rel, t.sns, t.sobj, t.srel});
        pdest.push_back((int)fresh[i][0]);
      }
    std::vector<Row<7>> mine;
    if (int rc = a2a_rows<7>(c, pay, pdest, &mine)) return rc;
    std::set<Row<3>> next;
    for (const Row<7>& r : mine) {
      region->push_back(kg_tuple{(uint32_t)r[1], (uint32_t)r[2], (uint32_t)r[3], (uint32_t)r[4], (uint32_t)r[5],
                                 (uint32_t)r[6]});
      if (hop <= gdepth && (uint32_t)r[4] != KG_SUBJECT_ID) next.insert(Row<3>{(uint64_t)c->rank, r[4], r[5]});
    }
    req.assign(next.begin(), next.end());
    uint64_t any = req.empty() ? 0 : 1;
    if (int rc = h_allreduce_max(c, &any, 1)) return rc;
    if (!any) break;
  }
  return 0;
}

static int general_phase(Snapshot* s, ShardComm* c, const kg_query* d_q, size_t n, int32_t gdepth) {
  std::vector<uint8_t> hres(n);
  std::vector<uint32_t> herr(n);
  std::vector<kg_query> hq(n);
  if (n) {
    HIPC(hipMemcpyAsync(hres.data(), c->res, n, hipMemcpyDeviceToHost, c->run));
    HIPC(hipMemcpyAsync(herr.data(), c->err, n * 4, hipMemcpyDeviceToHost, c->run));
    HIPC(hipMemcpyAsync(hq.data(), d_q, n * sizeof(kg_query), hipMemcpyDeviceToHost, c->run));
  }
  HIPC(hipStreamSynchronize(c->run));
  std::vector<uint32_t> open;
  std::vector<kg_query> oq;
  for (size_t i = 0; i < n; i++)
    if (hres[i] == KG_ERROR && herr[i] == KG_ERR_NOT_IMPLEMENTED) {
      open.push_back((uint32_t)i);
      oq.push_back(hq[i]);
    }
  std::vector<kg_tuple> region;
  std::vector<std::pair<uint32_t, uint32_t>> starts;
  for (const kg_query& q : oq) starts.emplace_back(q.t.ns, q.t.obj);
  if (int rc = gather_region(s, c, starts, gdepth, &region)) return rc;
  c->st[5] = open.size();
  c->st[6] = region.size();
  if (open.empty()) return 0;
  // the single-GPU engine (rewrite interpreter included) on a snapshot of the gathered rows
  Snapshot* g = new (std::nothrow) Snapshot();
  if (!g) return set_error(KG_ERR_RESOURCE_CODE, "general phase snapshot");
  kg_rewrite_prog p = s->prog_copy.view();
  const bool prog = s->prog_copy.have && !s->prog_copy.ns_has_rel.empty();
  int rc = g->init_device(s->device);
  if (!rc) rc = g->create_from_tuples(region.data(), region.size(), &s->prog_copy.dict, prog ? &p : nullptr);
  const size_t m = open.size();
  kg_query* dq = nullptr;
  uint8_t* dout = nullptr;
  uint32_t* derr = nullptr;
  std::vector<uint8_t> r(m);
  std::vector<uint32_t> e(m);
  if (!rc && (hipMalloc(&dq, m * sizeof(kg_query)) != hipSuccess || hipMalloc(&dout, m) != hipSuccess ||
              hipMalloc(&derr, m * 4) != hipSuccess))
    rc = set_error(-1, "general phase buffers");
  // everything on the region snapshot's own stream (non-blocking: the null stream would not wait for
  // it), completed before the results are read
  if (!rc && hipMemcpyAsync(dq, oq.data(), m * sizeof(kg_query), hipMemcpyHostToDevice, g->stream) != hipSuccess)
    rc = set_error(-1, "general phase H2D");
  if (!rc) rc = check_batch_device(g, g->workspace(g->stream), dq, m, gdepth, dout, derr, nullptr);
  if (!rc && (hipMemcpyAsync(r.data(), dout, m, hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
              hipMemcpyAsync(e.data(), derr, m * 4, hipMemcpyDeviceToHost, g->stream) != hipSuccess ||
              hipStreamSynchronize(g->stream) != hipSuccess))
    rc = set_error(-1, "general phase D2H");
  if (g->stream) (void)hipStreamSynchronize(g->stream);  // nothing of g's still running when it is freed
  hipFree(dq);
  hipFree(dout);
  hipFree(derr);
  delete g;
  hipSetDevice(s->device);
  if (rc) return rc;
  for (size_t k = 0; k < m; k++) {
    hres[open[k]] = r[k];
    herr[open[k]] = e[k];
  }
  HIPC(hipMemcpyAsync(c->res, hres.data(), n, hipMemcpyHostToDevice, c->run));
  HIPC(hipMemcpyAsync(c->err, herr.data(), n * 4, hipMemcpyHostToDevice, c->run));
  HIPC(hipStreamSynchronize(c->run));
  return 0;
}

// BuildTree on a hash-sharded snapshot (internal/expand/engine.go:35-104): the rows of every object
// within gdepth + 1 subject-set hops of the roots are gathered to this rank (collective, as the general
// phase) and the single-GPU expand runs on a snapshot of them -- the same rows in the same shard order
// per (ns, obj, rel), so the same trees.
int shard_expand(Snapshot* s, const kg_set* roots, size_t n, int32_t gdepth, kg_tree_buf* out) {
  std::shared_ptr<ShardComm> cp = shard_comm_of(s, nullptr);
  ShardComm* c = cp.get();
  if (!c) return set_error(-2, "sharded snapshot: bind a transport to its own stream first (kg_shard_comm_init)");
  std::lock_guard<std::mutex> lk(c->mu);
  HIPC(hipSetDevice(s->device));
  if (gdepth < 1) gdepth = 5;  // config.schema.json:308-315 default
  if (c->world == 1 && !s->shard_force_exchange && s->shard_local) {
    // one rank holds every row: nothing to gather (local-first, as shard_check); the buffers stay on
    // the comm for the next call (held under c->mu, like every other comm buffer)
    return expand_batch(s, s->stream, &c->xbufs, roots, n, gdepth, out);
  }
  std::vector<std::pair<uint32_t, uint32_t>> starts;
  for (size_t i = 0; i < n; i++)
    if (roots[i].sns != KG_SUBJECT_ID) starts.emplace_back(roots[i].sns, roots[i].sobj);
  std::vector<kg_tuple> region;
  if (int rc = gather_region(s, c, starts, gdepth, &region)) return rc;
  c->st[6] = region.size();
  Snapshot* g = new (std::nothrow) Snapshot();
  if (!g) return set_error(KG_ERR_RESOURCE_CODE, "expand region snapshot");
  kg_rewrite_prog p = s->prog_copy.view();
  const bool prog = s->prog_copy.have && !s->prog_copy.ns_has_rel.empty();
  int rc = g->init_device(s->device);
  if (!rc) rc = g->create_from_tuples(region.data(), region.size(), &s->prog_copy.dict, prog ? &p : nullptr);
  void* bufs = nullptr;
  if (!rc) rc = expand_batch(g, g->stream, &bufs, roots, n, gdepth, out);
  if (bufs) expand_bufs_free(bufs);
  delete g;
  hipSetDevice(s->device);
  return rc;
}

// ------------------------------------------------------------------ one batch
// Device buffers a failed step left half-grown are dropped on EVERY rank together, so the next batch
// finds the same allocation state on all of them (allocation decisions stay symmetric: a rank that
// allocates alone would wait in the all-reduce below for ranks that never get there).
static void drop_buffers(ShardComm* c) {
  for (kg_frec** p : {&c->buf[0], &c->buf[1], &c->recv}) {
    hipFree(*p);
    *p = nullptr;
  }
  c->recs = 0;
  hipFree(c->bits);
  hipFree(c->bits_all);
  c->bits = c->bits_all = nullptr;
  c->words_cap = c->all_cap = 0;
}

// Bucket buffers may take this much (kg_snapshot_tune "shard_max_bytes"; default a quarter of the free
// HBM, counting what the buffers being replaced hold).
static uint64_t bucket_byte_cap(const Snapshot* s, const ShardComm* c) {
  if (s->shard_max_bytes) return s->shard_max_bytes;
  size_t fr = 0, total = 0;
  if (hipMemGetInfo(&fr, &total) != hipSuccess) return ~0ull;
  return (fr + 3 * c->recs * sizeof(kg_frec)) / 4;
}

// Grows the buffers of one run of the protocol.  Collective when `xch`: every rank reaches this with
// the same B and the same history, so all of them allocate (and agree) on the same runs; a failure on
// any rank -- a cap or an out-of-memory -- is returned by all of them.
static int grow_run(Snapshot* s, ShardComm* c, bool xch, size_t B, uint32_t words) {
  const size_t N = (size_t)c->world;
  const bool g_bits = !c->bits || !c->bits_all || (size_t)words + 1 > c->words_cap || N * words + 1 > c->all_cap;
  const bool g_recs = N * B > c->recs || !c->buf[0];
  if (!g_bits && !g_recs) return 0;
  uint64_t f = 0;
  const uint64_t bytes = 3ull * N * B * sizeof(kg_frec), cap = bucket_byte_cap(s, c);
  if (g_recs) {
    for (kg_frec** p : {&c->buf[0], &c->buf[1], &c->recv}) {
      hipFree(*p);
      *p = nullptr;
    }
    c->recs = 0;
    if (bytes > cap) f = 1;
    for (kg_frec** p : {&c->buf[0], &c->buf[1], &c->recv})
      if (!f && hipMalloc((void**)p, N * B * sizeof(kg_frec)) != hipSuccess) f = 2;
    if (!f) c->recs = N * B;
  }
  if (!f && g_bits &&
      (grow((void**)&c->bits, &c->words_cap, (size_t)words + 1, 4) ||
       grow((void**)&c->bits_all, &c->all_cap, N * words + 1, 4)))
    f = 2;
  const uint64_t mine = f;
  if (xch) {
    if (int rc = h_allreduce_max(c, &f, 1)) return rc;
    c->st[2]++;
  }
  if (!f) return 0;
  drop_buffers(c);
  if (f == 1 && mine)
    return set_error(KG_ERR_RESOURCE_CODE,
                     "sharded batch: bucket buffers of %zu records per destination need %.3g GB, over the %.3g GB "
                     "cap (kg_snapshot_tune shard_max_bytes)", B, bytes / 1e9, cap / 1e9);
  return set_error(KG_ERR_RESOURCE_CODE, "sharded batch: buffer allocation failed on %s",
                   mine ? "this rank" : "another rank");
}

int shard_check(Snapshot* s, ShardComm* c, const kg_query* d_q, size_t n, int32_t gdepth, uint8_t* d_out,
                uint32_t* d_err, kg_stats* stats) {
  std::lock_guard<std::mutex> lk(c->mu);
  HIPC(hipSetDevice(s->device));
  if (gdepth < 1) gdepth = 5;  // config.schema.json:308-315 default (as kg_shard_seed)
  hipStream_t st = c->run;
  const uint32_t N = (uint32_t)c->world;
  // the exchange protocol runs at N > 1, and at N = 1 when forced (kg_snapshot_tune
  // "shard_force_exchange": the same RCCL calls as N > 1, each rank its own peer)
  const bool xch = N > 1 || s->shard_force_exchange;
  memset(c->st, 0, sizeof c->st);
  if (!xch && s->shard_local) {
    // Local-first, one rank: every row is this rank's, so no record of the level protocol would ever
    // leave it -- the batch runs the replica engine's tier chain (k_resolve -> k_stream4 -> k_back ->
    // grid tiers / rewrite interpreter) on the bound stream's workspace instead of level-synchronous
    // records with a (query, node) CAS each (kg_snapshot_tune "shard_local" 0: the device
    // level loop below).
    c->st[10] = 0;
    Workspace* w = s->workspace(st);
    std::lock_guard<std::mutex> wl(w->mu);
    return check_batch_device(s, w, d_q, n, gdepth, d_out, d_err, stats);
  }
  c->st[10] = xch ? 2 : 1;
  if (stats) {
    memset(stats, 0, sizeof *stats);
    for (auto& e : c->ev)
      if (!e) HIPC(hipEventCreate(&e));
    HIPC(hipEventRecord(c->ev[0], st));
  }
  // Before the first collective, what only this rank can know: whether it can run its batch at all
  // and its result buffers (sized by its own batch).  The agreement all-reduce then carries a failure
  // flag beside the largest result-slot count of any rank (the done bitmap's width), so a rank that
  // cannot go on never leaves the others waiting in a later collective (host round trip 1; one rank
  // without the exchange needs none).
  const size_t slots = shard_result_slots(s, n);
  uint64_t bad = (n > 0x7FFFFFFFull || slots > shard_slot_limit()) ? 1 : 0;
  if (!bad && (slots > c->slots_cap || !c->res)) {
    hipFree(c->res);
    hipFree(c->err);
    c->res = nullptr;
    c->err = nullptr;
    c->slots_cap = 0;
    const size_t m = std::max<size_t>(slots, 1024);
    if (hipMalloc((void**)&c->res, m) != hipSuccess || hipMalloc((void**)&c->err, m * 4) != hipSuccess) bad = 2;
    else c->slots_cap = m;
  }
  uint64_t agree[2] = {slots, bad};
  if (xch) {
    if (int rc = h_allreduce_max(c, agree, 2)) return rc;
    c->st[2]++;
  }
  if (agree[1]) {
    if (bad == 1) return set_error(-2, "sharded batch too large (%zu queries, %zu result slots > %zu)", n, slots,
                                   shard_slot_limit());
    return set_error(bad ? KG_ERR_RESOURCE_CODE : -2, "sharded batch: %s", bad ? "result buffers" :
                     "another rank cannot run its batch (too large, or out of memory)");
  }
  const uint64_t smax = agree[0];
  const uint32_t words = (uint32_t)((smax + 31) / 32);
  const size_t B0 = std::min<size_t>(2 * smax / N + 1024, 1ull << 26);
  // exchanges k = 0 .. L - 1 (L = gdepth + 1); lb[L] bounds what the last level emits (nothing)
  const int L = gdepth + 1;
  if (xch && (int)c->lb.size() != L + 1) c->lb.assign((size_t)L + 1, c->bucket ? c->bucket : B0);
  if (xch && c->red_cap < (size_t)(8 + L)) {
    hipFree(c->red);
    c->red = nullptr;
    c->red_cap = 0;
    uint64_t f = hipMalloc((void**)&c->red, (size_t)(8 + L) * 8) != hipSuccess ? 1 : 0;
    const uint64_t mine = f;
    if (int rc = h_allreduce_max(c, &f, 1)) return rc;
    c->st[2]++;
    if (f) {
      hipFree(c->red);
      c->red = nullptr;
      return set_error(KG_ERR_RESOURCE_CODE, "sharded batch: reduction buffer (%s)", mine ? "this rank" : "another rank");
    }
    c->red_cap = (size_t)(8 + L);
  }
  uint32_t* counts[2] = {c->cnt, c->cnt + (N + 1)};
  uint32_t* rcv = c->cnt + 2 * (N + 1);
  // the backward phase's (count, flags) pairs and received counts (escalation)
  uint32_t* cb[2] = {c->cnt + 3 * N + 2, c->cnt + 3 * N + 4};
  uint32_t* rcvb = c->cnt + 3 * N + 6;
  unsigned long long* acc = c->acc;
  // tot[0..5] = (bucket overflow, visited overflow, largest bucket / bucket needed, records left, a
  // query needs the general phase, largest backward bucket), then per exchange its largest bucket
  unsigned long long* tot = xch ? c->red : c->acc + 4;
  unsigned long long* lvl = xch ? c->red + 8 : nullptr;
  const size_t nred = xch ? (size_t)(8 + L) : 6;
  std::vector<uint64_t> h(nred + 2);
  // Escalation (kg_snapshot_tune "shard_budget"; no namespace program): the forward phase drops a query
  // past its set-edge budget on a rank (ESC), a backward phase from the subjects' holders answers it, and
  // queries past the backward budget too (ESC2) walk forward once more from their roots without one
  // (keto_amd/sharded.py ShardedChecker's three phases; the single-GPU k_stream4 -> k_back -> grid chain)
  const bool esc = shard_escalates(s);
  if (esc && !c->bb) c->bb = B0;
  // reruns after a bucket overflow are bounded (kg_snapshot_tune "shard_max_reruns"); the visited table
  // grows 4x per visited-overflow rerun up to 2^34 keys, its own bound
  uint32_t run = 0;
  for (;;) {
    size_t B;
    if (xch) B = *std::max_element(c->lb.begin(), c->lb.end());
    else B = c->bucket ? c->bucket : B0;
    if (!xch) c->bucket = B;
    if (esc) B = std::max(B, c->bb);  // the backward phase all-gathers N buckets of bb into recv
    if (int rc = grow_run(s, c, xch, B, words)) return rc;
    HIPC(hipMemsetAsync(acc, 0, 32 * 8, st));
    if (xch) HIPC(hipMemsetAsync(c->red, 0, (size_t)(8 + L) * 8, st));
    // every count buffer starts clear: the flags word counts[k][N] accumulates over the levels that
    // write buffer k, and shard_seed / shard_level clear only what they write
    HIPC(hipMemsetAsync(c->cnt, 0, (4 * (size_t)N + 6) * 4, st));
    if (int rc = shard_seed(s, d_q, n, gdepth, c->buf[0], xch ? c->lb[0] : B, counts[0], c->res, c->err, st))
      return rc;
    int cur = 0;
    uint64_t wire = 0;  // bytes this rank puts on the wire (every destination but itself gets B_k records)
    c->st[12] = 0;
    if (!xch) {
      // one rank, device loop: nothing to exchange -- gdepth levels back to back (per-XCD sub-buckets,
      // hub rows grid-wide; kg_shard_levels), hit reports stay local; the loop reports the bucket
      // size its levels needed (tot[2]), so an overflow reruns once at the right size
      kg_frec* bufs[2] = {c->buf[0], c->buf[1]};
      if (int rc = shard_levels(s, gdepth, bufs, B, counts, 0, c->res, c->err, c->prune ? slots : 0, esc ? 1 : 0, &cur,
                                st, tot + 2))
        return rc;
      c->st[0] += (uint64_t)gdepth;
      if (esc) {
        hipLaunchKernelGGL(k_sc_loop_end, dim3(1), dim3(64), 0, st, counts[0], counts[1], cur, acc);
        HIPC(hipGetLastError());
        // backward: this rank's escalated queries (the list) -> their subjects' holders -> gdepth
        // reverse levels, the done bitmap counting members and queries past the backward budget
        if (int rc = shard_back_list(s, slots, c->res, c->err, c->recv, B, cb[0], st)) return rc;
        hipLaunchKernelGGL(k_sc_back, dim3(1), dim3(64), 0, st, cb[0], (uint32_t)B, 0, acc);
        if (int rc = shard_back_seed(s, c->recv, B, cb[0], bufs[0], B, cb[1], st)) return rc;
        hipLaunchKernelGGL(k_sc_back, dim3(1), dim3(64), 0, st, cb[1], (uint32_t)B, 0, acc);
        uint32_t* cbl[2] = {cb[1], cb[0]};  // the seed wrote buffer 0 with cb[1]
        int bc = 0;
        for (int k = 0; k < gdepth; k++) {
          if (int rc = shard_done(s, slots, c->res, c->err, 2, c->bits, words, st)) return rc;
          if (int rc = shard_back_level(s, bufs[bc], B, cbl[bc], bufs[bc ^ 1], B, cbl[bc ^ 1], c->res, c->err, c->bits,
                                        words, st))
            return rc;
          hipLaunchKernelGGL(k_sc_back, dim3(1), dim3(64), 0, st, cbl[bc ^ 1], (uint32_t)B, k == gdepth - 1 ? 1 : 0,
                             acc);
          bc ^= 1;
          c->st[12]++;
        }
        // final forward phase: queries past both budgets, re-seeded at their roots, no budget
        if (int rc = shard_refwd_seed(s, slots, c->res, c->err, bufs[0], B, counts[0], st)) return rc;
        HIPC(hipMemsetAsync(counts[1], 0, (N + 1) * 4, st));
        if (int rc = shard_levels(s, gdepth, bufs, B, counts, 0, c->res, c->err, c->prune ? slots : 0, 0, &cur, st,
                                  tot + 2))
          return rc;
        c->st[12] += (uint64_t)gdepth;
      }
      hipLaunchKernelGGL(k_sc_final1, dim3(1), dim3(64), 0, st, counts[0], counts[1], cur, acc, tot);
      HIPC(hipGetLastError());
    }
    // the forward exchange protocol: L exchanges, then (escalation) the backward phase over all-gathers
    // and a second forward pass for the queries past both budgets
    // exchanges of this run: the learned count (no escalation: its phases keep all L)
    const int LX = (xch && !esc && c->lx > 0) ? std::min(L, c->lx) : L;
    for (int phase = 0; xch && phase < (esc ? 2 : 1); phase++) {
      for (int k = 0; k < LX; k++) {
        const size_t Bk = c->lb[(size_t)k], Bn = c->lb[(size_t)k + 1];
        const int nx = cur ^ 1;
        // one kernel: the outgoing counts into the accumulators, the level's output counters and hub
        // head cleared, and (from the second exchange) the done bitmap -- the escalating forward phase
        // counts escalated queries as done too
        const bool with_done = c->prune && k > 0;
        if (int rc = shard_pre_level(s, st, counts[cur], N, (uint32_t)Bk, (uint32_t)c->rank, acc, lvl + k, counts[nx],
                                     slots, c->res, c->err, esc && phase == 0 ? 1 : 0, c->bits, with_done ? words : 0u))
          return rc;
        if (int rc = x_alltoall2(c, counts[cur], rcv, 4, c->buf[cur], c->recv, Bk * sizeof(kg_frec))) return rc;
        wire += (uint64_t)(N - 1) * (4 + Bk * sizeof(kg_frec));
        const uint32_t* done = nullptr;
        if (with_done) {
          if (int rc = x_allgather(c, c->bits, c->bits_all, (size_t)words * 4)) return rc;
          wire += (uint64_t)(N - 1) * words * 4;
          done = c->bits_all;
        }
        if (int rc = shard_level(s, c->recv, (size_t)N * Bk, rcv, c->buf[nx], Bn, counts[nx], c->res, c->err, done,
                                 words, st, N, Bk, true))
          return rc;
        cur = nx;
        c->st[phase ? 12 : 0]++;
      }
      if (!esc || phase == 1) break;
      hipLaunchKernelGGL(k_sc_phase_end, dim3(1), dim3(64), 0, st, counts[cur], N, (uint32_t)c->lb[(size_t)L], acc);
      HIPC(hipGetLastError());
      // backward phase: every rank sees every backward record (a node's parents sit in their owners'
      // rows, and every rank holds the reverse set-adjacency of its own rows), so each level all-gathers
      // fixed buckets of bb records with their counts; gdepth levels after the seed drain it (rest depths
      // fall by one per level; the last one only delivers hit / escalation reports)
      const size_t bb = c->bb;
      if (int rc = shard_back_list(s, slots, c->res, c->err, c->buf[0], bb, cb[0], st)) return rc;
      hipLaunchKernelGGL(k_sc_back, dim3(1), dim3(64), 0, st, cb[0], (uint32_t)bb, 0, acc);
      if (int rc = x_allgather(c, cb[0], rcvb, 4)) return rc;
      if (int rc = x_allgather(c, c->buf[0], c->recv, bb * sizeof(kg_frec))) return rc;
      wire += (uint64_t)(N - 1) * (4 + bb * sizeof(kg_frec));
      if (int rc = shard_back_seed(s, c->recv, (size_t)N * bb, rcvb, c->buf[1], bb, cb[1], st, N, bb)) return rc;
      hipLaunchKernelGGL(k_sc_back, dim3(1), dim3(64), 0, st, cb[1], (uint32_t)bb, 0, acc);
      int bc = 1;
      for (int k = 0; k < gdepth; k++) {
        if (int rc = x_allgather(c, cb[bc], rcvb, 4)) return rc;
        if (int rc = x_allgather(c, c->buf[bc], c->recv, bb * sizeof(kg_frec))) return rc;
        if (int rc = shard_done(s, slots, c->res, c->err, 2, c->bits, words, st)) return rc;
        if (int rc = x_allgather(c, c->bits, c->bits_all, (size_t)words * 4)) return rc;
        wire += (uint64_t)(N - 1) * (8 + bb * sizeof(kg_frec) + words * 4);
        if (int rc = shard_back_level(s, c->recv, (size_t)N * bb, rcvb, c->buf[bc ^ 1], bb, cb[bc ^ 1], c->res, c->err,
                                      c->bits_all, words, st, N, bb))
          return rc;
        hipLaunchKernelGGL(k_sc_back, dim3(1), dim3(64), 0, st, cb[bc ^ 1], (uint32_t)bb, k == gdepth - 1 ? 1 : 0, acc);
        bc ^= 1;
        c->st[12]++;
      }
      // final forward phase: this rank's queries past both budgets, re-seeded at their roots' owners
      if (int rc = shard_refwd_seed(s, slots, c->res, c->err, c->buf[0], c->lb[0], counts[0], st)) return rc;
      cur = 0;
    }
    if (xch) {
      // what the last exchange run left for the next one: bounded by that exchange's bucket (LX < L) or
      // by nothing (LX = L: lb[L] -- the last level emits nothing)
      hipLaunchKernelGGL(k_sc_final, dim3(1), dim3(64), 0, st, counts[cur], N, (uint32_t)c->lb[(size_t)LX], acc, tot);
      HIPC(hipGetLastError());
    }
    // results final before the all-reduce, which then also carries "a query needs the general phase"
    if (int rc = shard_finish(s, n, c->res, c->err, st)) return rc;
    if (n) {
      hipLaunchKernelGGL(k_sc_open, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, (uint32_t)n, c->res, c->err,
                         tot);
      HIPC(hipGetLastError());
    }
    if (xch)
      if (int rc = x_allreduce_max(c, tot, nred)) return rc;
    HIPC(hipMemcpyAsync(h.data(), tot, nred * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(h.data() + nred, acc + 2, 16, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));  // host round trip 2
    c->st[2]++;
    if (xch && LX < L && h[3]) {  // records left after the learned exchanges: rerun with all of them
      c->lx = L;
      c->st[13]++;
      continue;
    }
    if (h[0] || h[1] || s->shard_force_overflow) {  // dropped records somewhere: every rank reruns with more room
      const bool bucket_over = h[0] || s->shard_force_overflow;
      // a run whose visited table overflowed too dropped records for that reason as well, so its
      // bucket counts are lower bounds: only runs without it count against the bucket-rerun bound
      // an exchange downstream of one that dropped records reports a lower bound, so each rerun may
      // fix one more exchange: the default (0) allows max(4, L + 1) reruns
      const uint32_t max_reruns = s->shard_max_reruns ? s->shard_max_reruns : std::max<uint32_t>(4, xch ? (uint32_t)L + 1 : 0u);
      if (bucket_over && !h[1] && run++ >= max_reruns) {
        drop_buffers(c);
        return set_error(KG_ERR_RESOURCE_CODE,
                         "sharded batch still overflows after %u reruns (bucket %zu records per destination, "
                         "visited table 2^%d keys; kg_snapshot_tune shard_max_reruns)", run - 1, B, s->shard_vis_log2);
      }
      if (bucket_over) {
        c->st[3]++;
        const size_t top = 1ull << 30;
        if (xch) {
          // every exchange that overflowed gets at least what it needed (its counter counted past
          // B_k) plus a quarter, and at least twice its old size; records it dropped were missing
          // downstream, so the counts of every later exchange are lower bounds: they get at least the
          // largest size any overflowed exchange now has (levels are the same order of magnitude)
          size_t grown = 0;
          bool after = false;
          for (int k = 0; k <= L; k++) {
            const uint64_t need = k < L ? h[8 + (size_t)k] : 0;
            size_t& b = c->lb[(size_t)k];
            if (need > b || (s->shard_force_overflow && !h[0])) {
              b = std::min(top, std::max((size_t)(need * 1.25) + 1024, 2 * b));
              grown = std::max(grown, b);
              after = true;
            } else if (after) {
              b = std::min(top, std::max(b, grown));
            }
          }
        } else {
          // the device loop's fold reported the bucket its levels needed (a lower bound past the first
          // level that dropped records): that plus a quarter, and at least twice the old size
          const uint64_t need = h[2];
          c->bucket = std::min(top, std::max<size_t>(2 * B, (size_t)(need * 1.25) + 1024));
        }
      }
      if (esc && h[5] > c->bb) c->bb = std::min<size_t>(1ull << 30, std::max((size_t)(h[5] * 1.25) + 1024, 2 * c->bb));
      if (h[1]) {
        c->st[4]++;
        if (s->shard_vis_log2 >= 34) return set_error(KG_ERR_RESOURCE_CODE, "sharded visited table overflow");
        s->shard_vis_log2 = std::min(34, s->shard_vis_log2 + 2);
      }
      continue;
    }
    if (h[3]) return set_error(-1, "sharded batch: records left after %d levels", xch ? L : gdepth);
    if (esc && h[5] * 2 < c->bb) c->bb = std::max<size_t>(1024, std::min<size_t>(c->bb, (size_t)(h[5] * 1.25) + 1024));
    if (xch) {
      // next batch: each exchange's bucket 25 % above what it needed this batch (shrinking slowly)
      c->st[9] = wire;
      for (int k = 0; k <= L; k++) {
        const uint64_t need = k < L ? h[8 + (size_t)k] : 0;
        size_t& b = c->lb[(size_t)k];
        if (need * 2 < b) b = std::max<size_t>(1024, std::min<size_t>(b, (size_t)(need * 1.25) + 1024));
      }
      c->lvl_last.assign(h.begin() + 8, h.begin() + 8 + L);
      c->lb_last.assign(c->lb.begin(), c->lb.begin() + L);
      int last = -1;  // the last exchange that carried records (per-exchange largest bucket, max over ranks)
      for (int k = 0; k < LX; k++)
        if (h[8 + (size_t)k]) last = k;
      c->lx = std::min(L, last + 2);
      c->st[11] = (uint64_t)LX;
    }
    c->st[1] = h[nred];
    c->st[8] = h[nred + 1];
    if (h[4])
      if (int rc = general_phase(s, c, d_q, n, gdepth)) return rc;
    break;
  }
  c->st[7] = xch ? *std::max_element(c->lb.begin(), c->lb.end()) : c->bucket;
  if (!xch) c->st[11] = 0;
  if (n) {
    HIPC(hipMemcpyAsync(d_out, c->res, n, hipMemcpyDeviceToDevice, st));
    if (d_err) HIPC(hipMemcpyAsync(d_err, c->err, n * 4, hipMemcpyDeviceToDevice, st));
  }
  if (stats) {
    HIPC(hipEventRecord(c->ev[1], st));
    HIPC(hipEventSynchronize(c->ev[1]));
    float ms = 0;
    HIPC(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    stats->kernel_ms = ms;
  }
  return 0;
}

// Host buffers: staged through the binding's device buffers, on the bound stream (one host batch at a
// time per binding: the staging buffers are the binding's).
static int shard_check_host(Snapshot* s, ShardComm* c, const kg_query* q, size_t n, int32_t gdepth, uint8_t* out,
                            uint32_t* err, kg_stats* stats) {
  std::lock_guard<std::mutex> hl(c->host_mu);
  {
    std::lock_guard<std::mutex> lk(c->mu);
    HIPC(hipSetDevice(s->device));
    if (n > c->dq_cap || !c->dq) {
      hipFree(c->dq);
      hipFree(c->dout);
      hipFree(c->derr);
      c->dq = nullptr;
      c->dout = nullptr;
      c->derr = nullptr;
      c->dq_cap = 0;
      const size_t m = std::max<size_t>(n, 1024);
      HIPC(hipMalloc((void**)&c->dq, m * sizeof(kg_query)));
      HIPC(hipMalloc((void**)&c->dout, m));
      HIPC(hipMalloc((void**)&c->derr, m * 4));
      c->dq_cap = m;
    }
    if (n) HIPC(hipMemcpyAsync(c->dq, q, n * sizeof(kg_query), hipMemcpyHostToDevice, c->run));
  }
  if (int rc = shard_check(s, c, c->dq, n, gdepth, c->dout, c->derr, stats)) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  if (n) {
    HIPC(hipMemcpyAsync(out, c->dout, n, hipMemcpyDeviceToHost, c->run));
    if (err) HIPC(hipMemcpyAsync(err, c->derr, n * 4, hipMemcpyDeviceToHost, c->run));
  }
  HIPC(hipStreamSynchronize(c->run));
  return 0;
}

int shard_check_host_entry(Snapshot* s, const kg_query* q, size_t n, int32_t gdepth, uint8_t* out, uint32_t* err,
                           kg_stats* stats) {
  std::shared_ptr<ShardComm> c = shard_comm_of(s, nullptr);
  if (!c) return set_error(-2, "sharded snapshot: bind a transport to its own stream first (kg_shard_comm_init)");
  return shard_check_host(s, c.get(), q, n, gdepth, out, err, stats);
}

int shard_check_entry(Snapshot* s, hipStream_t stream, const kg_query* d_q, size_t n, int32_t gdepth, uint8_t* d_out,
                      uint32_t* d_err, kg_stats* stats, bool* handled) {
  std::shared_ptr<ShardComm> c = shard_comm_of(s, stream);
  *handled = c != nullptr;
  if (!c) return 0;
  return shard_check(s, c.get(), d_q, n, gdepth, d_out, d_err, stats);
}

}  // namespace kg

using kg::set_error;

extern "C" {

int kg_shard_unique_id(void* id) {
  if (!id) return set_error(-2, "NULL argument");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return set_error(-1, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  static_assert(sizeof(u) == KG_SHARD_UNIQUE_ID_BYTES, "ncclUniqueId size");
  memcpy(id, &u, sizeof u);
  return 0;
}

int kg_shard_comm_init(kg_snapshot* sp, const void* id, int rank, int world, void* stream) {
  try {
    if (!sp || !id) return set_error(-2, "NULL argument");
    if (world < 1 || world > KG_SHARD_MAX_RANKS || rank < 0 || rank >= world)
      return set_error(-2, "bad rank %d of %d", rank, world);
    kg::Snapshot* s = reinterpret_cast<kg::Snapshot*>(sp);
    HIPC(hipSetDevice(s->device));
    kg::ShardComm* c = new kg::ShardComm();
    c->rank = rank;
    c->world = world;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclResult_t r = ncclCommInitRank(&c->nccl, world, u, rank);
    if (r != ncclSuccess) {
      c->nccl = nullptr;
      delete c;
      return set_error(-1, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    c->t = kg_shard_transport{c, rank, world, 0, kg::rccl_alltoall2, kg::rccl_allgather, kg::rccl_allreduce_max};
    return kg::bind(s, c, (hipStream_t)stream);  // owns c
  } catch (...) {
    return set_error(-4, "kg_shard_comm_init: exception");
  }
}

int kg_shard_transport_attach(kg_snapshot* sp, const kg_shard_transport* t, void* stream) {
  try {
    if (!sp || !t || !t->alltoall2 || !t->allgather || !t->allreduce_max_u64) return set_error(-2, "NULL argument");
    if (t->world < 1 || t->world > KG_SHARD_MAX_RANKS || t->rank < 0 || t->rank >= t->world)
      return set_error(-2, "bad rank %d of %d", t->rank, t->world);
    kg::Snapshot* s = reinterpret_cast<kg::Snapshot*>(sp);
    HIPC(hipSetDevice(s->device));
    kg::ShardComm* c = new kg::ShardComm();
    c->rank = t->rank;
    c->world = t->world;
    c->t = *t;
    return kg::bind(s, c, (hipStream_t)stream);  // owns c
  } catch (...) {
    return set_error(-4, "kg_shard_transport_attach: exception");
  }
}

int kg_shard_comm_release(kg_snapshot* sp, void* stream) {
  if (!sp) return set_error(-2, "NULL snapshot");
  kg::Snapshot* s = reinterpret_cast<kg::Snapshot*>(sp);
  std::shared_ptr<kg::ShardComm> gone;  // destroyed outside the lock, once no caller is inside a batch with it
  std::lock_guard<std::mutex> lk(s->comm_mu);
  for (auto it = s->comms.begin(); it != s->comms.end(); ++it)
    if ((*it)->bound == (hipStream_t)stream) {
      gone = *it;
      s->comms.erase(it);
      s->n_comms.store((int)s->comms.size(), std::memory_order_release);
      return 0;
    }
  return set_error(-2, "no transport bound to this stream");
}

int kg_shard_comm_stats_ex(const kg_snapshot* sp, void* stream, uint64_t* out, size_t n) {
  if (!sp || (n && !out)) return set_error(-2, "NULL argument");
  kg::Snapshot* s = const_cast<kg::Snapshot*>(reinterpret_cast<const kg::Snapshot*>(sp));
  std::shared_ptr<kg::ShardComm> c = kg::shard_comm_of(s, (hipStream_t)stream);
  if (!c) return set_error(-2, "no transport bound to this stream");
  std::lock_guard<std::mutex> lk(c->mu);
  const size_t m = sizeof c->st / sizeof c->st[0];
  for (size_t i = 0; i < n; i++) out[i] = i < m ? c->st[i] : 0;
  return 0;
}

int kg_shard_comm_stats(const kg_snapshot* sp, void* stream, uint64_t out8[8]) {
  return kg_shard_comm_stats_ex(sp, stream, out8, 8);
}

int64_t kg_shard_comm_levels(const kg_snapshot* sp, void* stream, uint64_t* out, size_t cap) {
  if (!sp || (cap && !out)) return set_error(-2, "NULL argument");
  kg::Snapshot* s = const_cast<kg::Snapshot*>(reinterpret_cast<const kg::Snapshot*>(sp));
  std::shared_ptr<kg::ShardComm> c = kg::shard_comm_of(s, (hipStream_t)stream);
  if (!c) return set_error(-2, "no transport bound to this stream");
  std::lock_guard<std::mutex> lk(c->mu);
  const size_t L = c->lvl_last.size();
  for (size_t k = 0; k < L && 2 * k + 1 < cap; k++) {
    out[2 * k] = c->lb_last[k];
    out[2 * k + 1] = c->lvl_last[k];
  }
  return (int64_t)L;
}

}  // extern "C"
