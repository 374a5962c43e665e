"""Hash-sharded batched checks: graphs larger than one GPU's HBM.

Rank r of N holds the rows of the nodes (ns, obj, rel) with kg_shard_owner(ns, obj, N) == r
(all relations of one object on one rank).  A batch is a level-synchronous BFS across ranks:

  seed    each rank maps its own queries (its slice of the batch) and sends one frontier record
          (query, root, subject, depth) to the root's owner            -- kg_shard_seed
  level   every rank processes the records it received: hit reports set its queries' results;
          otherwise the owner deduplicates (query, node), probes checkDirect on its rows, reports
          a hit to the query's home rank or expands the node's set row into records for the
          children's owners                                             -- kg_shard_level
  exchange the per-destination buckets go through one all-to-all (RCCL over xGMI with the
          "nccl" backend; staged through host memory with gloo) after an all-to-all of
          per-destination metadata (bucket size, records sent in total, overflow flags), which
          gives every rank its receive sizes, termination (nothing sent anywhere) and overflow
          (every rank reruns the batch with larger buckets) for ONE host round trip per level;
          a single rank enqueues every level without any (record counts stay on the device)

Results are those of the single-GPU engine (bounded reachability, internal/check/engine.go:87-207
with the SURVEY.md 8a semantics).  Union rewrites (or / computedUserset / tupleToUserset) are
materialised into plain union nodes on every rank alike; a query whose relation is a boolean formula
over plain or union relations is split into parts (its own rows and one per leaf relation) that
travel as queries of their own in extra result slots, and kg_shard_finish evaluates the formula.  A
query that reaches any other rewrite or an undeclared relation (an impure union, a formula recursive
through tuple-to-subject-set such as the reference parser's full example's `view`) ends the level
protocol as KG_ERR_NOT_IMPLEMENTED and goes to the general phase: the rows of every object within
gdepth + 1 subject-set hops of its root are gathered to its home rank and the single-GPU engine
(rewrite interpreter included) answers it on a snapshot of them.  The local steps are
`ShardOps` objects: `HipShardOps` runs them on the GPU through the C ABI; the multi-rank CPU
tests substitute a test-only restatement to exercise this exchange protocol under gloo.

Round 4: the product path is `LibShardedChecker` -- the same fixed-bucket protocol and general phase
inside libketogpu.so (kg_shard_comm.hip), one kg_check_batch_device call per batch over RCCL, as a
Go host calls it.  `ShardedChecker` stays as the CPU-tested restatement of the protocol and the
driver of the opt-in escalation phases (kg_snapshot_tune "shard_budget").
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Tuple

import numpy as np

from . import _lib

REC_WORDS = 4  # kg_frec = (q, node, subj, depth) as int32


class HipShardOps:
    """The local steps of one rank on its GPU (kg_shard_seed / kg_shard_level / kg_shard_finish)."""

    device_counts = True  # kg_shard_level can read its record count from device memory

    @property
    def escalates(self) -> bool:
        """The backward and final forward phases run only with a forward budget (kg_snapshot_tune
        "shard_budget", off by default): their levels cost launches even when empty."""
        return getattr(self.snapshot, "tuned", {}).get("shard_budget", 0) > 0

    def __init__(self, snapshot):
        import torch
        self.snapshot = snapshot
        # a dedicated (non-null) torch stream: the C ABI reads a NULL stream as "the snapshot's own
        # stream", so the null stream could not order the library's kernels with torch's copies
        self.torch_stream = torch.cuda.Stream()
        self.L = _lib.load()

    def _s(self):
        return C.c_void_p(self.torch_stream.cuda_stream)

    def seed(self, dq, n, gdepth, out, cap, counts, res, err):
        _lib.check(self.L.kg_shard_seed(self.snapshot.handle, dq.data_ptr() if n else None, n, gdepth,
                                        out.data_ptr(), cap, counts.data_ptr(), res.data_ptr(), err.data_ptr(),
                                        self._s()), "kg_shard_seed")

    def grow_visited(self):
        self.vis_log2 = getattr(self, "vis_log2", 23) + 1
        self.snapshot.tune("shard_vis", self.vis_log2)

    def level(self, din, n_in, n_in_dev, out, cap, counts, res, err, done=None, done_words=0):
        """n_in_dev: None, or a device int32 tensor whose element 0 is the record count (n_in bounds it).
        done: None, or the batch's done bitmap (done_words int32 words per rank)."""
        _lib.check(self.L.kg_shard_level(self.snapshot.handle, din.data_ptr() if n_in else None, n_in,
                                         n_in_dev.data_ptr() if n_in_dev is not None else None, out.data_ptr(), cap,
                                         counts.data_ptr(), res.data_ptr(), err.data_ptr(),
                                         done.data_ptr() if done is not None else None, done_words, self._s()),
                   "kg_shard_level")

    def levels(self, k, bufs, cap, counts, cur, res, err, slots, esc_mode=0):
        """One rank: k levels back to back in one library call (kg_shard_levels); returns the buffer the
        last level wrote."""
        end = C.c_int32(cur)
        _lib.check(self.L.kg_shard_levels(self.snapshot.handle, k, bufs[0].data_ptr(), bufs[1].data_ptr(), cap,
                                          counts[0].data_ptr(), counts[1].data_ptr(), cur, res.data_ptr(),
                                          err.data_ptr(), slots, esc_mode, C.byref(end), self._s()), "kg_shard_levels")
        return int(end.value)

    def level_seg(self, din, n_seg, seg_cap, seg_counts, out, cap, counts, res, err, done=None, done_words=0):
        """kg_shard_level over a fixed-split receive buffer: segment k = din[k * seg_cap:], seg_counts[k]
        records (a device int32 tensor, clamped to seg_cap)."""
        _lib.check(self.L.kg_shard_level_seg(self.snapshot.handle, din.data_ptr(), n_seg, seg_cap,
                                             seg_counts.data_ptr(), out.data_ptr(), cap, counts.data_ptr(),
                                             res.data_ptr(), err.data_ptr(),
                                             done.data_ptr() if done is not None else None, done_words, self._s()),
                   "kg_shard_level_seg")

    def done_bits(self, res, n, words, err=None, mode=1):
        """err given: queries escalated out of the current phase count as done (mode 1: the forward
        phase, 2: the backward phase)."""
        import torch
        bits = torch.empty(max(words, 1), dtype=torch.int32, device=res.device)
        _lib.check(self.L.kg_shard_done(self.snapshot.handle, n, res.data_ptr(),
                                        err.data_ptr() if err is not None else None, mode if err is not None else 0,
                                        bits.data_ptr(), words, self._s()), "kg_shard_done")
        return bits[:words]

    # ---- backward phase (escalated queries; kg_shard_back_*)
    def back_list(self, n, res, err, out, cap, counts):
        _lib.check(self.L.kg_shard_back_list(self.snapshot.handle, n, res.data_ptr(), err.data_ptr(), out.data_ptr(),
                                             cap, counts.data_ptr(), self._s()), "kg_shard_back_list")

    def back_seed(self, lst, m, m_dev, out, cap, counts):
        _lib.check(self.L.kg_shard_back_seed(self.snapshot.handle, lst.data_ptr() if m else None, m,
                                             m_dev.data_ptr() if m_dev is not None else None, out.data_ptr(), cap,
                                             counts.data_ptr(), self._s()), "kg_shard_back_seed")

    def back_level(self, din, n_in, n_in_dev, out, cap, counts, res, err, done=None, done_words=0):
        _lib.check(self.L.kg_shard_back_level(self.snapshot.handle, din.data_ptr() if n_in else None, n_in,
                                              n_in_dev.data_ptr() if n_in_dev is not None else None, out.data_ptr(),
                                              cap, counts.data_ptr(), res.data_ptr(), err.data_ptr(),
                                              done.data_ptr() if done is not None else None, done_words, self._s()),
                   "kg_shard_back_level")

    def refwd_seed(self, n, res, err, out, cap, counts):
        _lib.check(self.L.kg_shard_refwd_seed(self.snapshot.handle, n, res.data_ptr(), err.data_ptr(), out.data_ptr(),
                                              cap, counts.data_ptr(), self._s()), "kg_shard_refwd_seed")

    def held_words(self) -> int:
        w = C.c_size_t(0)
        _lib.check(self.L.kg_shard_held_words(self.snapshot.handle, C.byref(w)), "kg_shard_held_words")
        return int(w.value)

    def held_export(self, words):
        import torch
        bits = torch.empty(max(words, 1), dtype=torch.int32, device="cuda")
        _lib.check(self.L.kg_shard_held(self.snapshot.handle, bits.data_ptr(), words, 0, self._s()), "kg_shard_held")
        return bits[:words]

    def held_import(self, bits):
        _lib.check(self.L.kg_shard_held(self.snapshot.handle, bits.data_ptr(), int(bits.shape[0]), 1, self._s()),
                   "kg_shard_held")

    def errors_possible(self) -> bool:
        """Some node this rank owns can end a check in an error (kg_shard_bad_nodes)."""
        c = C.c_uint64(0)
        _lib.check(self.L.kg_shard_bad_nodes(self.snapshot.handle, C.byref(c)), "kg_shard_bad_nodes")
        return c.value > 0

    def result_slots(self, n: int) -> int:
        """Result slots of a batch of n queries: n, plus the parts of formula-split queries."""
        return int(self.L.kg_shard_result_slots(self.snapshot.handle, n))

    def finish(self, n, res, err):
        _lib.check(self.L.kg_shard_finish(self.snapshot.handle, n, res.data_ptr(), err.data_ptr(), self._s()),
                   "kg_shard_finish")

    # ---- general rewrites (queries the level protocol ends as KG_ERR_NOT_IMPLEMENTED)
    def region_rows(self, objs: np.ndarray):
        """GetRelationTuples (kg_snapshot_rows) of every relation of each (ns, obj) row of `objs` that this
        rank holds, rows of each relation in shard order.  Returns (offs[m + 1], tuples (t, 6) uint32):
        object j's rows at tuples[offs[j]:offs[j + 1]]."""
        nrel = self.snapshot.interner.n_relations
        m = int(objs.shape[0])
        if m == 0:
            return np.zeros(1, np.int64), np.zeros((0, 6), np.uint32)
        keys = np.empty((m * nrel, 3), np.uint32)
        keys[:, 0] = np.repeat(objs[:, 0], nrel)
        keys[:, 1] = np.repeat(objs[:, 1], nrel)
        keys[:, 2] = np.tile(np.arange(nrel, dtype=np.uint32), m)
        off, tup = self.snapshot.rows(keys)
        return off[::nrel].copy(), tup

    def general_check(self, region: np.ndarray, q7: np.ndarray, gdepth: int):
        """The single-GPU engine (tiers + rewrite interpreter) on a snapshot of `region` -- every row the
        queries can read -- with this snapshot's namespace program.  Returns (res u8, err u32) host arrays."""
        from .engine import Config, Engine, Snapshot
        snap = Snapshot(region, self.snapshot.interner, self.snapshot.program, self.snapshot.device)
        try:
            return Engine(snap, Config(gdepth)).batch_check_ids(q7)
        finally:
            snap.close()


class GlooTransport:
    """kg_shard_transport over torch.distributed on host buffers (host_memory 1): any backend that moves
    CPU tensors (gloo).  The library's hash-sharded batch calls these from kg_check_batch(_device)
    on the calling thread; the product transport is RCCL (kg_shard_comm_init)."""

    def __init__(self, dist, rank: int, world: int, group=None):
        import torch
        self.dist, self.rank, self.world, self.group, self.torch = dist, rank, world, group, torch
        self.error = None
        L = _lib.load()
        self._fns = (_lib.ALLTOALL2_FN(self._alltoall2), _lib.ALLGATHER_FN(self._allgather),
                     _lib.ALLREDUCE_FN(self._allreduce))  # kept alive as long as the binding
        self.struct = _lib.kg_shard_transport(None, rank, world, 1, *self._fns)
        self.L = L

    def _i32(self, ptr, nbytes):
        return np.ctypeslib.as_array((C.c_int32 * (nbytes // 4)).from_address(ptr)) if nbytes else np.zeros(0, np.int32)

    def _alltoall2(self, ctx, s0, r0, b0, s1, r1, b1, stream):
        try:
            N = self.world
            for s, r, b in ((s0, r0, b0), (s1, r1, b1)):
                if not b:
                    continue
                src = self.torch.from_numpy(self._i32(s, N * b).copy())
                dst = self.torch.empty(N * b // 4, dtype=self.torch.int32)
                self.dist.all_to_all_single(dst, src, group=self.group)
                self._i32(r, N * b)[:] = dst.numpy()
            return 0
        except Exception as x:  # noqa: BLE001 -- a C callback must not raise
            self.error = x
            return 1

    def _allgather(self, ctx, s, r, nbytes, stream):
        try:
            src = self.torch.from_numpy(self._i32(s, nbytes).copy())
            dst = self.torch.empty(self.world * (nbytes // 4), dtype=self.torch.int32)
            self.dist.all_gather_into_tensor(dst, src, group=self.group)
            self._i32(r, self.world * nbytes)[:] = dst.numpy()
            return 0
        except Exception as x:  # noqa: BLE001
            self.error = x
            return 1

    def _allreduce(self, ctx, buf, count, stream):
        try:
            a = np.ctypeslib.as_array(buf, shape=(count,))
            # unsigned max as a signed one: flipping bit 63 maps u64 order onto i64 order (the remote
            # child metadata words use all 64 bits)
            top = np.uint64(1 << 63)
            t = self.torch.from_numpy((a ^ top).view(np.int64).copy())
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
            a[:] = t.numpy().view(np.uint64) ^ top
            return 0
        except Exception as x:  # noqa: BLE001
            self.error = x
            return 1


class LibShardedChecker:
    """One rank's side of hash-sharded batches run INSIDE libketogpu.so (kg_shard_comm.hip): seed, the
    gdepth + 1 levels with their exchanges, finish and the general phase are all one
    kg_check_batch_device call, as a Go host makes it.  transport "rccl" (default):
    an RCCL communicator bound to this checker's stream, its unique id broadcast over `dist` (or made
    locally at world 1); "host": GlooTransport callbacks over `dist` (CPU tensors; two ranks may share
    one GPU, which RCCL does not allow)."""

    def __init__(self, snapshot, rank: int = 0, world: int = 1, dist=None, group=None, transport: str = "rccl",
                 stream=None, snapshot_stream: bool = False):
        """snapshot_stream: bind the snapshot's own stream (what kg_check_batch with host buffers and
        kg_expand_batch use -- sharded expand goes through it) instead of a torch stream of this checker."""
        import torch
        self.snapshot, self.rank, self.world = snapshot, rank, world
        self.L = _lib.load()
        self.snapshot_stream = snapshot_stream
        self.stream = None if snapshot_stream else (stream if stream is not None else torch.cuda.Stream())
        self._sp = C.c_void_p(None if snapshot_stream else self.stream.cuda_stream)
        self.transport = transport
        if transport == "rccl":
            uid = (C.c_uint8 * _lib.KG_SHARD_UNIQUE_ID_BYTES)()
            if rank == 0:
                _lib.check(self.L.kg_shard_unique_id(uid), "kg_shard_unique_id")
            if world > 1:
                t = torch.tensor(bytearray(uid), dtype=torch.uint8)
                if dist.get_backend(group) == "nccl":
                    t = t.cuda()
                dist.broadcast(t, 0, group=group)
                C.memmove(uid, bytes(t.cpu().numpy().tobytes()), _lib.KG_SHARD_UNIQUE_ID_BYTES)
            _lib.check(self.L.kg_shard_comm_init(snapshot.handle, uid, rank, world, self._sp), "kg_shard_comm_init")
            self._t = None
        elif transport == "host":
            self._t = GlooTransport(dist, rank, world, group)
            self._check_t(self.L.kg_shard_transport_attach(snapshot.handle, C.byref(self._t.struct), self._sp),
                          "kg_shard_transport_attach")
        else:
            raise ValueError("transport must be 'rccl' or 'host'")

    def _check_t(self, rc, what):
        if rc != 0 and self._t is not None and self._t.error is not None:
            raise _lib.KetoGPUError(f"{what}: transport callback failed: {self._t.error!r}")
        _lib.check(rc, what)

    def check(self, dq, gdepth: int, res=None, err=None):
        """dq: (n, 7) int32 kg_query rows of THIS rank's queries (device tensor).  Returns (res u8, err i32)
        device tensors, ordered after the caller's current stream's work; `res` / `err` (>= n u8 / i32 device
        tensors) are written in place when given."""
        import torch
        n = int(dq.shape[0])
        if res is None:
            res = torch.empty(max(n, 1), dtype=torch.uint8, device=dq.device)
        if err is None:
            err = torch.empty(max(n, 1), dtype=torch.int32, device=dq.device)
        assert res.numel() >= n and err.numel() >= n and res.dtype == torch.uint8 and err.dtype == torch.int32
        if self.snapshot_stream:  # the library's own stream: order through the device
            torch.cuda.synchronize()
        else:
            self.stream.wait_stream(torch.cuda.current_stream())
        self._check_t(self.L.kg_check_batch_device(self.snapshot.handle, dq.data_ptr() if n else None, n, gdepth,
                                                   res.data_ptr(), err.data_ptr(), None, self._sp),
                      "kg_check_batch_device (sharded)")
        if self.snapshot_stream:
            torch.cuda.synchronize()
        else:
            torch.cuda.current_stream().wait_stream(self.stream)
        return res[:n], err[:n]

    def expand(self, roots: np.ndarray, gdepth: int):
        """BuildTree for this rank's roots ((n, 4) uint32 kg_set rows) on the sharded snapshot
        (collective: every rank calls it; needs snapshot_stream=True).  Per root the pre-order records or
        None, as ExpandEngine.build_trees_ids."""
        from .engine import Config, ExpandEngine
        if not self.snapshot_stream:
            raise ValueError("sharded expand runs on the snapshot's own stream (snapshot_stream=True)")
        return ExpandEngine(self.snapshot, Config(gdepth)).build_trees_ids(roots)

    STAT_KEYS = ("levels", "records_sent", "host_syncs", "reruns_bucket", "reruns_visited", "general_queries",
                 "general_rows", "bucket", "records_to_peers", "wire_bytes", "path", "exchanges", "escalation_levels",
                 "exchange_reruns")
    PATHS = {0: "local-first (replica tier chain)", 1: "one-rank device level loop", 2: "exchange protocol"}

    def stats(self) -> dict:
        """kg_shard_comm_stats_ex of the last batch (include/ketogpu.h)."""
        out = (C.c_uint64 * 16)()
        _lib.check(self.L.kg_shard_comm_stats_ex(self.snapshot.handle, self._sp, out, 16), "kg_shard_comm_stats_ex")
        return dict(zip(self.STAT_KEYS, (int(x) for x in out)))

    def levels(self) -> list:
        """Per exchange of the last batch: (B_k records per destination, largest bucket)."""
        out = (C.c_uint64 * 256)()
        n = int(self.L.kg_shard_comm_levels(self.snapshot.handle, self._sp, out, 256))
        if n < 0:
            _lib.check(n, "kg_shard_comm_levels")
        return [(int(out[2 * k]), int(out[2 * k + 1])) for k in range(min(n, 128))]

    def close(self):
        if self.snapshot.handle:
            self.L.kg_shard_comm_release(self.snapshot.handle, self._sp)


KG_SUBJECT_ID = 0xFFFFFFFF
ERR_NOT_IMPLEMENTED = 2


def shard_owners(ns: np.ndarray, obj: np.ndarray, nranks: int) -> np.ndarray:
    """kg_shard_owner (kg_internal.h shard_owner) over arrays: hash(ns, obj) mod nranks."""
    ns = np.asarray(ns, np.uint64)
    obj = np.asarray(obj, np.uint64)
    if nranks <= 1:
        return np.zeros(ns.shape, np.int64)
    with np.errstate(over="ignore"):
        x = (ns << np.uint64(32)) | obj
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xbf58476d1ce4e5b9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94d049bb133111eb)
        x ^= x >> np.uint64(31)
    return ((x >> np.uint64(20)) % np.uint64(nranks)).astype(np.int64)


class ShardOverflow(Exception):
    """Some rank dropped records: 1 = a bucket, 2 = its visited table.  Every rank reruns."""

    def __init__(self, flags: int):
        super().__init__(flags)
        self.flags = flags


class ShardedChecker:
    """Drives one rank's side of a sharded batch.  dist = torch.distributed (initialised) or None
    for a single rank; device = the torch device the records live on."""

    def __init__(self, ops, rank: int = 0, world: int = 1, dist=None, device="cuda", cap: int = 1 << 20,
                 protocol: str = "auto", group=None, general: bool = True):
        """protocol (world > 1): "fixed" = every level exchanges fixed-size buckets (records per destination
        <= bucket) and the batch runs gdepth + 1 levels with no host round trip inside it (counts, flags and
        termination stay on the device; one readback at the end); "dynamic" = one metadata exchange and
        host round trip per level, buckets sized by the real counts, early termination; "auto" = fixed
        when the ops support it and no backward escalation phase is enabled."""
        if world > _lib.KG_SHARD_MAX_RANKS:
            raise ValueError("at most %d ranks" % _lib.KG_SHARD_MAX_RANKS)
        self.ops, self.rank, self.world, self.dist, self.device, self.cap = ops, rank, world, dist, device, cap
        self.protocol = protocol
        # process group of this checker's collectives (None: the default group).  Batches in flight at
        # once on one rank each need their own group (and ops on their own stream): collectives of
        # one group are matched across ranks in issue order
        self.group = group
        self.bucket = None  # fixed protocol: records per destination per level (learned per batch)
        self.levels = 0
        self.records_sent = 0
        self.host_syncs = 0
        self._held_ready = world == 1 or not hasattr(ops, "held_export")
        self.trace = bool(int(os.environ.get("KG_SHARD_TRACE", "0")))  # per-level record counts (diagnostics)
        self.level_records = None
        # general rewrites: queries the level protocol ends as NOT_IMPLEMENTED are answered by the
        # single-GPU engine on a snapshot of the rows they can read, gathered to their home rank
        self.general = bool(general) and hasattr(ops, "general_check")
        self._gen_any = False
        # the done bitmap drops a member query's records; with errors possible anywhere it must not
        # (an error in an earlier branch wins over a member found at a shallower level in a later one:
        # the reference's first-decisive order), so it is on only when no rank has a node that errors
        self._prune = None
        self.general_queries = 0
        self.general_rows = 0
        self.reruns = {1: 0, 2: 0}  # batches rerun after a bucket (1) / visited-table (2) overflow

    def _install_held(self):
        """Once per snapshot: the OR of every rank's holder bitmap, so kg_shard_seed's no-holder test
        sees all rows (an all-reduce of the word count, an all-gather of the bitmaps)."""
        import torch
        dev = self.device if not self._host_staged() else "cpu"
        w = torch.tensor([self.ops.held_words()], dtype=torch.int64, device=dev)
        self.dist.all_reduce(w, op=self.dist.ReduceOp.MAX, group=self.group)
        words = int(w.item())
        mine = self.ops.held_export(words)
        if self._host_staged():
            mine = mine.cpu()
        allb = [torch.empty(words, dtype=torch.int32, device=mine.device) for _ in range(self.world)]
        self.dist.all_gather(allb, mine.contiguous(), group=self.group)
        acc = allb[0].clone()
        for r in range(1, self.world):
            acc |= allb[r]
        self.ops.held_import(acc.to(self.device))
        self._held_ready = True

    def _done(self, res, n, words, err=None, mode=1):
        """The batch's done bitmap for the next level: every rank's packed results (err given:
        queries escalated out of the phase too), all-gathered."""
        import torch
        mine = self.ops.done_bits(res, n, words, err, mode) if err is not None else self.ops.done_bits(res, n, words)
        if self.dist is None or self.world == 1:
            return mine
        staged = self._host_staged()
        if staged:
            mine = mine.cpu()
        parts = [torch.empty(words, dtype=torch.int32, device=mine.device) for _ in range(self.world)]
        self.dist.all_gather(parts, mine.contiguous(), group=self.group)
        allb = torch.cat(parts)
        return allb.to(self.device) if staged else allb

    # ---- exchange
    def _host_staged(self) -> bool:
        return self.dist is not None and self.dist.get_backend() == "gloo" and str(self.device).startswith("cuda")

    def _meta_exchange(self, counts):
        """One all-to-all of per-destination metadata, then ONE device->host copy for the level.

        Rank r sends every destination d the triple (records for d, records r sends in total, r's
        overflow flags); so each rank learns its receive sizes, the global record total (termination:
        nothing sent anywhere) and every rank's flags (all ranks rerun together on overflow).
        Returns (send_splits, recv_splits, global_total, flags) as host ints."""
        import torch
        N, cap = self.world, self.cap
        if self._host_staged():
            counts = counts.cpu()  # gloo moves host tensors: stage here (the one host copy of the level)
        c = counts.to(torch.int64)
        myflags = c[N] | (c[:N] > cap).any().to(torch.int64)  # a count past cap = dropped records
        nq = torch.full((N,), self._n, dtype=torch.int64, device=c.device)
        meta = torch.stack([c[:N], c[:N].sum().expand(N), myflags.expand(N), nq], dim=1).contiguous()
        recv = torch.empty_like(meta)
        if self.dist is None:
            recv.copy_(meta)
        else:
            self.dist.all_to_all_single(recv, meta, group=self.group)
        h = torch.cat([c[:N], recv.flatten()]).cpu().numpy()  # the level's host round trip
        self.host_syncs += 1
        send = [int(x) for x in h[:N]]
        rm = h[N:].reshape(N, 4)
        flags = 0
        for f in rm[:, 2]:
            flags |= int(f)
        self._n_max = int(rm[:, 3].max())  # the largest batch of any rank: sizes the done bitmap
        return send, [int(x) for x in rm[:, 0]], int(rm[:, 1].sum()), flags

    def _exchange(self, out, send_splits, recv_splits):
        import torch
        cap = self.cap
        if self.dist is None:
            return out[:send_splits[0]]
        send = torch.cat([out[d * cap: d * cap + send_splits[d]] for d in range(self.world)])
        staged = self._host_staged()
        if staged:
            send = send.cpu()
        recv = torch.empty((sum(recv_splits), REC_WORDS), dtype=torch.int32, device=send.device)
        self.dist.all_to_all_single(recv, send, recv_splits, send_splits, group=self.group)
        return recv.to(self.device) if staged else recv

    def _all_gather_rows(self, t, n: int, flags: int):
        """All-gather the first n rows of int32 tensor t from every rank (variable counts, padded to the
        largest) with every rank's flags; returns (concatenated rows on self.device, OR of the flags)."""
        import torch
        if self.dist is None:
            return t[:0 if flags else n], flags
        staged = self._host_staged()
        meta = torch.tensor([n, flags], dtype=torch.int64, device="cpu" if staged else self.device)
        metas = [torch.empty_like(meta) for _ in range(self.world)]
        self.dist.all_gather(metas, meta, group=self.group)
        h = torch.stack(metas).cpu().numpy()
        self.host_syncs += 1
        sizes = [int(x) for x in h[:, 0]]
        fl = 0
        for f in h[:, 1]:
            fl |= int(f)
        mx = max(sizes)
        if mx == 0 or fl:
            return t[:0], fl
        mine = torch.zeros((mx, t.shape[1]), dtype=t.dtype, device=t.device)
        mine[:n] = t[:n]
        if staged:
            mine = mine.cpu()
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        self.dist.all_gather(parts, mine, group=self.group)
        allr = torch.cat([parts[r][:sizes[r]] for r in range(self.world)])
        return (allr.to(self.device) if staged else allr), 0

    def _backward(self, res, err, slots: int, gdepth: int):
        """The backward phase of the escalated queries (kg_shard_back_*): level 0 = every rank's holders of
        their subjects, then reverse hops over all-gathered records until no rank emits any."""
        import torch
        cap = self.cap
        lst = torch.empty((cap, REC_WORDS), dtype=torch.int32, device=self.device)
        cl = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.ops.back_list(slots, res, err, lst, cap, cl)
        bufs = [torch.empty((cap, REC_WORDS), dtype=torch.int32, device=self.device) for _ in range(2)]
        cb = [torch.zeros(2, dtype=torch.int32, device=self.device) for _ in range(2)]
        words = (slots + 31) // 32
        if self.world == 1 and self.dist is None and getattr(self.ops, "device_counts", False):
            # one rank: no gathers; a level lowers the rest depth by one, so gdepth levels drain it
            self.ops.back_seed(lst, cap, cl, bufs[0], cap, cb[0])
            cur = 0
            for _ in range(gdepth):
                done = self.ops.done_bits(res, slots, words, err, 2)
                self.ops.back_level(bufs[cur], cap, cb[cur], bufs[cur ^ 1], cap, cb[cur ^ 1], res, err, done, words)
                cur ^= 1
                self.back_levels += 1
            return torch.stack([cl[1] | cb[0][1] | cb[1][1], cb[cur][0]])  # (flags, records left): read by the caller
        h = torch.stack([cl[0], cl[1]]).cpu().numpy()
        self.host_syncs += 1
        glist, fl = self._all_gather_rows(lst, min(int(h[0]), cap), int(h[1]) | (int(h[0]) > cap))
        if fl:
            raise ShardOverflow(fl)
        if glist.shape[0] == 0:
            return None
        self.ops.back_seed(glist, int(glist.shape[0]), None, bufs[0], cap, cb[0])
        cur = 0
        while True:
            h = cb[cur].cpu().numpy()
            self.host_syncs += 1
            n_loc = int(h[0])
            recs, fl = self._all_gather_rows(bufs[cur], min(n_loc, cap), int(h[1]) | (n_loc > cap))
            if fl:
                raise ShardOverflow(fl)
            if recs.shape[0] == 0:
                return None
            wmax = (self._n_max + 31) // 32
            done = self._done(res, slots, wmax, err, 2)
            cb[cur ^ 1].zero_()
            self.ops.back_level(recs, int(recs.shape[0]), None, bufs[cur ^ 1], cap, cb[cur ^ 1], res, err, done, wmax)
            cur ^= 1
            self.back_levels += 1

    def _pruning(self) -> bool:
        """Whether the done bitmap may drop member queries' records: no rank can end a check in an error
        below its root (kg_shard_bad_nodes; asked once, all-reduced)."""
        if self._prune is None:
            if self.dist is not None and self.world > 1:
                self._max_slots(self._n)  # its one-time all-reduce carries the flag
            else:
                mine = bool(self.ops.errors_possible()) if hasattr(self.ops, "errors_possible") else False
                self._prune = hasattr(self.ops, "done_bits") and not mine
        return self._prune

    def _device_levels(self, bufs, counts, cur, res, err, slots, gdepth, words, esc_mode, trace, final=False):
        """One rank: gdepth forward levels enqueued back to back, record counts read on the device
        (esc_mode 1: escalated queries are done for the done bitmap; final: the batch's final forward
        phase, counted apart).  Returns the current buffer."""
        cap = self.cap
        prune = self._pruning()
        if trace is None and hasattr(self.ops, "done_bits") and hasattr(self.ops, "levels"):  # one library call
            if not final:
                self.levels += gdepth
            return self.ops.levels(gdepth, bufs, cap, counts, cur, res, err, slots if prune else 0, esc_mode)
        for k in range(gdepth):
            c = counts[cur]
            if trace is not None:  # diagnostics: records entering each level (a host sync per level)
                trace.append(int(c[0].item()))
            done = None
            if prune and k > 0:
                done = (self.ops.done_bits(res, slots, words, err, esc_mode) if esc_mode
                        else self.ops.done_bits(res, slots, words))
            self.ops.level(bufs[cur], cap, c, bufs[cur ^ 1], cap, counts[cur ^ 1], res, err, done, words)
            cur ^= 1
            if not final:
                self.levels += 1
        return cur

    # ---- general rewrites across shards
    def _open_general(self, res, err, n):
        """Device flag: some query of this rank ended KG_ERROR / NOT_IMPLEMENTED (after kg_shard_finish)."""
        import torch
        return ((res[:n] == 2) & (err[:n] == ERR_NOT_IMPLEMENTED)).any().to(torch.int64)

    def _xdev(self):
        return "cpu" if self.dist is None or self.dist.get_backend() == "gloo" else self.device

    def _any_rank(self, flag: bool) -> bool:
        import torch
        if self.dist is None or self.world == 1:
            return bool(flag)
        t = torch.tensor([1 if flag else 0], dtype=torch.int64, device=self._xdev())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        self.host_syncs += 1
        return bool(int(t.item()))

    def _a2a_rows(self, rows: np.ndarray, dest: np.ndarray) -> np.ndarray:
        """All-to-all of int64 host rows: row i goes to rank dest[i]; returns the rows this rank received."""
        import torch
        if self.dist is None or self.world == 1:
            return rows
        N = self.world
        order = np.argsort(dest, kind="stable")
        rows = np.ascontiguousarray(rows[order])
        send = np.bincount(dest, minlength=N).astype(np.int64)
        dev = self._xdev()
        rc = torch.empty(N, dtype=torch.int64, device=dev)
        self.dist.all_to_all_single(rc, torch.from_numpy(send).to(dev), group=self.group)
        recv_n = [int(x) for x in rc.cpu().numpy()]
        w = rows.shape[1]
        out = torch.empty((sum(recv_n), w), dtype=torch.int64, device=dev)
        self.dist.all_to_all_single(out, torch.from_numpy(rows).to(dev), recv_n, [int(x) for x in send],
                                    group=self.group)
        self.host_syncs += 1
        return out.cpu().numpy()

    def _gather_region(self, q: np.ndarray, gdepth: int) -> np.ndarray:
        """Every row of every object within gdepth + 1 subject-set hops of this rank's queries' root objects,
        gathered at this rank (collective: every rank takes part, with or without queries).  Hop h+1 =
        the objects of the subject sets in hop h's rows: the objects an expand row or a tuple-to-subject-set
        row leads to (rewrites.go:205-260); computed subject sets stay on the object, and the owner ships
        all of an object's relations (every relation of an object lives on one rank).  Owners ship an
        object once per home; rows keep their shard order per (ns, obj, rel)."""
        N = self.world
        req = np.unique(np.stack([np.full(q.shape[0], self.rank, np.int64), q[:, 0].astype(np.int64),
                                  q[:, 1].astype(np.int64)], 1), axis=0) if q.shape[0] else np.zeros((0, 3), np.int64)
        seen = set()
        got_rows = []
        for hop in range(gdepth + 2):
            recv = self._a2a_rows(req, shard_owners(req[:, 1], req[:, 2], N))
            keep = []
            for i, (h, ns, obj) in enumerate(recv.tolist()):
                if (h, ns, obj) not in seen:
                    seen.add((h, ns, obj))
                    keep.append(i)
            new = recv[keep] if keep else np.zeros((0, 3), np.int64)
            off, tup = self.ops.region_rows(new[:, 1:3].astype(np.uint32))
            homes = np.repeat(new[:, 0], np.diff(off).astype(np.int64))
            payload = np.concatenate([homes[:, None], tup.astype(np.int64)], 1)
            got_rows.append(self._a2a_rows(payload, homes))
            sets = tup[:, 3] != KG_SUBJECT_ID
            if hop <= gdepth and sets.any():
                req = np.unique(np.stack([homes[sets], tup[sets, 3].astype(np.int64), tup[sets, 4].astype(np.int64)],
                                         1), axis=0)
            else:
                req = np.zeros((0, 3), np.int64)
            if not self._any_rank(req.shape[0] > 0):
                break
        allr = np.concatenate(got_rows) if got_rows else np.zeros((0, 7), np.int64)
        return np.ascontiguousarray(allr[:, 1:7].astype(np.uint32))

    def _general_phase(self, dq, res, err, gdepth: int):
        """Queries that reached a rewrite the level protocol cannot evaluate across ranks (an impure union,
        a recursive formula through tuple-to-subject-set, an undeclared relation): their rows are gathered
        to their home rank and the single-GPU engine answers them there (rewrite interpreter included),
        so the sharded mode returns the reference's answers and errors for every program."""
        import torch
        n = int(dq.shape[0])
        sel = ((res[:n] == 2) & (err[:n] == ERR_NOT_IMPLEMENTED)).nonzero().flatten()
        q = dq[sel].cpu().numpy().view(np.uint32).reshape(-1, 7) if sel.numel() else np.zeros((0, 7), np.uint32)
        region = self._gather_region(q, gdepth)
        self.general_queries += int(q.shape[0])
        self.general_rows += int(region.shape[0])
        if q.shape[0]:
            r, e = self.ops.general_check(region, q, gdepth)
            res[sel] = torch.from_numpy(np.asarray(r, np.uint8)).to(res.device)
            err[sel] = torch.from_numpy(np.asarray(e, np.uint32).view(np.int32)).to(err.device)

    # ---- one batch
    def check(self, dq, gdepth: int) -> Tuple["object", "object"]:
        """dq: (n, 7) int32 kg_query rows of THIS rank's queries (device tensor).  Returns (res u8, err i32)
        device tensors: res 0 NotMember / 1 IsMember / 2 error (err = KG_ERR_*)."""
        import torch
        ts = getattr(self.ops, "torch_stream", None)
        if ts is not None:  # the local steps and every torch op of the batch run on the ops' stream
            ts.wait_stream(torch.cuda.current_stream())
        gd = gdepth if gdepth >= 1 else 5
        while True:
            try:
                self._gen_any = False
                if ts is None:
                    res, err = self._check(dq, gdepth)
                    if self._gen_any:
                        self._general_phase(dq, res, err, gd)
                    return res, err
                with torch.cuda.stream(ts):
                    res, err = self._check(dq, gdepth)
                    if self._gen_any:
                        self._general_phase(dq, res, err, gd)
                torch.cuda.current_stream().wait_stream(ts)
                return res, err
            except ShardOverflow as e:  # every rank saw the same flags: all rerun with more room
                for f in (1, 2):
                    self.reruns[f] += 1 if e.flags & f else 0
                if e.flags & 1:
                    self.cap *= 2
                if e.flags & 2:
                    if not hasattr(self.ops, "grow_visited"):
                        raise _lib.KetoGPUError("sharded visited table overflow")
                    self.ops.grow_visited()

    def _check(self, dq, gdepth: int):
        import torch
        n = int(dq.shape[0])
        N, cap = self.world, self.cap
        gdepth = gdepth if gdepth >= 1 else 5  # config.schema.json:308-315 default (as kg_shard_seed)
        if not self._held_ready:
            self._install_held()
        # result slots: the queries, then the parts of formula-split queries (kg_shard_result_slots)
        slots = self.ops.result_slots(n) if hasattr(self.ops, "result_slots") else n
        self._n = slots
        # escalation: forward done bits carry escalated queries; backward and final forward phases follow
        backward = hasattr(self.ops, "back_level") and getattr(self.ops, "escalates", True)
        self.back_levels = self.final_levels = 0
        fixed = self.dist is not None and hasattr(self.ops, "level_seg") and \
            (self.protocol == "fixed" or (self.protocol == "auto" and not backward))
        if fixed:  # decided before any buffer or seed of the other protocols
            if backward:
                raise ValueError("the fixed-bucket protocol has no backward escalation phase")
            res = torch.zeros(slots, dtype=torch.uint8, device=self.device)
            err = torch.zeros(slots, dtype=torch.int32, device=self.device)
            return self._check_fixed(dq, n, slots, gdepth, res, err)
        prune = self._pruning()
        final = False
        bufs = [torch.empty((N * cap, REC_WORDS), dtype=torch.int32, device=self.device) for _ in range(2)]
        counts = [torch.zeros(N + 1, dtype=torch.int32, device=self.device) for _ in range(2)]
        res = torch.zeros(slots, dtype=torch.uint8, device=self.device)
        err = torch.zeros(slots, dtype=torch.int32, device=self.device)
        self.ops.seed(dq, n, gdepth, bufs[0], cap, counts[0], res, err)
        cur = 0
        self.levels = 0
        self.records_sent = 0
        if N == 1 and self.dist is None and getattr(self.ops, "device_counts", False):
            # one rank: nothing to exchange, so every level is enqueued back to back with its record
            # count read on the device.  A record's depth falls by one per level and seeds carry
            # <= gdepth, so gdepth levels drain the batch; overflow is checked once at the end.
            words = (slots + 31) // 32
            trace = [] if self.trace else None
            cur = self._device_levels(bufs, counts, cur, res, err, slots, gdepth, words, 1 if backward else 0, trace)
            self.level_records = trace
            # kg_shard_level accumulates the flags word (counts[N]: a bucket or the visited table
            # overflowed) over the levels of each of the two count buffers
            parts = [counts[0][1] | counts[1][1], counts[cur][0]]
            if backward:
                parts += list(self._backward(res, err, slots, gdepth))
                # the final forward phase: queries past both budgets, from their roots, no budget
                self.ops.refwd_seed(slots, res, err, bufs[0], cap, counts[0])
                counts[1].zero_()
                self.final_levels = gdepth
                cur = self._device_levels(bufs, counts, 0, res, err, slots, gdepth, words, 0, None, final=True)
                parts += [counts[0][1] | counts[1][1], counts[cur][0]]
            if self.general:  # results final before the readback, so it also says whether any query is open
                self.ops.finish(n, res, err)
                parts.append(self._open_general(res, err, n).to(parts[0].dtype))
            h = torch.stack(parts).cpu().numpy()  # the batch's one host round trip
            self.host_syncs += 1
            if self.general:
                self._gen_any = bool(h[-1])
                h = h[:-1]
            fl = 0
            for k in range(0, len(h), 2):
                fl |= int(h[k])
            if fl & 3:  # dropped records (a bucket or the visited table): rerun before judging what is left
                raise ShardOverflow(fl & 3)
            left = [int(h[k + 1]) for k in range(0, len(h), 2)]
            if any(left):
                raise _lib.KetoGPUError("sharded batch: records left after %d levels (%s)" % (gdepth, left))
            if not self.general:
                self.ops.finish(n, res, err)
            return res[:n], err[:n]
        while True:
            send, recv_splits, total, flags = self._meta_exchange(counts[cur])
            if flags & 3:
                raise ShardOverflow(flags)
            if total == 0:
                if backward and not final:
                    self._backward(res, err, slots, gdepth)
                    # the final forward phase: queries past both budgets, re-seeded at their roots
                    self.ops.refwd_seed(slots, res, err, bufs[cur], cap, counts[cur])
                    final = True
                    continue
                self.ops.finish(n, res, err)
                if self.general:
                    self._gen_any = self._any_rank(bool(self._open_general(res, err, n).item()))
                return res[:n], err[:n]
            self.records_sent += sum(send)
            recv = self._exchange(bufs[cur], send, recv_splits)
            words = (self._n_max + 31) // 32
            done = None
            if prune and self.levels > 0:
                done = self._done(res, slots, words, err if backward and not final else None)
            if final:
                self.final_levels += 1
                self.levels -= 1  # counted apart
            cur ^= 1
            self.ops.level(recv, int(recv.shape[0]), None, bufs[cur], cap, counts[cur], res, err, done, words)
            self.levels += 1

    # ---- fixed-bucket protocol (world > 1): no host round trip inside a batch
    def _max_slots(self, slots: int) -> int:
        """The largest result-slot count of any rank (it sizes the done bitmap and the first bucket, which
        every rank must agree on): one small all-reduce on EVERY batch.  Ranks' slot counts differ and
        change from batch to batch, so a per-rank cache would let one rank skip the collective another
        rank issues (a mismatched collective).  The same all-reduce carries "some rank can
        end a check in an error" (_pruning), this rank's part of which is asked once."""
        import torch
        if not hasattr(self, "_errors_mine"):
            self._errors_mine = bool(self.ops.errors_possible()) if hasattr(self.ops, "errors_possible") else False
        t = torch.tensor([slots, int(self._errors_mine)], dtype=torch.int64,
                         device="cpu" if self._host_staged() else self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        self.host_syncs += 1
        h = t.cpu().numpy()
        if self._prune is None:
            self._prune = hasattr(self.ops, "done_bits") and not bool(h[1])
        return int(h[0])

    def _check_fixed(self, dq, n: int, slots: int, gdepth: int, res, err):
        """gdepth + 1 levels (a record's rest depth falls by one per level and seeds carry <= gdepth; the
        last level only delivers hit / error reports to their home ranks), each: an all-to-all of the
        per-destination counts, an all-to-all of fixed-size buckets (B records per destination), an
        all-gather of the done bitmap, and kg_shard_level_seg over the received segments.  Counts,
        overflow flags and the records-left check stay on the device; the batch reads them back once
        (all-reduced over ranks), and a bucket or visited-table overflow anywhere reruns the batch on
        every rank with room to spare (ShardOverflow)."""
        import torch
        N = self.world
        smax = self._max_slots(slots)
        words = (smax + 31) // 32
        B = self.bucket or min(self.cap, (2 * smax) // N + 1024)  # the same on every rank
        self.bucket = B
        staged = self._host_staged()
        xdev = "cpu" if staged else self.device
        bufs = [torch.empty((N * B, REC_WORDS), dtype=torch.int32, device=self.device) for _ in range(2)]
        counts = [torch.zeros(N + 1, dtype=torch.int32, device=self.device) for _ in range(2)]
        recv = torch.empty((N * B, REC_WORDS), dtype=torch.int32, device=xdev)
        rc = torch.empty(N, dtype=torch.int32, device=xdev)
        acc = torch.zeros(3, dtype=torch.int64, device=self.device)  # flags, largest bucket, records sent
        self.ops.seed(dq, n, gdepth, bufs[0], B, counts[0], res, err)
        cur = 0
        self.levels = 0
        prune = self._pruning()
        for k in range(gdepth + 1):
            c = counts[cur]
            c64 = c[:N].to(torch.int64)
            acc[0] |= c[N].to(torch.int64) | (c64 > B).any().to(torch.int64)
            acc[1] = torch.maximum(acc[1], c64.max())
            acc[2] += c64.sum()
            sc = c[:N].contiguous()
            self.dist.all_to_all_single(rc, sc.cpu() if staged else sc, group=self.group)
            snd = bufs[cur].cpu() if staged else bufs[cur]
            self.dist.all_to_all_single(recv, snd, group=self.group)
            done = None
            if prune and k > 0:
                mine = self.ops.done_bits(res, slots, words)
                parts = torch.empty(N * words, dtype=torch.int32, device=xdev)
                self.dist.all_gather_into_tensor(parts, mine.cpu() if staged else mine, group=self.group)
                done = parts.to(self.device) if staged else parts
            nxt = cur ^ 1
            self.ops.level_seg(recv.to(self.device) if staged else recv, N, B, rc.to(self.device) if staged else rc,
                               bufs[nxt], B, counts[nxt], res, err, done, words)
            cur = nxt
            self.levels += 1
        c = counts[cur]
        acc[0] |= c[N].to(torch.int64) | (c[:N].to(torch.int64) > B).any().to(torch.int64)
        left = c[:N].to(torch.int64).sum()
        if self.general:  # results final before the all-reduce, which then also carries "a query is open"
            self.ops.finish(n, res, err)
        gen = self._open_general(res, err, n) if self.general else torch.zeros((), dtype=torch.int64,
                                                                                   device=self.device)
        # over ranks: each flag bit (bucket / visited-table overflow), the largest bucket, records left, open
        tot = torch.stack([acc[0] & 1, (acc[0] >> 1) & 1, acc[1], left, gen]).to(xdev)
        self.dist.all_reduce(tot, op=self.dist.ReduceOp.MAX, group=self.group)
        h = torch.cat([tot, acc[2:3].to(xdev)]).cpu().numpy()  # the batch's one host round trip
        self.host_syncs += 1
        flags = int(h[0]) | (int(h[1]) << 1)
        self._gen_any = bool(h[4])
        self.records_sent = int(h[5])
        big = int(h[2])
        if flags & 3:
            if flags & 1:
                self.reruns[1] += 1
                self.bucket = max(2 * B, int(big * 1.25) + 1024)
                self.cap = max(self.cap, self.bucket)
            raise ShardOverflow(flags & 2)  # a bucket overflow is handled here (bigger buckets); 2 = visited
        if int(h[3]) != 0:
            raise _lib.KetoGPUError("sharded batch: records left after %d levels" % (gdepth + 1))
        # next batch: buckets 25 % above the largest one this batch needed (shrinking slowly)
        self.bucket = max(1024, min(B, int(big * 1.25) + 1024)) if big * 2 < B else B
        if not self.general:
            self.ops.finish(n, res, err)
        return res[:n], err[:n]
