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
          "nccl" backend; staged through host memory with gloo) after an all-gather of the
          N x N bucket sizes, which also carries termination (nothing sent anywhere) and
          overflow (every rank reruns the batch with larger buckets)

Results are those of the single-GPU engine (bounded reachability over rewrite-free nodes,
internal/check/engine.go:87-207 with the SURVEY.md 8a semantics).  The local steps are
`ShardOps` objects: `HipShardOps` runs them on the GPU through the C ABI; the multi-rank CPU
tests substitute a test-only restatement to exercise this exchange protocol under gloo.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np

from . import _lib

REC_WORDS = 4  # kg_frec = (q, node, subj, depth) as int32


class HipShardOps:
    """The local steps of one rank on its GPU (kg_shard_seed / kg_shard_level)."""

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
        self.vis_log2 = getattr(self, "vis_log2", 25) + 1
        self.snapshot.tune("shard_vis", self.vis_log2)

    def level(self, din, n_in, out, cap, counts, res):
        _lib.check(self.L.kg_shard_level(self.snapshot.handle, din.data_ptr() if n_in else None, n_in,
                                         out.data_ptr(), cap, counts.data_ptr(), res.data_ptr(), self._s()),
                   "kg_shard_level")


class ShardOverflow(Exception):
    """Some rank dropped records: 1 = a bucket, 2 = its visited table.  Every rank reruns."""

    def __init__(self, flags: int):
        super().__init__(flags)
        self.flags = flags


class ShardedChecker:
    """Drives one rank's side of a sharded batch.  dist = torch.distributed (initialised) or None
    for a single rank; device = the torch device the records live on."""

    def __init__(self, ops, rank: int = 0, world: int = 1, dist=None, device="cuda", cap: int = 1 << 20):
        if world > _lib.KG_SHARD_MAX_RANKS:
            raise ValueError("at most %d ranks" % _lib.KG_SHARD_MAX_RANKS)
        self.ops, self.rank, self.world, self.dist, self.device, self.cap = ops, rank, world, dist, device, cap
        self.levels = 0
        self.records_sent = 0

    # ---- exchange
    def _host_staged(self) -> bool:
        return self.dist is not None and self.dist.get_backend() == "gloo" and str(self.device).startswith("cuda")

    def _gather_counts(self, counts_h: np.ndarray):
        """All-gather of every rank's (bucket sizes..., flags) -> (N x N matrix, OR of flags)."""
        import torch
        if self.dist is None:
            return counts_h[None, :self.world].astype(np.int64), int(counts_h[self.world])
        dev = "cpu" if self._host_staged() or not str(self.device).startswith("cuda") else self.device
        t = torch.as_tensor(counts_h.astype(np.int64), device=dev)
        parts = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        m = torch.stack(parts).cpu().numpy()
        flags = 0
        for f in m[:, self.world]:
            flags |= int(f)
        return m[:, :self.world], flags

    def _exchange(self, out, counts_h: np.ndarray, m: np.ndarray):
        import torch
        cap = self.cap
        if self.world == 1:
            return out[:int(counts_h[0])]
        send_splits = [int(x) for x in m[self.rank]]
        recv_splits = [int(x) for x in m[:, self.rank]]
        send = torch.cat([out[d * cap: d * cap + send_splits[d]] for d in range(self.world)])
        staged = self._host_staged()
        if staged:
            send = send.cpu()
        recv = torch.empty((sum(recv_splits), REC_WORDS), dtype=torch.int32, device=send.device)
        self.dist.all_to_all_single(recv, send, recv_splits, send_splits)
        return recv.to(self.device) if staged else recv

    # ---- one batch
    def check(self, dq, gdepth: int) -> Tuple["object", "object"]:
        """dq: (n, 7) int32 kg_query rows of THIS rank's queries (device tensor).  Returns (res u8, err i32)
        device tensors: res 0 NotMember / 1 IsMember / 2 error (err = KG_ERR_*)."""
        import torch
        ts = getattr(self.ops, "torch_stream", None)
        if ts is not None:  # the local steps and every torch op of the batch run on the ops' stream
            ts.wait_stream(torch.cuda.current_stream())
        while True:
            try:
                if ts is None:
                    return self._check(dq, gdepth)
                with torch.cuda.stream(ts):
                    res, err = self._check(dq, gdepth)
                torch.cuda.current_stream().wait_stream(ts)
                return res, err
            except ShardOverflow as e:  # every rank saw the same flags: all rerun with more room
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
        bufs = [torch.empty((N * cap, REC_WORDS), dtype=torch.int32, device=self.device) for _ in range(2)]
        counts = torch.zeros(N + 1, dtype=torch.int32, device=self.device)
        res = torch.zeros(n, dtype=torch.uint8, device=self.device)
        err = torch.zeros(n, dtype=torch.int32, device=self.device)
        self.ops.seed(dq, n, gdepth, bufs[0], cap, counts, res, err)
        cur = 0
        self.levels = 0
        self.records_sent = 0
        while True:
            counts_h = counts.cpu().numpy().view(np.uint32).astype(np.int64)
            counts_h[N] |= int((counts_h[:N] > cap).any())  # a count past cap = dropped records
            m, flags = self._gather_counts(counts_h)
            if flags & 3:
                raise ShardOverflow(flags)
            if int(m.sum()) == 0:
                return res, err
            self.records_sent += int(m[self.rank].sum())
            recv = self._exchange(bufs[cur], counts_h, m)
            cur ^= 1
            self.ops.level(recv, int(recv.shape[0]), bufs[cur], cap, counts, res)
            self.levels += 1
