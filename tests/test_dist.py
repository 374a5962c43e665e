"""Multi-rank path on CPU (gloo, world_size 2): bench.py's replica aggregation (max elapsed over
ranks, summed edges) -- the only cross-rank exchange of the replica mode."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed, edges = bench.aggregate(dist, elapsed=1.0 + rank, edges=10.0 * (rank + 1))
    q.put((rank, elapsed, edges))
    dist.destroy_process_group()


def test_replica_aggregation_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=10) for _ in range(2))
    assert got == [(0, 2.0, 30.0), (1, 2.0, 30.0)]


def test_single_rank_passthrough():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.aggregate(None, 3.5, 7.0) == (3.5, 7.0)


def test_bench_spawns_ranks_without_launcher():
    """`bench.py --gpus 3` with no WORLD_SIZE in the environment starts 3 ranks itself (the parent never
    touches a GPU) and forwards rank 0's whole-job line: n_gpus 3, work summed over the 3 ranks."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--mode", "rehearse",
                        "--steps", "5", "--batch", "100"], env=env, capture_output=True, timeout=180)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == 3 and line["config"]["parallelism"] == "replica3"
    assert line["units"] == 3 * 5 * 100


def _max_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import ctypes
    import numpy as np
    import torch.distributed as dist
    from keto_amd.sharded import GlooTransport
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = GlooTransport(dist, rank, world)
    # the remote child metadata words use all 64 bits: one rank holds a value >= 2^63, the other 0
    vals = [[0, 5, 1 << 63, (1 << 64) - 1], [(1 << 63) | 7, 3, 0, 1]][rank]
    a = np.array(vals, dtype=np.uint64)
    rc = t._allreduce(None, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(vals), None)
    q.put((rank, rc, [int(x) for x in a]))
    dist.destroy_process_group()


def test_gloo_transport_allreduce_is_unsigned_max():
    """kg_shard_transport.allreduce_max_u64 is an unsigned max (include/ketogpu.h); the gloo transport
    used to reduce as int64, which drops any word with bit 63 set."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_max_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    want = [(1 << 63) | 7, 5, 1 << 63, (1 << 64) - 1]
    assert sorted(q.get(timeout=10) for _ in range(2)) == [(0, 0, want), (1, 0, want)]
