"""bench.py -- batched permission checks/s on MI355X (one process per GPU, snapshot replicas).

Workload (BASELINE.json metric "permission checks/sec + GTEPS @1B tuples"): the synthetic
Drive-like tuple graph (SURVEY.md 8d, C2/C4 generator; 8 layered group levels, power-law
out-degrees, Zipf-ish popularity, seed 20250131) generated directly in HBM, and per GPU a
1,000,000-check batch of doc#viewer@user queries (50% positive by random walks, 50% uniform,
max_depth drawn from {0 (global), 1..10}, global max_read_depth 10).  A "step" is one
kg_check_batch_device call over the whole batch (queries resident in HBM).  By default four
batches are in flight per GPU (--inflight): each on its own HIP stream with its own workspace,
driven by its own host thread, so the low-occupancy tail tiers of one batch (backward and grid
tiers) overlap the next batch's k_resolve / k_stream.  p99_batch_ms is per call, submit to done.

Multi-GPU: `torch.distributed.run --nproc-per-node N bench.py --gpus N`: each rank builds the
same snapshot on its GPU and checks its own batch (weak scaling, no data-path collective;
SURVEY.md 8e "replicas").  Timing: barrier + synchronize on both sides of exactly K steps, max
over ranks; rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import collections
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# independent random 16-B loads/s from HBM-sized tables (16-160 GiB) on one MI355X: tools/randprobe.hip,
# profiles/r2_randprobe_sizes.jsonl (~37 G/s; the line, not the byte, is the unit of a random gather)
RAND_REQ_PEAK = 37.0e9
STREAM_KERNEL = "k_stream4<8,256,2>"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--tuples", type=float, default=None,
                    help="synthetic graph size in tuples (rows actually generated; default 1e9, 1e7 for --mode refresh, "
                         "1.2e8 with --heavy-tail).  The generator's size parameter is calibrated so the snapshot "
                         "holds at least this many rows")
    ap.add_argument("--heavy-tail", action="store_true",
                    help="out-degree law P(k) ~ k^-1.5 (Pareto tail index 0.5 for docs and groups, SURVEY.md 8d) "
                         "instead of the default 1.3 / 1.1; ~40x the rows per node")
    ap.add_argument("--batch", type=int, default=None,
                    help="checks per step per GPU (default 1 M; 62,500 with --heavy-tail, its latency point: "
                         "DESIGN.md 7f)")
    ap.add_argument("--global-depth", type=int, default=10)
    ap.add_argument("--seed", type=int, default=20250131)
    ap.add_argument("--stream-ecap", type=int, default=512, help="kg_snapshot_tune stream_ecap (stream-tier edges per query, 0 = none)")
    ap.add_argument("--sharded-steps", type=int, default=20,
                    help="check mode: timed batches of the hash-sharded sub-line (the C4 engine through "
                         "kg_check_batch_device over RCCL, one shard per rank; 0 = off)")
    ap.add_argument("--sharded-warmup", type=int, default=4)
    ap.add_argument("--sharded-batch", type=int, default=4_000_000,
                    help="checks per sharded batch per rank (0: --batch).  C4 names 1-8 M; across ranks one batch "
                         "is in flight per rank, and 4 M amortises the exchanges' fixed cost: one-rank exchange "
                         "protocol 0.80 / 1.19 / 1.29 x 10^9 checks/s at 1 / 4 / 8 M (DESIGN.md 7f)")
    ap.add_argument("--expand-steps", type=int, default=100,
                    help="check mode, one rank: timed calls of the C5 expand sub-line over the headline graph (0 = off; "
                         "at least twice --expand-inflight).  100: five calls per caller thread -- a 40-call region (two "
                         "per thread, ~0.1 s) read 2.55-3.78 x 10^7 trees/s on runs of the same code")
    ap.add_argument("--expand-inflight", type=int, default=20,
                    help="check mode: kg_expand_batch_device calls in flight in the C5 sub-line (one HIP stream each; "
                         "a call's critical path is its largest root's walk on one workgroup, so calls overlap: "
                         "12 / 16 / 20 gave 2.80 / 3.34 / 3.74 x 10^7 trees/s at 32 hardware queues, "
                         "profiles/r6t_operating_points.txt; 16 / 20 / 24 beside the headline graph 3.19 / 3.70 / "
                         "3.09 x 10^7, profiles/r6z9_c5_inflight.txt)")
    ap.add_argument("--c3-steps", type=int, default=60,
                    help="check mode, one rank: timed batches of the C3 sub-line (OPL rewrites; 0 = off; 60: a ~30-ms "
                         "region -- 20 batches were ~10 ms)")
    ap.add_argument("--c3-tuples", type=float, default=1e7, help="C3 sub-line graph size (BASELINE configs[2]: 10M)")
    ap.add_argument("--c3-inflight", type=int, default=6,
                    help="C3 sub-line batches in flight: standalone 3 / 4 / 6 gave 2.01 / 1.84 / 1.97 x 10^9 checks/s at p99 "
                         "1.6 / 2.9 / 3.9 ms (profiles/r6z8_c3_inflight_ab.jsonl), but inside the default line 3 was erratic "
                         "(1.54-2.00 vs 1.98-2.05 x 10^9 at 6, profiles/r6z11_c3_subline.txt)")
    ap.add_argument("--c3-parity", type=int, default=200_000)
    ap.add_argument("--heavy-steps", type=int, default=20,
                    help="check mode, one rank: timed batches of the heavy-tail sub-line (SURVEY.md 8d's out-degree "
                         "law P(k) ~ k^-1.5 at 1.2e8 tuples, 62.5 k checks per batch, 4 in flight; a child "
                         "`bench.py --heavy-tail` run; 0 = off)")
    ap.add_argument("--heavy-parity", type=int, default=62_500, help="heavy-tail sub-line: checks compared with the oracle")
    ap.add_argument("--sharded-inflight", type=int, default=0,
                    help="sharded batches in flight per rank, each with its own communicator (0: 3 at one rank -- "
                         "4 measured 20 %% slower, 6 slower still (DESIGN.md 7f) -- and 1 across ranks: streams "
                         "share HIP's hardware queues, and collectives of different communicators queued in "
                         "different orders on different ranks can deadlock)")
    ap.add_argument("--sharded-timeout", type=float, default=300.0,
                    help="watchdog of the sharded sub-line: past it rank 0 prints the line without it")
    ap.add_argument("--shard-budget", type=int, default=0,
                    help="kg_snapshot_tune shard_budget (sharded mode: forward set edges per query and rank before "
                         "the query escalates to the backward phase; 0 = off)")
    ap.add_argument("--shard-back-budget", type=int, default=1 << 14,
                    help="kg_snapshot_tune shard_back_budget (reverse edges per query and rank before the final "
                         "forward phase takes it)")
    ap.add_argument("--shard-heavy", type=int, default=-1,
                    help="kg_snapshot_tune shard_heavy: set rows longer than this are expanded grid-wide (k_shard_heavy; "
                         "0: every expansion; -1: the library default)")
    ap.add_argument("--shard-vis", type=int, default=0,
                    help="kg_snapshot_tune shard_vis: log2 of the sharded mode's (query, node) visited table (0: library default)")
    ap.add_argument("--packed", type=int, default=0,
                    help="check mode: the headline's queries as 16-B kg_query_packed in HBM through "
                         "kg_check_batch_packed_device (k_resolve reads them itself) instead of 28-B kg_query "
                         "through kg_check_batch_device (packed by the library on the snapshot's stream, "
                         "DESIGN.md 5d)")
    ap.add_argument("--shard-remote-meta", type=int, default=1,
                    help="kg_snapshot_tune shard_remote_meta (N > 1: owners' row length + signature of remote "
                         "children in adjx at bind time, so remote leaves that cannot hit are never sent)")
    ap.add_argument("--stream-steal", type=int, default=4,
                    help="kg_snapshot_tune stream_steal (XCD ranges a k_stream4 wave dequeues from, 1..8)")
    ap.add_argument("--grid-wgs", type=int, default=None,
                    help="kg_snapshot_tune grid_wgs (k_grid_level WGs per CU; default 2 for C2/C4, 4 for C3: "
                         "profiles/r4w_grid_stream_wgs_ab.jsonl)")
    ap.add_argument("--grid-ms", type=int, default=1,
                    help="kg_snapshot_tune grid_ms: the grid tier's queries as a multi-source bit-parallel BFS "
                         "(64 queries per group) when dense per-node masks fit (graphs up to ~4 M nodes)")
    ap.add_argument("--grid-ms-words", type=int, default=8,
                    help="kg_snapshot_tune grid_ms_words: 64-bit words per MS-BFS node mask (64 queries each)")
    ap.add_argument("--grid-ms-bytes", type=float, default=0,
                    help="kg_snapshot_tune grid_ms_bytes: MS-BFS mask budget per workspace in bytes (0: library default)")
    ap.add_argument("--grid-ms-tg-cap", type=int, default=256,
                    help="kg_snapshot_tune grid_ms_tg_cap: holders above which MS-BFS probes a query's subject in dset")
    ap.add_argument("--stream-wgs", type=int, default=None,
                    help="kg_snapshot_tune stream_wgs (k_stream4 WGs per CU; default 2 for C2/C4 -- LDS left to the "
                         "other batches' tail tiers, profiles/r4w_grid_stream_wgs_ab.jsonl -- and 3 for C3)")
    ap.add_argument("--back-wgs", type=int, default=None,
                    help="kg_snapshot_tune back_wgs (k_back WGs per CU; default 3 for C2/C4 with 4 batches in "
                         "flight, 1 for C3 with 6: profiles/r4s_back_wgs_ab.jsonl, r2bwc3_back_wgs_c3_ab.jsonl)")
    ap.add_argument("--back-edges", type=int, default=0,
                    help="kg_snapshot_tune back_edges (k_back reverse-edge budget per query, 0 = library default 2^12)")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="HIP hardware queues for this process (GPU_MAX_HW_QUEUES, 1..32; 0 = HIP's default, 4; "
                         "default 16): streams map onto queues round-robin as they are created, and in-flight "
                         "streams that share a queue serialise (DESIGN.md 7f).  32 helps C5's 12 callers (1.87 -> "
                         "2.99 x 10^7 trees/s) but cost C3 (1.83 -> 1.00 x 10^9) and the sharded lines in the same "
                         "process (profiles/r6o_c5_hw_queues.txt, r6q_hw_queues_default_line_ab.jsonl), so the C5 "
                         "sub-line runs as a child process at 32")
    ap.add_argument("--inflight", type=int, default=None,
                    help="batches in flight per GPU: one HIP stream (own workspace) and one host thread each "
                         "(default 4; 16 for --mode expand, whose batches end in long sequential roots; 2 with "
                         "--heavy-tail)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget (0 = skip)")
    ap.add_argument("--parity", type=int, default=1_000_000,
                    help="checks of the first timed batch compared with the oracle (Go-order DFS; 0 = skip).  Any "
                         "mismatch makes bench.py exit 1 after printing its line")
    ap.add_argument("--parity-canonical", type=int, default=100_000,
                    help="of those, checks also compared under the oracle's schedule-free (canonical) policy")
    ap.add_argument("--parity-roots", type=int, default=300, help="--mode expand: roots compared with oracle.expand")
    ap.add_argument("--latency-batches", type=int, default=240,
                    help="batches of the separate latency phase (after the timed region, same batches in flight): "
                         "p50 / p99 batch latency, submit to done")
    ap.add_argument("--stream-base", type=int, default=0,
                    help="diagnostics: the headline's in-flight streams start at this one (0 = the current stream)")
    ap.add_argument("--host-calls", type=int, default=20,
                    help="kg_check_batch calls per in-flight thread in the host-path leg (1 M-check host batches, "
                         "PCIe both ways; 0 = skip)")
    ap.add_argument("--stats-every", type=int, default=10,
                    help="collect kernel stats (HIP events around the batch and k_stream4, the in-kernel counters) on "
                         "every k-th timed batch (1 = all).  Default 10: two of the driver's 20 steps -- the event "
                         "records between a batch's launches cost ~9 %% of the 20-step line when every batch carries "
                         "them (profiles/r6i_stats_every_ab.jsonl)")
    ap.add_argument("--replay", type=int, default=0,
                    help="cycle over this many distinct batches (0 = a distinct batch for every step; diagnostics)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = os.cpu_count(), also timed at the affinity count, 16 and 1)")
    ap.add_argument("--preset", type=int, default=0,
                    help="0 = C2/C4 rewrite-free (headline); 1 = C3 (OPL view/edit/share via the rewrite interpreter)")
    ap.add_argument("--mode", choices=["check", "expand", "sharded", "host", "refresh", "rehearse"], default="check",
                    help="expand = config C5: batched BuildTree of hot group#member roots; sharded = the "
                         "hash-sharded mode (each rank holds 1/N of the graph, all-to-all frontier exchange); "
                         "host = the host-buffer boundary end to end: kg_check_batch over a snapshot replicated "
                         "on every visible GPU (PCIe included), then the request batcher fed single checks; "
                         "rehearse = the multi-rank launch and aggregation alone on CPU ranks (gloo; tests)")
    ap.add_argument("--callers", type=int, default=4, help="--mode host: threads calling kg_check_batch at once")
    ap.add_argument("--clients", type=int, default=256,
                    help="--mode host: native caller threads of the request batcher (one blocking call per request)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for --mode sharded (nccl = RCCL)")
    ap.add_argument("--shard-protocol", default="auto", choices=["auto", "fixed", "dynamic"],
                    help="--mode sharded --shard-driver py: exchange protocol (keto_amd.sharded.ShardedChecker)")
    ap.add_argument("--shard-driver", default="lib", choices=["lib", "py"],
                    help="--mode sharded: lib = the whole batch inside libketogpu.so over RCCL (kg_shard_comm_init; "
                         "the gloo host transport with --backend gloo), one kg_check_batch_device call per batch as "
                         "a Go host makes it; py = keto_amd.sharded.ShardedChecker driving the kg_shard_* steps "
                         "(needed for --shard-budget)")
    ap.add_argument("--roots", type=int, default=100_000, help="expand roots per step (C5)")
    ap.add_argument("--expand-gw", type=int, default=1,
                    help="kg_snapshot_tune expand_gw (1: large expand roots gather their neighbourhood, then walk the copy)")
    ap.add_argument("--delta", type=int, default=1000, help="--mode refresh: rows per transaction")
    a = ap.parse_args(argv)
    if a.hw_queues is None:
        a.hw_queues = 16
    if a.batch is None:
        a.batch = 62_500 if a.heavy_tail else 1_000_000
    if a.inflight is None:
        # --heavy-tail: 4 (round 6: 2 / 3 / 4 / 6 in flight gave 6.2 / 9.1 / 12.0 / 10.3 x 10^6 checks/s at p99
        # 21.4 / 21.5 / 22.4 / 40.6 ms per 62.5 k-check batch, profiles/r6t_operating_points.txt)
        # --preset 1 (C3): 6, as the C3 sub-line (--c3-inflight)
        a.inflight = 20 if a.mode == "expand" else (6 if a.preset else 4)
    if a.back_wgs is None:
        a.back_wgs = 1 if a.preset else 3
    if a.grid_wgs is None:
        a.grid_wgs = 4 if a.preset else 2
    if a.stream_wgs is None:
        a.stream_wgs = 3 if a.preset else 2
    if a.tuples is None:
        a.tuples = 1.2e8 if a.heavy_tail else (1e7 if a.mode == "refresh" else 1e9)
    return a


def apply_tune(snap, a) -> None:
    """The engine knobs of the check bench (tests/test_gpu_check.py::test_bench_tune_set_vs_oracle runs
    the parity test with exactly this set)."""
    snap.tune("stream_ecap", a.stream_ecap)
    snap.tune("stream_steal", a.stream_steal)
    snap.tune("grid_wgs", a.grid_wgs)
    snap.tune("grid_ms", a.grid_ms)
    snap.tune("grid_ms_words", a.grid_ms_words)
    snap.tune("grid_ms_tg_cap", a.grid_ms_tg_cap)
    if a.grid_ms_bytes:
        snap.tune("grid_ms_bytes", int(a.grid_ms_bytes))
    snap.tune("stream_wgs", a.stream_wgs)
    snap.tune("back_wgs", a.back_wgs)
    if a.back_edges:
        snap.tune("back_edges", a.back_edges)
    snap.tune("grid_reserve", 1)  # a server pays this once at start-up, not inside some request's batch


def bench_expand(a):
    """Config C5: full subject-set trees for the most popular group#member roots at max_read_depth
    (SURVEY.md 8d), one kg_expand_batch call per step (trees delivered to host memory)."""
    import torch
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    # one process per GPU under torchrun (each rank its own replica and batches, max-over-ranks time:
    # weak scaling); ranks beyond the GPU count share GPUs (a gloo rehearsal on a 1-GPU box)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(a.backend, rank=rank, world_size=world)
    L = _lib.load()
    snap, _ = build_synthetic(a, a.tuples, device=local)
    snap.tune("expand_gw", a.expand_gw)
    from keto_amd.synth import hot_group_roots
    roots = hot_group_roots(snap.synth_ids(), a.roots)
    depth = a.global_depth if a.global_depth != 10 else 5

    P = max(1, a.inflight)  # batches in flight: P host threads, each on its own lane (stream + buffers)
    # the value: roots and trees resident in HBM (kg_expand_batch_device); then the host-buffer boundary
    el, results = expand_steps(L, snap, roots, depth, P, a.steps, a.warmup, dist, device=True)
    el, _ = aggregate(dist, el, 0.0, f"cuda:{local}" if a.backend == "nccl" else None)
    # host-buffer leg at <= 4 callers: every library lane holds ~3 GB of expand buffers, and 16 device lanes + 16
    # host lanes beside the parent's and this child's 1e9-tuple graphs ran out of HBM (r6z closing run)
    P_h = min(P, 4)
    el_h, res_h = expand_steps(L, snap, roots, depth, P_h, a.steps, a.warmup, dist)
    el_h, _ = aggregate(dist, el_h, 0.0, f"cuda:{local}" if a.backend == "nccl" else None)
    nodes = sum(r[0] for r in results)
    kms = sum(r[1] for r in results)
    off = res_h[-1][2]
    out = {"metric": "expand trees/sec (batched BuildTree, hot group#member roots)",
           "value": world * a.roots * a.steps / el, "unit": "trees/s", "n_gpus": world, "scaling": "weak",
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": el / a.steps * 1e3,
           "higher_is_better": True, "dtype": "u32", "data": "synthetic (device-generated, seed %d)" % a.seed,
           "config": {"workload": "C5: %d hot roots @ %.4g tuples (rows), max_read_depth %d" % (a.roots, snap.info()["rows"],
                                                                                            depth),
                      "inflight_per_gpu": P, "hw_queues": a.hw_queues, "parallelism": f"replica{world}",
                      "expand_gw": a.expand_gw},
           "tree_nodes_per_step": nodes / a.steps, "tree_nodes_per_s": nodes / el,
           "kernel_ms_per_step": kms / a.steps, "io": "kg_expand_batch_device: roots and trees in HBM",
           "host_path": {"value": world * a.roots * a.steps / el_h, "unit": "trees/s", "ms_per_step": el_h / a.steps * 1e3, "inflight": P_h,
                         "what": "kg_expand_batch (roots from / trees to pinned host memory, PCIe both ways): "
                                 "not the value"}}
    if off is not None:
        sz = np.diff(off.astype(np.int64))
        out["records_per_root"] = {"p50": float(np.percentile(sz, 50)), "p99": float(np.percentile(sz, 99)),
                                   "max": int(sz.max()), "roots_over_512": int((sz > 512).sum()),
                                   "top10_share": float(np.sort(sz)[-10:].sum() / max(1, sz.sum()))}
    if off is not None:
        # the batch's tail: the largest root's walk alone (one sequential pre-order DFS on one wave)
        big = int(np.argmax(np.diff(off.astype(np.int64))))
        one = np.ascontiguousarray(roots[big:big + 1])
        walk = []
        for _ in range(3):
            buf = _lib.kg_tree_buf()
            _lib.check(L.kg_expand_batch(snap.handle, one.ctypes.data_as(C.c_void_p), 1, depth, C.byref(buf)),
                       "kg_expand_batch")
            walk.append(buf.kernel_ms)
            n_big = int(buf.n_nodes)
            L.kg_tree_free(C.byref(buf))
        out["largest_root"] = {"records": n_big, "walk_kernel_ms": float(min(walk))}
    # traffic: PMC bytes of every k_expand* dispatch per call (scripts/gpu_r6_final.sh, same roots and callers)
    rf = expand_roofline(L, snap, roots, depth, kms / a.steps, pmc_traffic("k_expand", int(a.tuples), a.roots, 0, P, "x"))
    if rf:
        out["roofline"] = rf
    orc = None
    if rank == 0 and ((a.parity_roots > 0 and off is not None) or (world == 1 and a.cpu_seconds > 0)):
        orc = expand_oracle(snap)
    if rank == 0 and a.parity_roots > 0 and off is not None:
        out["parity"] = expand_parity(snap, roots, np.diff(off.astype(np.int64)), depth, a, orc)
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        out["cpu_baseline"] = expand_cpu_baseline(orc, roots, depth, a)
    if rank == 0:
        print(json.dumps(out), flush=True)
        if out.get("parity") and out["parity"]["mismatches"]:
            sys.stderr.write("PARITY FAILURE: GPU expand trees differ from the oracle\n")
            if dist:
                dist.destroy_process_group()
            sys.exit(1)
    if dist:
        dist.destroy_process_group()


def expand_steps(L, snap, roots: np.ndarray, depth: int, P: int, steps: int, warmup: int, dist=None,
                 device: bool = False):
    """C5's timed region: P host threads, each on its own lane (stream + cached buffers), run `steps`
    kg_expand_batch calls over the same roots after a warm-up, between barriers.  Returns (elapsed s,
    per call (tree records, kernel ms, root offsets)).  device: kg_expand_batch_device -- the roots
    resident in HBM before the timed region, the trees left in HBM (each thread on a HIP stream of its
    own; root offsets are not copied back, the caller reads them from an untimed call)."""
    import torch
    from keto_amd import _lib
    n = len(roots)
    nw = min(P, steps)
    if device:
        dev = torch.device("cuda", snap.device)
        droots = torch.from_numpy(np.ascontiguousarray(roots, np.uint32).view(np.int32)).to(dev)
        streams = [torch.cuda.Stream(dev) for _ in range(nw)]
        torch.cuda.synchronize(dev)

    def step(p=0):
        buf = _lib.kg_tree_buf()
        if device:
            _lib.check(L.kg_expand_batch_device(snap.handle, C.c_void_p(droots.data_ptr()), n, depth, C.byref(buf),
                                                C.c_void_p(streams[p].cuda_stream)), "kg_expand_batch_device")
            res = (buf.n_nodes, buf.kernel_ms, None)
        else:
            _lib.check(L.kg_expand_batch(snap.handle, roots.ctypes.data_as(C.c_void_p), n, depth, C.byref(buf)),
                       "kg_expand_batch")
            off = np.ctypeslib.as_array(buf.root_off, shape=(n + 1,)).copy() if buf.root_off else None
            res = (buf.n_nodes, buf.kernel_ms, off)
        L.kg_tree_free(C.byref(buf))
        return res

    results = [None] * steps
    errors = []
    warm = threading.Barrier(nw + 1)  # every lane warmed up
    go = threading.Barrier(nw + 1)    # timed region starts (after the ranks' barrier)

    def worker(p):
        try:
            for _ in range(max(1, -(-warmup // nw))):  # warm-up: this thread's lane and buffers
                step(p)
        except Exception as e:  # noqa: BLE001 -- re-raised below
            errors.append(e)
        warm.wait()
        go.wait()
        try:
            for k in range(p, steps, nw):
                if not errors:
                    results[k] = step(p)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(p,)) for p in range(nw)]
    for t in th:
        t.start()
    warm.wait()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    go.wait()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    if errors:
        raise errors[0]
    return el, results


def expand_roofline(L, snap, roots: np.ndarray, depth: int, call_ms: float, traffic=None):
    """Roofline of the expand launch chain (8 B per row opened, 4 B per edge read, 12 B per
    emitted tree node), from one more call's records (every step expands the same roots) over the calls'
    mean device time (HIP events around k_expand_lds / _hash / _hbm + k_expand_compact on the call's
    stream; several calls overlap, so a call's time is contended wall time)."""
    from keto_amd import _lib
    buf = _lib.kg_tree_buf()
    _lib.check(L.kg_expand_batch(snap.handle, roots.ctypes.data_as(C.c_void_p), len(roots), depth, C.byref(buf)),
               "kg_expand_batch")
    rec = np.ctypeslib.as_array(C.cast(buf.nodes, C.POINTER(C.c_uint8)), shape=(int(buf.n_nodes) * 20,)).view(
        np.dtype([("type", "u1"), ("is_set", "u1"), ("pad", "<u2"), ("ns", "<u4"), ("obj", "<u4"), ("rel", "<u4"),
                  ("n_children", "<u4")])).copy() if buf.n_nodes else None
    L.kg_tree_free(C.byref(buf))
    if rec is None or call_ms <= 0:
        return None
    unions = rec["type"] == 1  # kg_tree_node type 1 = union (include/ketogpu.h)
    R, E, T = int(unions.sum()), int(rec["n_children"][unions].sum()), int(len(rec))
    byts = 8 * R + 4 * E + 12 * T
    gbs = byts / (call_ms * 1e-3) / 1e9
    return {"kernel": "k_expand_lds/_gw/_hash/_hbm + k_expand_compact (one call's chain)", "bound": "hbm",
            "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "traffic": traffic,
            "bytes_model": "8*unions(rows opened) + 4*children(edges read) + 12*tree records",
            "bytes_per_call": byts, "rows_opened": R, "edges_read": E, "records": T, "call_kernel_ms": call_ms}


def expand_oracle(snap):
    """The oracle (oracle/keto_oracle.c) over the snapshot's own rows in shard order, for the C5 parity
    leg and CPU baseline; its node arrays ride along as .nd."""
    from keto_amd import _lib
    from oracle.oracle import Oracle
    L = _lib.load()
    t0 = time.perf_counter()
    info = snap.info()
    nn, nr = info["nodes"], info["rows"]
    row_off = np.zeros(nn + 1, np.uint64)
    row_subj = np.zeros(nr, np.uint32)
    nd = [np.zeros(nn, np.uint32) for _ in range(3)]
    p = lambda x: x.ctypes.data_as(C.c_void_p)
    _lib.check(L.kg_snapshot_export_csr(snap.handle, p(row_off), p(row_subj), p(nd[0]), p(nd[1]), p(nd[2])),
               "kg_snapshot_export_csr")
    orc = Oracle.from_csr(0, nd[0], nd[1], nd[2], row_off, row_subj, nthreads=16)
    orc.nd = nd
    orc.build_s = time.perf_counter() - t0
    return orc


def expand_cpu_baseline(orc, roots: np.ndarray, depth: int, a) -> dict:
    """BuildTree (oracle/keto_oracle.c ko_expand_node: expand/engine.go:35-104, one visited set per request,
    rows in shard order) over the C5 roots on the host cores: a bounded sample of the same roots (grown
    until ~--cpu-seconds of work), at the usable CPU count and at 1 thread -- one C call per pass
    (ko_expand_nodes_batch: pthreads take 16-root chunks; no Python per root)."""
    cpus = effective_cpus()
    eff = cpus["effective"]

    nodes = np.ascontiguousarray(roots[:, 1]).astype(np.uint32)  # synthetic group#member: node id == object id
    dp = np.ascontiguousarray(roots[:, 3]).view(np.int32) if roots.dtype == np.uint32 else roots[:, 3].astype(np.int32)

    def run(n, th):  # one C call: the roots spread over th pthreads, no Python per root
        t = time.perf_counter()
        orc.expand_nodes_batch(nodes[:n], dp[:n], depth, th)
        return time.perf_counter() - t

    res = {}
    for th, budget in ((eff, a.cpu_seconds / 2), (1, a.cpu_seconds / 4)):
        n = 64
        t = run(n, th)
        while t < budget / 4 and n < len(roots):
            n = min(len(roots), n * 4)
            t = run(n, th)
        passes, tt = 1, t
        while tt < budget / 2:  # the whole set is quick on many cores: repeat it until the budget is spent
            tt += run(n, th)
            passes += 1
        res[th] = (n * passes / tt, n, tt, passes)
    best = max(res, key=lambda k: res[k][0])
    v, n, t, passes = res[best]
    return {"value": v, "unit": "trees/s", "cores": best, "kind": "port",
            "sample": f"{passes} pass(es) over the first {n} of the {len(roots)} C5 roots ({t:.1f} s), BuildTree with one "
                      f"visited set per request (oracle/keto_oracle.c ko_expand_nodes_batch: ko_expand_node per root), "
                      f"{best} host threads (best of {sorted(res)})",
            "by_threads": {str(k): r[0] for k, r in sorted(res.items())}, "value_1thread": res[1][0],
            "cpus": cpus, "host_cpu": host_cpu()}


def expand_parity(snap, roots: np.ndarray, sizes: np.ndarray, depth: int, a, orc=None) -> dict:
    """C5 trees vs the oracle's BuildTree (oracle/keto_oracle.c, expand/engine.go:35-104) on the snapshot's
    own rows: the 10 largest roots of the timed batch plus a seeded sample of the rest, same pre-order and
    same child order (rows are in shard order on both sides)."""
    from keto_amd.engine import ExpandEngine, Config
    t0 = time.perf_counter()
    orc = orc or expand_oracle(snap)
    nd = orc.nd
    rng = np.random.default_rng(a.seed)
    top = np.argsort(sizes)[-10:]
    rest = rng.choice(len(roots), size=min(len(roots), max(0, a.parity_roots - 10)), replace=False)
    pick = np.unique(np.concatenate([top, rest]))
    ex = ExpandEngine(snap, Config(depth))
    got = ex.build_trees_ids(roots[pick])
    bad, recs = [], 0
    for i, g in zip(pick, got):
        r = roots[i]
        node = int(r[1])  # synthetic group#member: node id == object id (kg_synth.h block layout)
        assert nd[0][node] == r[0] and nd[1][node] == r[1] and nd[2][node] == r[2], "root is not its node"
        exp = orc.expand_node(node, int(np.int32(np.uint32(r[3]))), depth)
        recs += 0 if exp is None else len(exp)
        if (exp is None) != (g is None):
            bad.append(int(i))
            continue
        if exp is None:
            continue
        e2, g2 = np.asarray(exp, np.int64).copy(), np.asarray(g, np.int64).copy()
        for x in (e2, g2):  # subject ids: oracle ns = rel = -1, GPU KG_SUBJECT_ID / 0
            x[x[:, 1] == 0, 2] = 0
            x[x[:, 1] == 0, 4] = 0
        if e2.shape != g2.shape or not (e2 == g2).all():
            bad.append(int(i))
    return {"roots": int(len(pick)), "records": int(recs), "mismatches": len(bad), "first_mismatches": bad[:8],
            "largest_roots_included": 10, "compare": "exact pre-order records, same child order",
            "oracle": "oracle/keto_oracle.c ko_expand_node", "seconds": time.perf_counter() - t0}


def bench_refresh(a):
    """Incremental snapshot refresh (kg_snapshot_apply): on a synthetic graph of
    --tuples (default 1e7), transactions of --delta rows (half inserts -- new doc#viewer@user and
    group#member@group#member rows -- half deletes of existing rows), each applied to the latest
    snapshot, then a 1 M-check batch on the refreshed snapshot.  Reports the commit -> snapshot-ready
    latency (host delta handling + device rebuild) next to a full rebuild of the same graph."""
    import torch
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    L = _lib.load()
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    base, _ = build_synthetic(a, a.tuples, device=0)
    t_full = time.perf_counter() - t0
    ids = base.synth_ids()
    rows = base.export()  # (n, 6) uint32, shard order
    rng = np.random.default_rng(a.seed)
    n_docs, n_groups, n_users = ids["n_docs"], ids["n_groups"], ids["n_users"]
    half = a.delta // 2

    def delta():
        ins = np.zeros((half, 6), np.uint32)
        k = rng.random(half) < 0.5
        ins[:, 0] = np.where(k, 0, 1)                                   # doc / group
        ins[:, 1] = np.where(k, rng.integers(0, n_docs, half), n_docs + rng.integers(0, n_groups, half))
        ins[:, 2] = np.where(k, 1, 2)                                   # viewer / member
        ins[:, 3] = np.where(k, _lib.KG_SUBJECT_ID, 1)
        ins[:, 4] = np.where(k, ids["user_obj0"] + rng.integers(0, n_users, half), n_docs + rng.integers(0, n_groups, half))
        ins[:, 5] = np.where(k, 0, 2)
        dels = rows[rng.integers(0, len(rows), a.delta - half)]
        return ins, dels

    cur = base.apply(*delta())  # warm-up: the first apply builds the host node map from the device
    dq = torch.empty((a.batch, 7), dtype=torch.int32, device="cuda")
    _lib.check(L.kg_synth_queries(base.handle, 99, a.batch, dq.data_ptr()), "kg_synth_queries")
    out = torch.empty(a.batch, dtype=torch.uint8, device="cuda")
    err = torch.empty(a.batch, dtype=torch.int32, device="cuda")
    lat, chk = [], []
    for _ in range(a.steps):
        ins, dels = delta()
        s0 = time.perf_counter()
        nxt = cur.apply(ins, dels)
        s1 = time.perf_counter()
        _lib.check(L.kg_check_batch_device(nxt.handle, dq.data_ptr(), a.batch, a.global_depth, out.data_ptr(),
                                           err.data_ptr(), None, None), "kg_check_batch_device")
        torch.cuda.synchronize()
        s2 = time.perf_counter()
        lat.append((s1 - s0) * 1e3)
        chk.append((s2 - s1) * 1e3)
        cur = nxt  # the previous snapshot is released here (no batch reads it any more)
    info = cur.info()
    res = {"metric": "snapshot refresh latency (commit -> snapshot ready, kg_snapshot_apply)",
           "value": float(np.percentile(lat, 50)), "unit": "ms", "n_gpus": 1, "steps": a.steps, "warmup": 1,
           "ms_per_step": float(np.mean(lat)), "higher_is_better": False, "dtype": "u32",
           "data": "synthetic (device-generated, seed %d) + random deltas" % a.seed,
           "config": {"workload": "%d-row transactions (%d inserts, %d deletes) on %.3g tuples" %
                      (a.delta, half, a.delta - half, a.tuples), "rows": info["rows"], "nodes": info["nodes"]},
           "apply_ms": {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                        "max": float(np.max(lat))},
           "first_check_batch_ms": float(np.percentile(chk, 50)), "full_build_s": t_full}
    print(json.dumps(res), flush=True)


def bench_sharded(a):
    """Config C4's hash-sharded mode: rank r builds only the rows it owns of the same
    synthetic graph and checks its own batches; every BFS level exchanges frontier records with an
    all-to-all (RCCL over xGMI under torchrun, backend "nccl") of fixed-size buckets, with no host
    round trip inside a batch (keto_amd.sharded, protocol "fixed").  --inflight batches per rank run at
    once, each on its own stream (own per-stream batch state in the library) and, across ranks, its own
    process group.  Weak scaling: B checks per rank per step."""
    import torch
    from keto_amd import _lib
    from keto_amd.sharded import HipShardOps, LibShardedChecker, ShardedChecker
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    lib = a.shard_driver == "lib"
    if lib and a.shard_budget:
        raise SystemExit("--shard-budget (escalation) runs with --shard-driver py")
    # one rank per GPU; ranks beyond the GPU count share GPUs (a gloo rehearsal on a 1-GPU box)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(a.backend, rank=rank, world_size=world)
    L = _lib.load()
    t_build = time.time()
    snap, _ = build_synthetic(a, a.tuples, device=local, shard=(rank, world))
    info = snap.info()
    t_build = time.time() - t_build
    snap.tune("shard_budget", a.shard_budget)
    snap.tune("shard_back_budget", a.shard_back_budget)
    if a.shard_vis:
        snap.tune("shard_vis", a.shard_vis)
    if a.shard_heavy >= 0:
        snap.tune("shard_heavy", a.shard_heavy)
    B = a.batch
    P = max(1, a.inflight)
    n_distinct = max(P, 2)
    dqs = []
    for k in range(n_distinct):
        dq = torch.empty((B, 7), dtype=torch.int32, device=f"cuda:{local}")
        _lib.check(L.kg_synth_queries(snap.handle, 1000 + rank + 7919 * k, B, dq.data_ptr()), "kg_synth_queries")
        dqs.append(dq)
    groups = [None] * P
    if dist is not None and P > 1:
        groups = [dist.new_group(list(range(world))) for _ in range(P)]
    if lib:  # one communicator per in-flight stream (RCCL ids broadcast over the default group, in order)
        transport = "rccl" if a.backend == "nccl" else "host"
        chks = [LibShardedChecker(snap, rank, world, dist, group=groups[p], transport=transport) for p in range(P)]
    else:
        chks = [ShardedChecker(HipShardOps(snap), rank, world, dist, device=f"cuda:{local}", cap=1 << 22,
                               protocol=a.shard_protocol, group=groups[p]) for p in range(P)]

    def cstats(c):  # the counters both drivers report
        if lib:
            st = c.stats()
            return {"levels": st["levels"], "back_levels": 0, "final_levels": 0, "records_sent": st["records_sent"],
                    "host_syncs": st["host_syncs"], "bucket": st["bucket"], "level_records": None,
                    "general_queries": st["general_queries"]}
        return {"levels": c.levels, "back_levels": c.back_levels, "final_levels": c.final_levels,
                "records_sent": c.records_sent, "host_syncs": c.host_syncs, "bucket": c.bucket,
                "level_records": c.level_records, "general_queries": c.general_queries}
    for p in range(P):  # warm-up: each checker sizes its buckets / per-stream state
        for _ in range(max(1, a.warmup // P)):
            chks[p].check(dqs[p % n_distinct], a.global_depth)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    lat, outs, errors = [], [None] * P, []
    sent = [0] * P
    syncs = [0] * P
    go = threading.Barrier(P + 1)

    def worker(p):
        try:
            go.wait()
            # this thread's current stream is its checker's own: no ordering through a shared stream
            with torch.cuda.stream(chks[p].stream if lib else chks[p].ops.torch_stream):
                for k in range(p, a.steps, P):
                    s0 = time.perf_counter()
                    h0 = chks[p].host_syncs if not lib else 0
                    res, err = chks[p].check(dqs[k % n_distinct], a.global_depth)
                    torch.cuda.current_stream().synchronize()
                    lat.append(time.perf_counter() - s0)
                    st = cstats(chks[p])
                    sent[p] += st["records_sent"]
                    syncs[p] += st["host_syncs"] - h0
                    outs[p] = (res, err)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(p,)) for p in range(P)]
    [t.start() for t in th]
    t0 = time.perf_counter()
    go.wait()
    [t.join() for t in th]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if errors:
        raise errors[0]
    for o in outs:
        if o is None:
            continue
        r = o[0].cpu().numpy()
        assert (o[1].cpu().numpy() == 0).all() and (r <= 1).all(), "unexpected errors in the synthetic batch"
    elapsed, recs = aggregate(dist, elapsed, float(sum(sent)), f"cuda:{local}" if a.backend == "nccl" else None)
    cs = cstats(chks[0])
    out = {"metric": "permission checks/sec (batched check, synthetic Drive-like graph, hash-sharded)",
           "value": world * B * a.steps / elapsed, "unit": "checks/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (device-generated Drive-like tuple graph, seed %d)" % a.seed,
           "config": {"workload": "%s generator @ %.3g tuples hash-sharded over %d rank(s), %d checks/step/rank, "
                                  "max_read_depth %d" % ("C3" if a.preset else "C4", a.tuples, world, B,
                                                         a.global_depth),
                      "materialized": snap.materialized() if a.preset else None,
                      "rows_on_rank": info["rows"], "nodes": info["nodes"], "batch_per_gpu": B,
                      "inflight_per_gpu": P, "driver": ("in-library kg_check_batch_device (kg_shard_comm.hip, %s)"
                                                        % ("RCCL" if a.backend == "nccl" else "host transport")
                                                        if lib else "keto_amd.sharded.ShardedChecker"),
                      "protocol": "fixed" if lib else a.shard_protocol, "parallelism": f"shard{world}"},
           "p99_batch_ms": float(np.percentile(np.array(lat) * 1e3, 99)),
           "batch_ms_p50": float(np.percentile(np.array(lat) * 1e3, 50)),
           "allowed_fraction": float(outs[0][0].float().mean().item()) if outs[0] is not None else None,
           "levels_per_batch": cs["levels"], "backward_levels_per_batch": cs["back_levels"],
           "final_levels_per_batch": cs["final_levels"], "shard_budget": a.shard_budget,
           "host_syncs_per_batch": sum(syncs) / max(1, a.steps),
           "bucket": cs["bucket"], "shard_back_budget": a.shard_back_budget,
           "shard_heavy": a.shard_heavy, "records_exchanged_per_batch": recs / a.steps,
           **({"level_records": cs["level_records"]} if cs["level_records"] else {}),
           "snapshot_build_s": t_build}
    bad = 0
    if rank == 0 and world == 1 and a.parity > 0:
        # untimed: batch 0 once more through the sharded path, against the oracle over the same rows
        res0, _ = chks[0].check(dqs[0], a.global_depth)
        orc = CheckOracle(snap, a, effective_cpus()["effective"])
        out["parity"] = orc.parity(dqs[0].cpu().numpy().view(np.uint32), res0.cpu().numpy(), a.parity,
                                   a.parity_canonical)
        bad = out["parity"]["mismatches"] + out["parity"]["canonical_mismatches"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    if bad:
        sys.stderr.write("PARITY FAILURE: sharded answers differ from the oracle\n")
        sys.exit(1)


def bench_host(a):
    """The host-buffer boundary end to end (what the cgo binding in INTEGRATION.md calls): one process,
    the snapshot replicated on every visible GPU (kg_snapshot_synthetic_on), and
      (1) `callers` threads each calling kg_check_batch on its own 1M-check host batches -- H2D, the
          tiers, D2H, split over the replicas inside the library; checks/s and p50/p99 per call;
      (2) the library's request batcher (kg_batcher_check: one blocking call per request, the shape of
          one goroutine per Check RPC, internal/check/handler.go:248) driven by `clients` native caller
          threads (tools/kg_loadgen.cpp, no Python on the request path) for a few seconds, every answer
          checked against a direct batch; checks/s, per-call and per-batch p50/p99.
      (3) the same batcher from Python threads (keto_amd.batcher.NativeBatcher.check_ids), for scale."""
    import torch
    from keto_amd import _lib
    from keto_amd.batcher import NativeBatcher
    from keto_amd.build import TOOLS_LIB
    from keto_amd.engine import Config, Engine, Snapshot
    L = _lib.load()
    n_dev = max(1, torch.cuda.device_count()) if a.gpus <= 1 else a.gpus
    devices = list(range(n_dev))
    t_build = time.time()
    snap, _ = build_synthetic(a, a.tuples, devices=devices)
    snap.tune("stream_wgs", a.stream_wgs)
    snap.tune("back_wgs", a.back_wgs)
    snap.tune("grid_wgs", a.grid_wgs)
    t_build = time.time() - t_build
    B, T = a.batch, max(1, a.callers)
    torch.cuda.set_device(0)
    qs = []
    for t in range(T):  # distinct batches per caller, generated on the device then held on the host
        d = torch.empty((B, 7), dtype=torch.int32, device="cuda:0")
        _lib.check(L.kg_synth_queries(snap.handle, 1000 + 7919 * t, B, d.data_ptr()), "kg_synth_queries")
        qs.append(np.ascontiguousarray(d.cpu().numpy().view(np.uint32)))
    eng = Engine(snap, Config(a.global_depth))
    expect = eng.batch_check_ids(qs[0])[0]

    def call(t, out, err):
        rc = L.kg_check_batch(snap.handle, qs[t].ctypes.data_as(C.c_void_p), B, a.global_depth,
                              out.ctypes.data_as(C.c_void_p), err.ctypes.data_as(C.c_void_p), None)
        _lib.check(rc, "kg_check_batch")

    lat, errs = [], []
    per = max(1, a.steps // T)
    ready = threading.Barrier(T + 1)

    def worker(t):
        try:
            out = np.empty(B, np.uint8)
            err = np.empty(B, np.uint32)
            call(t, out, err)  # this thread's lanes (stream, pinned staging, workspace) exist before timing
            ready.wait()
            for _ in range(per):
                s0 = time.perf_counter()
                call(t, out, err)
                lat.append(time.perf_counter() - s0)
            if t == 0:
                assert (out == expect).all() and (err == 0).all()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            ready.abort()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    [x.start() for x in th]
    ready.wait()
    t0 = time.perf_counter()
    [x.join() for x in th]
    el = time.perf_counter() - t0
    if errs:
        raise errs[0]
    host_rate = B * per * T / el
    # (2) native batcher under native callers
    LG = C.CDLL(TOOLS_LIB)
    LG.kgl_batcher_load.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_int, C.c_double,
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    q0 = qs[0]
    batcher = {}
    for clients, per_call in ((a.clients, 1), (a.clients, 16), (64, 1)):
        with NativeBatcher(snap, a.global_depth, max_batch=1 << 16, max_wait_us=200, dispatchers=4) as nb:
            n_chk, el2, bad = C.c_uint64(), C.c_double(), C.c_uint64()
            rc = LG.kgl_batcher_load(nb.handle, q0.ctypes.data_as(C.c_void_p), len(q0),
                                     expect.ctypes.data_as(C.c_void_p), 64, per_call, 0.5, C.byref(n_chk),
                                     C.byref(el2), C.byref(bad))  # warm-up
            nb.reset_stats()
            rc = LG.kgl_batcher_load(nb.handle, q0.ctypes.data_as(C.c_void_p), len(q0),
                                     expect.ctypes.data_as(C.c_void_p), clients, per_call, 3.0, C.byref(n_chk),
                                     C.byref(el2), C.byref(bad))
            assert rc == 0 and bad.value == 0, (rc, bad.value)
            st = nb.stats()
            batcher[f"native_{clients}x{per_call}"] = {
                "callers": clients, "checks_per_call": per_call, "checks_per_s": n_chk.value / el2.value,
                "p50_call_ms": st["call_p50_ms"], "p99_call_ms": st["call_p99_ms"],
                "p50_batch_ms": st["batch_p50_ms"], "p99_batch_ms": st["batch_p99_ms"],
                "mean_batch": st["checks"] / max(1, st["batches"]), "answers_checked": n_chk.value}
    # (3) the same batcher from Python threads
    with NativeBatcher(snap, a.global_depth, max_batch=1 << 16, max_wait_us=200, dispatchers=4) as nb:
        n_py, stop = [0], [False]

        def pyclient(c):
            i, k = c * 9973 % len(q0), 0
            while not stop[0]:
                o, e = nb.check_ids(q0[i:i + 1])
                assert o[0] == expect[i]
                i = (i + 1) % len(q0)
                k += 1
            n_py[0] += k

        th = [threading.Thread(target=pyclient, args=(c,)) for c in range(16)]
        t0 = time.perf_counter()
        [x.start() for x in th]
        time.sleep(2.0)
        stop[0] = True
        [x.join() for x in th]
        el3 = time.perf_counter() - t0
        st = nb.stats()
        batcher["python_16x1"] = {"callers": 16, "checks_per_call": 1, "checks_per_s": n_py[0] / el3,
                                  "p50_call_ms": st["call_p50_ms"], "p99_call_ms": st["call_p99_ms"],
                                  "p99_batch_ms": st["batch_p99_ms"], "mean_batch": st["checks"] / max(1, st["batches"])}
    out = {"metric": "permission checks/sec through the host-buffer boundary (kg_check_batch, PCIe included)",
           "value": host_rate, "unit": "checks/s", "n_gpus": n_dev, "steps": per * T, "warmup": T,
           "ms_per_step": el / per * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "u32", "data": "synthetic (device-generated Drive-like tuple graph, seed %d)" % a.seed,
           "config": {"workload": "C2/C4 generator @ %.3g tuples, %d-check host batches, %d caller threads, "
                                  "max_read_depth %d" % (a.tuples, B, T, a.global_depth),
                      "replicas": devices, "parallelism": "replicas in one process"},
           "p50_call_ms": float(np.percentile(np.array(lat) * 1e3, 50)),
           "p99_call_ms": float(np.percentile(np.array(lat) * 1e3, 99)),
           "batcher": batcher, "snapshot_build_s": t_build}
    print(json.dumps(out), flush=True)


# rows per unit of the generator's size parameter (kg_synth.h: out-degree laws truncated at 1e5), measured at
# 1e9 (preset 0: 945,129,335 rows; preset 1: ~1.34e9) and 2e6 (--heavy-tail: 239,847,864)
ROWS_PER_T = {(0, False): 0.94513, (1, False): 1.3400, (0, True): 119.92, (1, True): 119.92}


def pack_queries_device(dq):
    """kg_pack_query (include/ketogpu.h) over an (n, 7) int32 kg_query tensor on the device: (n, 4) int32
    kg_query_packed rows (the bit layout of keto_amd._lib.pack_queries, which tests pin to the header)."""
    import torch
    q = dq.to(torch.int64) & 0xFFFFFFFF
    ns, obj, rel, sns, sobj, srel, d = (q[:, j] for j in range(7))
    sid = sns == 0xFFFFFFFF
    assert bool((ns <= 4094).all()) and bool((rel <= 4094).all()) and bool(((sns <= 4094) | sid).all()), \
        "ids do not fit kg_query_packed"
    snsp = torch.where(sid, torch.full_like(sns, 4095), sns)
    srelp = torch.where(sid, torch.zeros_like(srel), srel)
    dd = torch.where(d >= 0x80000000, torch.zeros_like(d), d).clamp(0, 65535)  # a negative depth is 0
    w2 = ns | (rel << 12) | ((snsp & 0xFF) << 24)
    w3 = (snsp >> 8) | (srelp << 4) | (dd << 16)
    out = torch.stack([obj, sobj, w2, w3], 1)
    return torch.where(out >= 0x80000000, out - (1 << 32), out).to(torch.int32).contiguous()


def build_synthetic(a, target_rows: float, **kw):
    """Snapshot.synthetic sized so that it holds at least `target_rows` rows: the generator's size
    parameter is the row target over the measured rows-per-parameter ratio (+0.2 %), and a build that
    still falls short is rebuilt once with the ratio it measured (a build is ~1.4 s at 1e9)."""
    from keto_amd.engine import Snapshot
    ratio = ROWS_PER_T[(a.preset, bool(a.heavy_tail))]
    shard = kw.get("shard")
    for _ in range(2):
        T = int(target_rows / ratio * 1.002) + 1
        snap = Snapshot.synthetic(T, seed=a.seed, preset=a.preset, **kw)
        rows = snap.info()["rows"]
        if shard is not None or rows >= target_rows:
            return snap, T
        ratio = rows / T
        snap.close()
    raise RuntimeError(f"synthetic graph holds {rows} rows, below the {target_rows:.3g} target")


def effective_cpus() -> dict:
    """CPUs this process can actually use: the affinity mask, capped by the cgroup CPU quota
    (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us) -- the GPU box's cgroup allows 16 of 256."""
    ncpu = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = ncpu
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    eff = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return {"nproc": ncpu, "affinity": aff, "cgroup_quota": quota, "effective": eff}


def aggregate(dist, elapsed: float, edges: float, device=None):
    """Whole-job numbers over ranks: elapsed = MAX over ranks (the job ends with its slowest
    rank), edges = SUM.  Replicas exchange nothing else."""
    if dist is None:
        return elapsed, edges
    import torch
    t = torch.tensor([elapsed, -edges], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    e = torch.tensor([edges], dtype=torch.float64, device=device)
    dist.all_reduce(e, op=dist.ReduceOp.SUM)
    return float(t[0].item()), float(e[0].item())


def spawn_ranks(a, argv) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: this process becomes a launcher that never
    touches the GPU.  It starts N children -- this script with the same arguments and RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, one per GPU, the environment torch.distributed.run
    gives its workers -- forwards rank 0's stdout (its one JSON line), and exits non-zero if any rank
    fails (the other ranks are then killed: they would wait in a collective forever)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    chunks = []  # rank 0's stdout, read beside the wait loop (a failed rank must not block the launcher)
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            c = p.poll()
            if c is None:
                continue
            pending.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in pending:  # exact children of this launcher
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    reader.join(30)
    out = b"".join(chunks).decode(errors="replace")
    sys.stdout.write(out)
    sys.stdout.flush()
    return rc


def bench_rehearse(a):
    """--mode rehearse: the multi-rank contract without a GPU -- every rank joins a gloo group, times K
    empty steps between barriers and reports fixed per-rank work; rank 0 prints the JSON line of the
    whole job (max elapsed over ranks, work summed), as the GPU modes do."""
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist.barrier()
    t = time.perf_counter()
    units = float(a.batch * a.steps)
    if world > 1:
        dist.barrier()
    elapsed, total = aggregate(dist if world > 1 else None, time.perf_counter() - t, units)
    if rank == 0:
        print(json.dumps({"metric": "rehearsal (no GPU)", "value": total / max(elapsed, 1e-9), "unit": "units/s",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "units": total,
                          "config": {"parallelism": f"replica{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and a.mode != "host":
        # no launcher around us: become one (one process per GPU; host mode spans the GPUs in-library)
        sys.exit(spawn_ranks(a, sys.argv[1:]))
    if a.mode == "rehearse":
        return bench_rehearse(a)
    if a.hw_queues > 0:  # before anything initialises HIP (torch and the library load lazily)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, a.hw_queues))
    if a.mode == "expand":
        return bench_expand(a)
    if a.mode == "sharded":
        return bench_sharded(a)
    if a.mode == "host":
        return bench_host(a)
    if a.mode == "refresh":
        return bench_refresh(a)
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    n_dev = max(1, torch.cuda.device_count())
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL; more ranks than GPUs (a rehearsal of the N-rank launch on a smaller
    # box) share GPUs and aggregate over gloo -- RCCL takes one rank per GPU
    backend = "nccl" if world <= n_dev else "gloo"
    local %= n_dev
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, rank=rank, world_size=world)
    torch.cuda.set_device(local)

    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    L = _lib.load()

    t_build = time.time()
    alpha = 0.5 if a.heavy_tail else 0.0
    snap, size_param = build_synthetic(a, a.tuples, device=local, doc_alpha=alpha, group_alpha=alpha)
    apply_tune(snap, a)
    info = snap.info()
    t_build = time.time() - t_build
    free_after_build = torch.cuda.mem_get_info(local)[0]

    B = a.batch
    P = max(1, a.inflight)
    dev = f"cuda:{local}"
    # P batches in flight: P host threads, each driving its own HIP stream (own workspace) with its
    # own result buffers (ctypes releases the GIL).  Every step checks a DISTINCT synthetic batch
    # (warm-up and timed steps alike), so no batch re-touches rows and probe lines a previous step
    # already pulled into L2 / the Infinity Cache.
    streams = inflight_streams(local, P + a.stream_base)[a.stream_base:]  # --stream-base: diagnostics
    warm = max(a.warmup, P)  # every stream's workspace is allocated before the timed region
    n_batches = warm + a.steps
    n_distinct = min(n_batches, a.replay) if a.replay > 0 else n_batches
    dq_all = torch.empty((n_distinct, B, 7), dtype=torch.int32, device=dev)
    for k in range(n_distinct):
        _lib.check(L.kg_synth_queries(snap.handle, 1000 + rank + 7919 * k, B, dq_all[k].data_ptr()),
                   "kg_synth_queries")
    douts = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(P)]
    derrs = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P)]
    dq = dq_all[warm % n_distinct]
    timed_out = torch.empty((a.steps, B), dtype=torch.uint8, device=dev)
    # --packed: the same queries as 16-B kg_query_packed rows (kg_pack_query, on the device)
    dp_all = None
    if a.packed:
        # packed by the library on the snapshot's own stream (kg_synth_queries' stream): no torch kernel or
        # copy touches a stream before the in-flight streams' first batches, which would shift the HIP
        # hardware queues they are bound to at their first launch
        dp_all = torch.empty((n_distinct, B, 4), dtype=torch.int32, device=dev)
        for k in range(n_distinct):
            _lib.check(L.kg_pack_queries_device(snap.handle, dq_all[k].data_ptr(), B, dp_all[k].data_ptr(), None),
                       "kg_pack_queries_device")
    check_fn = L.kg_check_batch_packed_device if a.packed else L.kg_check_batch_device
    qbatch = (lambda k: dp_all[k % n_distinct]) if a.packed else (lambda k: dq_all[k % n_distinct])

    # every pointer a step passes is taken here, once: a step's only Python work is the ctypes call itself
    # (tensor views and data_ptr() per call were ~20 us of GIL-held work between a caller's batches)
    q_ptrs = [qbatch(k).data_ptr() for k in range(n_batches)]
    o_ptrs = [timed_out[k - warm].data_ptr() if k >= warm else None for k in range(n_batches)]
    d_outp = [t.data_ptr() for t in douts]
    e_ptrs = [t.data_ptr() for t in derrs]
    s_ptrs = [C.c_void_p(st.cuda_stream) for st in streams]
    c_name = "kg_check_batch_packed_device" if a.packed else "kg_check_batch_device"

    def step(p, k, st=None):
        o = o_ptrs[k] if k >= warm else d_outp[p]  # every timed batch keeps its own results
        rc = check_fn(snap.handle, q_ptrs[k], B, a.global_depth, o, e_ptrs[p], C.byref(st) if st is not None else None,
                      s_ptrs[p])
        if rc:
            _lib.check(rc, c_name)

    def run_steps(k0, K, stats=None, lat=None):
        """Starts P host threads that run steps k0 .. k0+K-1 round-robin over the P streams once `go` is set."""
        go = threading.Event()
        errors = []

        def worker(p):
            try:
                go.wait()
                for k in range(p, K, P):
                    s0 = time.perf_counter()
                    step(p, k0 + k, stats[k] if stats is not None else None)  # stats => waits for its batch
                    if lat is not None:
                        lat[k] = time.perf_counter() - s0
                streams[p].synchronize()
            except Exception as e:  # noqa: BLE001 -- re-raised on the main thread
                errors.append(e)

        th = [threading.Thread(target=worker, args=(p,)) for p in range(min(P, max(K, 1)))]
        for t in th:
            t.start()
        return go, th, errors

    def finish(th, errors):
        for t in th:
            t.join()
        if errors:
            raise errors[0]

    go, th, errs = run_steps(0, warm)
    go.set()
    finish(th, errs)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # kernel stats (tier counts, in-kernel work counters, HIP-event kernel times) of every
    # `stats_every`-th timed batch (every kg_check_batch_device call waits for its batch anyway)
    stats = [_lib.kg_stats() if k % max(1, a.stats_every) == 0 else None for k in range(a.steps)]
    lat = [0.0] * a.steps
    go, th, errs = run_steps(warm, a.steps, stats, lat)
    t0 = time.perf_counter()
    go.set()
    finish(th, errs)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    res = timed_out.cpu().numpy()
    errs = torch.cat(derrs).cpu().numpy()
    assert (errs == 0).all() and (res <= 1).all(), "unexpected errors in the synthetic batch"
    stats = [x for x in stats if x is not None]
    elapsed, edges = aggregate(dist, elapsed, float(sum(s.edges_read for s in stats)) * a.steps / len(stats),
                               f"cuda:{local}" if backend == "nccl" else None)
    tag = "h" if a.heavy_tail else ""
    rf_stream = stream_roofline(stats, pmc_traffic(STREAM_KERNEL, int(a.tuples), B, a.preset, P, tag))
    # the tail tier's level launches are timed one by one (kg_snapshot_tune "level_events") in a stats phase
    # of their own after the timed region: an event pair per launch leaves gaps in the stream
    level_events(snap, 1)
    n_t = min(2 * P, warm)  # warm-up batch indices: their results go to the scratch outputs, not timed_out
    tstats = [_lib.kg_stats() for _ in range(n_t)]
    go, th, errs_t = run_steps(0, n_t, tstats)
    go.set()
    finish(th, errs_t)
    torch.cuda.synchronize()
    level_events(snap, 0)
    rf_tail = tail_roofline(tstats, lambda k: pmc_traffic(k, int(a.tuples), B, a.preset, P, tag))
    # the headline keeps k_stream4's roofline (its kernel since round 1); the heavy-tail point reports its
    # dominant kernel by device time per batch (k_ms_level); every measured kernel is in "rooflines"
    rf_main = dominant(rf_stream, rf_tail) if a.heavy_tail else rf_stream

    # ---- latency phase (outside the timed region): the same P batches in flight, every batch waited for
    # (submit -> results on the host side of the stream), distinct query batches
    lat_n = max(0, a.latency_batches)
    lat_ms = []
    if lat_n:
        n_ld = min(lat_n, 64)
        dq_lat = torch.empty((n_ld, B, 7), dtype=torch.int32, device=dev)
        for k in range(n_ld):
            _lib.check(L.kg_synth_queries(snap.handle, 500000 + rank + 7919 * k, B, dq_lat[k].data_ptr()),
                       "kg_synth_queries")
        if a.packed:
            dp_lat = torch.empty((n_ld, B, 4), dtype=torch.int32, device=dev)
            for k in range(n_ld):
                _lib.check(L.kg_pack_queries_device(snap.handle, dq_lat[k].data_ptr(), B, dp_lat[k].data_ptr(), None),
                           "kg_pack_queries_device")
            dq_lat = dp_lat
        lat = [0.0] * lat_n
        errors = []

        def lat_worker(p):
            try:
                st = _lib.kg_stats()
                for k in range(p, lat_n, P):
                    s0 = time.perf_counter()
                    _lib.check(check_fn(snap.handle, dq_lat[k % n_ld].data_ptr(), B, a.global_depth,
                                        douts[p].data_ptr(), derrs[p].data_ptr(), C.byref(st),
                                        C.c_void_p(streams[p].cuda_stream)), "check (latency phase)")
                    lat[k] = time.perf_counter() - s0  # a batch with stats returns once its results are in
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        th = [threading.Thread(target=lat_worker, args=(p,)) for p in range(P)]
        torch.cuda.synchronize()
        t_lat = time.perf_counter()
        [t.start() for t in th]
        [t.join() for t in th]
        torch.cuda.synchronize()
        lat_wall = time.perf_counter() - t_lat
        if errors:
            raise errors[0]
        lat_ms = np.array(lat) * 1e3
        del dq_lat
    # ---- host path: the same engine through kg_check_batch (host buffers, H2D + tiers + D2H)
    host = host_path(L, snap, dq_all, n_distinct, a, P) if a.host_calls > 0 else None

    value = world * B * a.steps / elapsed
    out = {
        "metric": "permission checks/sec (batched check, synthetic Drive-like graph)",
        "value": value,
        "unit": "checks/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": warm,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device-generated Drive-like tuple graph, seed %d)" % a.seed,
        "config": {"workload": "%s generator @ %.4g tuples (rows), %d checks/step/GPU, max_read_depth %d"
                               % ("C2/C4" if a.preset == 0 else "C3 (OPL view/edit/share)", info["rows"], B,
                                  a.global_depth) + (", out-degree law P(k)~k^-1.5" if a.heavy_tail else
                                  "; out-degrees truncated Pareto, tail index 1.3 (docs) / 1.1 (groups), "
                                  "mean ~4-10 per row (SURVEY.md 8d's Zipf 1.5 is the heavy sub-line); "
                                  "doc roots uniform (not Zipf popularity); positives by forward random walks"),
                   "tuples": info["rows"], "tuples_target": a.tuples, "generator_size_param": size_param,
                   "nodes": info["nodes"], "set_edges": info["set_edges"],
                   "batch_per_gpu": B, "global_max_read_depth": a.global_depth, "parallelism": f"replica{world}",
                   "inflight_per_gpu": P, "queries": ("16-B kg_query_packed, kg_check_batch_packed_device" if a.packed else "28-B kg_query, kg_check_batch_device"), "device_gb": info["device_bytes"] / 1e9,
                   "hbm_free_gb_after_build": free_after_build / 1e9,
                   "materialized": snap.materialized(), "tune": dict(snap.__dict__.get("tuned", {}))},
        "gteps": edges / elapsed / 1e9,
        "p99_batch_ms": float(np.percentile(lat_ms, 99)) if lat_n else None,
        # the latency phase is a second, longer throughput sample of the same workload (distinct batches,
        # same batches in flight, every batch waited for): the timed region alone is only a few ms long
        "steady": ({"value": lat_n * B / lat_wall, "unit": "checks/s", "batches": lat_n, "seconds": lat_wall,
                    "what": "rank-0 checks/s over the latency phase (outside the timed region)"} if lat_n else None),
        "batch_ms": ({"batches": lat_n, "inflight": P, **{q: float(np.percentile(lat_ms, v)) for q, v in
                     (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))}} if lat_n else None),
        "edges_per_batch": {q: float(np.percentile([x.edges_read for x in stats], v)) for q, v in
                            (("p50", 50), ("p90", 90), ("max", 100))},
        "allowed_fraction": float(res.mean()),
        "tiers": {"light": int(stats[-1].n_light),
                  "back": int(stats[-1].n_back), "grid": int(stats[-1].n_grid), "heavy": int(stats[-1].n_heavy),
                  "general": int(stats[-1].n_general), "no_holder": int(stats[-1].n_no_holder)},
        "work_per_batch": {"light": {"rows": int(stats[-1].light_rows_opened), "edges": int(stats[-1].light_edges_read),
                                     "probes": int(stats[-1].light_probes)},
                           "all": {"rows": int(stats[-1].rows_opened), "edges": int(stats[-1].edges_read),
                                   "probes": int(stats[-1].direct_probes)},
                           "back": {"rows": int(stats[-1].back_rows), "edges": int(stats[-1].back_edges)}},
        "stream_diag": stream_diag(stats[-1]),
        "snapshot_build_s": t_build,
        "roofline": rf_main,
        "rooflines": {r["kernel"]: r for r in (rf_stream, rf_tail) if r},
        "host_path": host,
    }
    orc = None
    if rank == 0:
        if a.parity > 0 or (world == 1 and a.cpu_seconds > 0):
            cpus = effective_cpus()
            orc = CheckOracle(snap, a, cpus["effective"])
            q0 = dq.cpu().numpy().view(np.uint32)
        if a.parity > 0:
            out["parity"] = orc.parity(q0, res[0], a.parity, a.parity_canonical)
        if world == 1 and a.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(orc, q0, a, cpus)
    bad = a.parity > 0 and rank == 0 and out["parity"]["mismatches"] + out["parity"]["canonical_mismatches"]
    # the other configurations beside the headline, on the driver's own runs (C3 and C5 had
    # builder-run numbers only): one rank -- C5 expand over the headline graph, C3 at its config size;
    # every rank -- the hash-sharded C4 engine (item 1).  A watchdog keeps a hung collective from costing
    # the whole line: rank 0 then prints it without the unfinished sub-line.
    current = [None]

    def on_timeout():
        if rank == 0:
            out[current[0] or "sub_lines"] = {"error": "did not finish within %.0f s" % a.sharded_timeout}
            print(json.dumps(out), flush=True)
        os._exit(1 if bad else 0)

    def sub_line(name, fn):
        current[0] = name
        wd = threading.Timer(a.sharded_timeout, on_timeout)
        wd.daemon = True
        wd.start()
        try:
            out[name] = fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line; the replica headline stands
            out[name] = {"error": f"{type(e).__name__}: {e}"}
        wd.cancel()
        subs = [out[name]] + [v for v in out[name].values() if isinstance(v, dict)]
        return any(x["parity"]["mismatches"] + x["parity"].get("canonical_mismatches", 0)
                   for x in subs if isinstance(x.get("parity"), dict) and "mismatches" in x["parity"])

    if world == 1 and a.preset == 0 and not a.heavy_tail and a.expand_steps > 0:
        bad = sub_line("expand", lambda: expand_leg(a)) or bad
    if world == 1 and a.preset == 0 and not a.heavy_tail and a.c3_steps > 0:
        bad = sub_line("c3", lambda: c3_leg(a, local)) or bad
    if world == 1 and a.preset == 0 and not a.heavy_tail and a.heavy_steps > 0:
        bad = sub_line("heavy", lambda: heavy_leg(a)) or bad
    if a.sharded_steps > 0 and a.preset == 0 and not a.heavy_tail:
        bad = sub_line("sharded", lambda: sharded_leg(a, snap, size_param, dist, rank, world, local, backend, orc)) or bad
    if rank == 0:
        print(json.dumps(out), flush=True)
        if bad:
            sys.stderr.write("PARITY FAILURE: GPU answers differ from the oracle\n")
            if dist:
                dist.destroy_process_group()
            sys.exit(1)
    if dist:
        dist.destroy_process_group()


def expand_leg(a) -> dict:
    """Config C5 (BASELINE.json configs[4]) beside the headline: BuildTree of the --roots most popular
    group#member sets of the headline's generator graph at the global max_read_depth 5, as a
    child `bench.py --mode expand` run on the same GPU (the parent idles): --expand-inflight callers, each on
    a HIP stream of its own through kg_expand_batch_device (roots and trees in HBM), --expand-steps calls in
    the timed region, 32 hardware queues (the parent keeps 16, which C3 and the sharded lines need); the
    host-buffer call (PCIe both ways) is reported beside it; roofline of the expand chain, parity against
    the oracle's BuildTree (the 10 largest roots + a sample) and a CPU baseline."""
    import subprocess
    P = max(1, a.expand_inflight)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mode", "expand", "--inflight", str(P),
           "--steps", str(a.expand_steps), "--warmup", str(P), "--cpu-seconds", str(a.cpu_seconds / 3),
           "--parity-roots", str(a.parity_roots), "--roots", str(a.roots), "--hw-queues", "32",
           "--tuples", str(a.tuples), "--seed", str(a.seed), "--expand-gw", str(a.expand_gw)]
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        env.pop(k, None)
    t0 = time.time()
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=max(60.0, a.sharded_timeout - 20))
    lines = [x for x in r.stdout.decode(errors="replace").splitlines() if x.startswith("{")]
    if not lines:
        raise RuntimeError("expand run printed no line (rc %d): %s" % (r.returncode, r.stderr.decode(errors="replace")[-600:]))
    d = json.loads(lines[-1])
    keep = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "config", "io", "host_path", "tree_nodes_per_s",
            "tree_nodes_per_step", "kernel_ms_per_step", "records_per_root", "largest_root", "roofline", "parity",
            "cpu_baseline")
    res = {k: d[k] for k in keep if k in d}
    res["metric"] = "expand trees/sec (C5: batched BuildTree, hot group#member roots)"
    res["inflight"] = P
    res["child"] = {"cmd": " ".join(cmd[1:]), "rc": r.returncode, "seconds": time.time() - t0}
    return res


def heavy_leg(a) -> dict:
    """SURVEY.md 8d's literal degree law beside the headline: the heavy-tail point
    (out-degrees P(k) ~ k^-1.5, 1.2e8 tuples, 62.5 k checks per batch, 4 in flight -- its p99 point,
    DESIGN.md 7f) as a child `bench.py --heavy-tail` run on the same GPU (the parent idles meanwhile), with
    its own timed region, latency phase, parity against the oracle, CPU baseline and the roofline of its
    dominant kernel (k_ms_level, HIP events per launch)."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--heavy-tail", "--steps", str(a.heavy_steps), "--warmup", "4",
           "--cpu-seconds", str(a.cpu_seconds / 3), "--parity", str(a.heavy_parity), "--parity-canonical",
           str(min(a.heavy_parity, 10_000)), "--latency-batches", "120", "--host-calls", "0",
           "--hw-queues", str(a.hw_queues), "--seed", str(a.seed), "--global-depth", str(a.global_depth)]
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        env.pop(k, None)
    t0 = time.time()
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=max(60.0, a.sharded_timeout - 20))
    lines = [x for x in r.stdout.decode(errors="replace").splitlines() if x.startswith("{")]
    if not lines:
        raise RuntimeError("heavy-tail run printed no line (rc %d): %s" % (r.returncode, r.stderr.decode(errors="replace")[-600:]))
    d = json.loads(lines[-1])
    keep = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "config", "gteps", "p99_batch_ms", "steady",
            "batch_ms", "edges_per_batch", "allowed_fraction", "tiers", "work_per_batch", "snapshot_build_s",
            "roofline", "rooflines", "parity", "cpu_baseline")
    res = {k: d[k] for k in keep if k in d}
    res["config"]["workload"] += ("; popularity: doc roots uniform (not Zipf), positives by forward random walks, "
                                  "out-degrees Pareto tail index 0.5 for docs and groups")
    res["child"] = {"cmd": " ".join(cmd[1:]), "rc": r.returncode, "seconds": time.time() - t0}
    return res


def c3_leg(a, local) -> dict:
    """Config C3 (BASELINE.json configs[2]: the generator graph at --c3-tuples, default its 10M, plus the
    folder forest and the OPL namespace view / edit / share) beside the headline: 1 M checks per batch
    through kg_check_batch_device, --c3-inflight batches in flight (C3's occupancy set: stream_wgs 3,
    grid_wgs 4, back_wgs 1), distinct batches, parity of the first timed batch against the oracle
    evaluating the program (Go-order DFS + canonical policy)."""
    import copy
    import torch
    from keto_amd import _lib
    L = _lib.load()
    a3 = copy.copy(a)
    a3.preset, a3.stream_wgs, a3.grid_wgs, a3.back_wgs = 1, 3, 4, 1
    t0 = time.time()
    snap3, _ = build_synthetic(a3, a.c3_tuples, device=local)
    apply_tune(snap3, a3)
    t_build = time.time() - t0
    dev = f"cuda:{local}"
    B, P, K = a.batch, max(1, a.c3_inflight), a.c3_steps
    W = P
    streams = inflight_streams(local, P)
    dqs = []
    for k in range(W + K):
        d = torch.empty((B, 7), dtype=torch.int32, device=dev)
        _lib.check(L.kg_synth_queries(snap3.handle, 700000 + 7919 * k, B, d.data_ptr()), "kg_synth_queries")
        dqs.append(d)
    outs = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(W + K)]
    errs = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P)]
    NS = 2 * P  # the stats phase (after the timed region): every batch with kernel stats, same P in flight
    sts = [_lib.kg_stats() for _ in range(NS)]

    def phase(k0, n, with_stats=False):
        errors = []

        def worker(p):
            try:
                for k in range(p, n, P):
                    kk = (k0 + k) % (W + K)
                    _lib.check(L.kg_check_batch_device(snap3.handle, dqs[kk].data_ptr(), B, a.global_depth,
                                                       outs[kk].data_ptr(), errs[p].data_ptr(),
                                                       C.byref(sts[k]) if with_stats else None,
                                                       C.c_void_p(streams[p].cuda_stream)), "kg_check_batch_device")
                streams[p].synchronize()
            except Exception as x:  # noqa: BLE001
                errors.append(x)

        th = [threading.Thread(target=worker, args=(p,)) for p in range(min(P, n))]
        [t.start() for t in th]
        [t.join() for t in th]
        if errors:
            raise errors[0]

    phase(0, W)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    phase(W, K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t1
    assert (torch.cat(errs).cpu().numpy() == 0).all(), "unexpected errors in the synthetic C3 batch"
    r0 = outs[W].cpu().numpy()
    q0 = dqs[W].cpu().numpy().view(np.uint32)
    level_events(snap3, 1)  # the tail tier's launches timed one by one (outside the timed region)
    phase(0, NS, with_stats=True)  # batches 0 .. NS-1 again (their results are not read)
    torch.cuda.synchronize()
    level_events(snap3, 0)
    st = sts[0]
    tr = lambda k: pmc_traffic(k, int(a.c3_tuples), B, 1, P)
    rf_stream = stream_roofline(sts, tr(STREAM_KERNEL))
    rf_tail = tail_roofline(sts, tr)
    res = {"metric": "permission checks/sec (C3: OPL view/edit/share rewrites)", "value": B * K / el,
           "unit": "checks/s", "steps": K, "inflight": P, "ms_per_step": el / K * 1e3,
           "config": {"workload": "C3 generator @ %.4g tuples (rows), %d checks/step, max_read_depth %d"
                                  % (snap3.info()["rows"], B, a.global_depth),
                      "materialized": snap3.materialized(), "tune": dict(snap3.__dict__.get("tuned", {}))},
           "allowed_fraction": float(r0.mean()), "snapshot_build_s": t_build,
           "tiers": {"light": int(st.n_light), "back": int(st.n_back), "grid": int(st.n_grid),
                     "general": int(st.n_general), "no_holder": int(st.n_no_holder)},
           # the dominant kernel by device time per batch (HIP events of a separate stats phase: every batch
           # waited for, same batches in flight); every measured kernel in "rooflines"
           "roofline": dominant(rf_stream, rf_tail),
           "rooflines": {r["kernel"]: r for r in (rf_stream, rf_tail) if r},
           "kernel_ms_per_batch": {"k_fsplit": float(np.mean([s.split_ms for s in sts])),
                                   "k_stream4": rf_stream["ms_per_batch"],
                                   **({rf_tail["kernel"]: rf_tail["ms_per_batch"]} if rf_tail else {}),
                                   "batch_span": float(np.mean([s.kernel_ms for s in sts]))},
           "stats_batches": NS}
    if a.c3_parity > 0 or a.cpu_seconds > 0:
        cpus = effective_cpus()
        orc3 = CheckOracle(snap3, a3, cpus["effective"])
        if a.c3_parity > 0:
            res["parity"] = orc3.parity(q0, r0, a.c3_parity, min(a.parity_canonical, a.c3_parity))
        if a.cpu_seconds > 0:  # a bounded sample: a third of the headline's CPU budget
            a3.cpu_seconds = a.cpu_seconds / 3
            res["cpu_baseline"] = cpu_baseline(orc3, q0, a3, cpus)
        orc3.o.close()
    snap3.close()
    return res


_STREAMS = {}


def inflight_streams(local: int, P: int) -> list:
    """The process's batches-in-flight streams on device `local`, created once and shared by the headline
    and the sub-lines (the current stream first, as the headline always used it)."""
    import torch
    v = _STREAMS.setdefault(local, [torch.cuda.current_stream(local)])
    while len(v) < P:
        v.append(torch.cuda.Stream(local))
    return v[:P]


def sharded_leg(a, snap, size_param, dist, rank, world, local, backend, orc) -> dict:
    """Config C4 hash-sharded (BASELINE.json configs[3]) beside the replica headline: rank r
    holds only the rows of the objects hash(ns, obj) mod N == r of the same generator graph, and every
    batch runs inside kg_check_batch_device over the rank's RCCL communicator (kg_shard_comm.hip: seed,
    gdepth + 1 exchanges of per-destination buckets, done-bitmap all-gathers, two host round trips) --
    the path a Go host drives.  Queries are the headline's kind (drawn from the full
    graph), B per rank per step, --sharded-inflight batches in flight per rank (one stream +
    communicator each).  One rank holds every row: its shard IS the replica snapshot, the batch runs
    local-first (the replica tier chain, `path`), and `exchange` times the same batches through the N > 1
    exchange protocol over RCCL anyway (kg_snapshot_tune shard_force_exchange: self send / recv), the
    baseline of the N-rank curve.  Weak scaling; value = all ranks' checks / max-over-ranks time."""
    import torch
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    from keto_amd.sharded import LibShardedChecker
    L = _lib.load()
    dev = f"cuda:{local}"
    t0 = time.time()
    if world == 1:
        ssnap = snap  # one rank: its shard is the whole graph, i.e. the replica snapshot itself
    else:
        alpha = 0.5 if a.heavy_tail else 0.0
        ssnap = Snapshot.synthetic(size_param, seed=a.seed, device=local, shard=(rank, world), preset=a.preset,
                                   doc_alpha=alpha, group_alpha=alpha)
        ssnap.tune("shard_remote_meta", a.shard_remote_meta)  # applied when the checkers bind below
    t_build = time.time() - t0
    transport = "rccl" if backend == "nccl" else "host"
    P = a.sharded_inflight if a.sharded_inflight > 0 else (3 if world == 1 else 1)
    groups = [None] * P
    if dist is not None and P > 1:
        groups = [dist.new_group(list(range(world))) for _ in range(P)]
    # the headline's streams: HIP maps streams onto its hardware queues (4 by default) round-robin as they
    # are created, so fresh streams here could share queues with each other and serialise.  Not the
    # current (null) stream: a transport bound to it would catch the library's null-stream calls.
    streams = inflight_streams(local, P + 1)[1:]
    chks = [LibShardedChecker(ssnap, rank, world, dist, group=groups[p], transport=transport, stream=streams[p])
            for p in range(P)]
    B, K, W = a.sharded_batch or a.batch, a.sharded_steps, max(a.sharded_warmup, P)
    dqs = []
    for k in range(W + K):  # distinct batches, drawn from the full graph (the replica snapshot)
        d = torch.empty((B, 7), dtype=torch.int32, device=dev)
        _lib.check(L.kg_synth_queries(snap.handle, 900000 + rank + 7919 * k, B, d.data_ptr()), "kg_synth_queries")
        dqs.append(d)

    res_k = torch.empty((K, B), dtype=torch.uint8, device=dev)  # every timed batch keeps its own results
    err_p = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(P)]
    res_p = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(P)]
    torch.cuda.synchronize()  # queries and buffers exist before the checkers' streams use them

    def run_phase(k0, n, lat=None, timed=False):
        """Batches k0 .. k0+n-1 round-robin over the P checkers.  Throughput phases enqueue back to back
        (each thread synchronises its stream once at the end); `lat` phases wait for every batch."""
        errors = []
        nth = min(P, max(n, 1))
        ready = threading.Barrier(nth + 1)  # threads exist before the clock starts (as the headline's `go`)

        def worker(p):
            try:
                c = chks[p]
                ready.wait()
                for k in range(p, n, P):
                    # what a Go host calls: kg_check_batch_device on the stream the communicator is bound to
                    s0 = time.perf_counter()
                    o = res_k[k] if timed else res_p[p]
                    c._check_t(L.kg_check_batch_device(ssnap.handle, dqs[k0 + k].data_ptr(), B, a.global_depth,
                                                       o.data_ptr(), err_p[p].data_ptr(), None, c._sp),
                               "kg_check_batch_device (sharded)")
                    if lat is not None:
                        c.stream.synchronize()
                        lat[k] = time.perf_counter() - s0
                c.stream.synchronize()
            except Exception as x:  # noqa: BLE001 -- re-raised below
                errors.append(x)
                ready.abort()

        th = [threading.Thread(target=worker, args=(p,)) for p in range(nth)]
        [t.start() for t in th]
        try:
            ready.wait()
        except threading.BrokenBarrierError:
            pass
        t_go = time.perf_counter()
        [t.join() for t in th]
        if errors:
            raise errors[0]
        return t_go

    def measure(tag):
        run_phase(0, W)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = run_phase(W, K, timed=True)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        el, _ = aggregate(dist, time.perf_counter() - t1, 0.0, dev if backend == "nccl" else None)
        st = chks[0].stats()
        lv = chks[0].levels()
        r0 = res_k[0].cpu().numpy()
        e_all = torch.stack(err_p).cpu().numpy()
        assert (e_all == 0).all() and (res_k <= 1).all().item(), "unexpected errors in the synthetic batch"
        # latency: after the throughput phase, KL more batches at the same in-flight depth, each waited for
        # by its thread (enqueue -> results on the host)
        KL = min(K, max(P, 8))
        lat = [0.0] * KL
        if dist:
            dist.barrier()
        run_phase(0, KL, lat)
        res = {"value": world * B * K / el, "unit": "checks/s", "steps": K, "warmup": W, "inflight": P,
               "ms_per_step": el / K * 1e3, "p99_batch_ms": float(np.percentile(np.array(lat) * 1e3, 99)),
               "p50_batch_ms": float(np.percentile(np.array(lat) * 1e3, 50)),
               "latency_batches": KL,
               "path": LibShardedChecker.PATHS.get(st["path"], st["path"]),
               "levels_per_batch": st["levels"], "host_syncs_per_batch": st["host_syncs"],
               "exchanges_per_batch": st["exchanges"], "exchange_reruns": st["exchange_reruns"],
               "records_sent_per_batch": st["records_sent"], "records_to_peers_per_batch": st["records_to_peers"],
               "wire_bytes_per_batch": st["wire_bytes"], "reruns_last_batch": st["reruns_bucket"] + st["reruns_visited"],
               "allowed_fraction": float(r0.mean())}
        if lv:  # per exchange: B_k (records per destination on the wire) and the largest bucket it needed
            res["exchanges"] = [{"bucket": b, "largest": m, "wire_bytes": (world - 1) * (4 + 16 * b)} for b, m in lv]
            res["padding_fraction"] = 1.0 - sum(m for _, m in lv) / max(1, sum(b for b, _ in lv))
        if rank == 0 and orc is not None and a.parity > 0:
            res["parity"] = orc.parity(dqs[W].cpu().numpy().view(np.uint32), r0, a.parity, a.parity_canonical)
            res["parity"]["batch"] = "rank 0's first timed sharded batch"
        return res

    out = {"metric": "permission checks/sec, hash-sharded (kg_check_batch_device, one shard per rank)",
           "n_gpus": world, "transport": "RCCL over xGMI" if transport == "rccl" else "host (gloo)",
           "config": {"workload": "C4: the headline's generator graph hash-sharded by object over %d rank(s), "
                                  "%d checks/step/rank, max_read_depth %d" % (world, B, a.global_depth),
                      "rows_on_rank": ssnap.info()["rows"], "parallelism": f"shard{world}",
                      "remote_meta": a.shard_remote_meta if world > 1 else None},
           "snapshot_build_s": t_build, "scaling": "weak"}
    out.update(measure("default"))
    if world == 1:
        ssnap.tune("shard_force_exchange", 1)
        try:
            out["exchange"] = measure("exchange")
        finally:
            ssnap.tune("shard_force_exchange", 0)
        out["exchange"]["what"] = ("the same batches through the N > 1 exchange protocol over a one-rank RCCL "
                                   "communicator (the N-rank curve's baseline)")
    for c in chks:
        c.close()
    if ssnap is not snap:
        ssnap.close()
    return out


def host_path(L, snap, dq_all, n_distinct, a, P) -> dict:
    """kg_check_batch (what the cgo binding calls) over 1 M-check HOST batches from P
    threads: H2D of the queries, the tier chain, D2H of results and error codes, all inside the call."""
    from keto_amd import _lib
    B = a.batch
    qs = [np.ascontiguousarray(dq_all[p % n_distinct].cpu().numpy().view(np.uint32)) for p in range(P)]
    lat, errors = [], []
    ready = threading.Barrier(P + 1)

    def worker(p):
        try:
            o = np.empty(B, np.uint8)
            e = np.empty(B, np.uint32)

            def call():
                _lib.check(L.kg_check_batch(snap.handle, qs[p].ctypes.data_as(C.c_void_p), B, a.global_depth,
                                            o.ctypes.data_as(C.c_void_p), e.ctypes.data_as(C.c_void_p), None),
                           "kg_check_batch")
            call()  # this thread's lane (stream, pinned staging, workspace) exists before timing
            ready.wait()
            for _ in range(a.host_calls):
                s0 = time.perf_counter()
                call()
                lat.append(time.perf_counter() - s0)
        except Exception as x:  # noqa: BLE001
            errors.append(x)
            ready.abort()

    th = [threading.Thread(target=worker, args=(p,)) for p in range(P)]
    [t.start() for t in th]
    ready.wait()
    t0 = time.perf_counter()
    [t.join() for t in th]
    el = time.perf_counter() - t0
    if errors:
        raise errors[0]
    ms = np.array(lat) * 1e3
    dense = {"value": B * a.host_calls * P / el, "unit": "checks/s", "callers": P, "calls": len(lat),
             "checks_per_call": B, "p50_call_ms": float(np.percentile(ms, 50)),
             "p99_call_ms": float(np.percentile(ms, 99)),
             "bytes_per_check": {"in": 28, "out": 5},
             "what": "kg_check_batch on 1 M-check host batches: PCIe both ways included (not the headline value)"}
    # the narrow boundary: kg_check_batch_packed (16-B queries in, 1-B answers out, error codes sparse),
    # every answer checked against the dense call's
    pks = [_lib.pack_queries(x) for x in qs]
    ref = []
    lat2, errors = [], []
    ready = threading.Barrier(P + 1)

    def worker2(p):
        try:
            o = np.empty(B, np.uint8)
            idx = np.empty(1024, np.uint32)
            code = np.empty(1024, np.uint32)
            ne = C.c_size_t(0)

            def call():
                _lib.check(L.kg_check_batch_packed(snap.handle, pks[p].ctypes.data_as(C.c_void_p), B, a.global_depth,
                                                   o.ctypes.data_as(C.c_void_p), idx.ctypes.data_as(C.c_void_p),
                                                   code.ctypes.data_as(C.c_void_p), 1024, C.byref(ne), None),
                           "kg_check_batch_packed")
            call()
            ready.wait()
            for _ in range(a.host_calls):
                s0 = time.perf_counter()
                call()
                lat2.append(time.perf_counter() - s0)
            ref.append((p, o.copy(), int(ne.value)))
        except Exception as x:  # noqa: BLE001
            errors.append(x)
            ready.abort()

    th = [threading.Thread(target=worker2, args=(p,)) for p in range(P)]
    [t.start() for t in th]
    ready.wait()
    t0 = time.perf_counter()
    [t.join() for t in th]
    el2 = time.perf_counter() - t0
    if errors:
        raise errors[0]
    # answers of the packed calls vs kg_check_batch on the same host batch
    o = np.empty(B, np.uint8)
    e = np.empty(B, np.uint32)
    mism = 0
    for p, got, ne in ref:
        _lib.check(L.kg_check_batch(snap.handle, qs[p].ctypes.data_as(C.c_void_p), B, a.global_depth,
                                    o.ctypes.data_as(C.c_void_p), e.ctypes.data_as(C.c_void_p), None), "kg_check_batch")
        mism += int((got != o).sum()) + abs(ne - int((o == 2).sum()))
    ms2 = np.array(lat2) * 1e3
    dense["packed"] = {"value": B * a.host_calls * P / el2, "unit": "checks/s", "callers": P, "calls": len(lat2),
                       "p50_call_ms": float(np.percentile(ms2, 50)), "p99_call_ms": float(np.percentile(ms2, 99)),
                       "bytes_per_check": {"in": 16, "out": 1}, "mismatches_vs_dense": mism,
                       "what": "kg_check_batch_packed (kg_query_packed in, answers + sparse error codes out)"}
    return dense


class CheckOracle:
    """The C restatement of the reference engine (oracle/keto_oracle.c) over the snapshot's own rows
    (kg_snapshot_export_csr, shard order), as the parity checker and the CPU baseline.  Preset 0 queries
    doc#viewer roots by node id (synthetic docs: node id == object id); preset 1 resolves (ns, obj, rel)
    through the oracle's own node map and evaluates the OPL program."""

    def __init__(self, snap, a, nthreads: int):
        from keto_amd import _lib
        from oracle.oracle import Oracle
        L = _lib.load()
        info = snap.info()
        nn, nr = info["nodes"], info["rows"]
        row_off = np.zeros(nn + 1, np.uint64)
        row_subj = np.zeros(nr, np.uint32)
        nd = [np.zeros(nn, np.uint32) for _ in range(3)]
        p = lambda x: x.ctypes.data_as(C.c_void_p)
        _lib.check(L.kg_snapshot_export_csr(snap.handle, p(row_off), p(row_subj), p(nd[0]), p(nd[1]), p(nd[2])),
                   "kg_snapshot_export_csr")
        self.by_node = a.preset == 0
        self.nd = nd  # node triples (the C5 expand parity's root check)
        t = time.perf_counter()
        self.o = Oracle.from_csr(0, nd[0], nd[1], nd[2], row_off, row_subj, with_node_map=not self.by_node,
                                 nthreads=min(nthreads, 64))
        if not self.by_node:
            self.o.set_program(snap.program)
        self.build_s = time.perf_counter() - t
        self.a = a
        self.nthreads = nthreads
        self.ids = snap.synth_ids()

    def run(self, q: np.ndarray, policy: int, nthreads: int) -> np.ndarray:
        dep = q[:, 6].view(np.int32)
        if self.by_node:
            assert (q[:, 3] == 0xFFFFFFFF).all() and (q[:, 1] < self.ids["n_docs"]).all(), "preset-0 batch shape"
            return self.o.check_nodes_batch(q[:, 1].copy(), q[:, 4].copy(), dep.copy(), self.a.global_depth, policy,
                                            nthreads)[0]
        return self.o.check_batch(q[:, :6], dep, self.a.global_depth, policy, nthreads)[0]

    def parity(self, q: np.ndarray, gpu: np.ndarray, n: int, n_canon: int) -> dict:
        """GPU answers of one timed batch vs the oracle: the Go-order DFS schedule on the first n checks
        and the schedule-free canonical policy on the first n_canon of them."""
        from oracle.oracle import POLICY_CANONICAL, POLICY_DFS
        n = min(n, len(q))
        t = time.perf_counter()
        dfs = self.run(q[:n], POLICY_DFS, self.nthreads)
        nc = min(n_canon, n)
        can = self.run(q[:nc], POLICY_CANONICAL, self.nthreads) if nc else np.zeros(0, np.uint8)
        bad = np.nonzero(dfs != gpu[:n])[0]
        return {"checks": int(n), "mismatches": int(bad.size), "canonical_checks": int(nc),
                "canonical_mismatches": int((can != gpu[:nc]).sum()),
                "schedule_variant": int((dfs[:nc] != can).sum()), "allowed": int((dfs == 1).sum()),
                "errors": int((dfs == 2).sum()), "first_mismatches": [int(i) for i in bad[:8]],
                "batch": "first timed batch (timed_out[0])", "oracle": "oracle/keto_oracle.c",
                "oracle_build_s": self.build_s, "seconds": time.perf_counter() - t}


def stream_diag(s) -> dict:
    """k_stream occupancy: wave steps (one HBM round trip each), edges per step, mean wave lifetime."""
    steps, waves = int(s.light_steps), int(s.light_waves)
    return {"steps": steps, "waves": waves, "edges_per_step": s.light_edges_read / steps if steps else 0.0,
            "steps_per_wave": steps / waves if waves else 0.0,
            "mean_wave_us": s.light_wave_ticks / waves / 100.0 if waves else 0.0,
            "max_wave_us": s.light_wave_max_ticks / 100.0, "span_us": s.light_span_ticks / 100.0}


TAIL_KERNELS = {1: "k_grid_level<0>", 2: "k_ms_level<8>"}


def stream_roofline(stats: list, traffic) -> dict:
    """k_stream4 (one launch per batch): the SURVEY.md 8d byte model over its in-kernel counters, per
    launch, against its HIP-event launch time."""
    b = np.array([8 * s.light_rows_opened + 4 * s.light_edges_read + 16 * s.light_probes for s in stats], float)
    r = np.array([s.light_rows_opened + s.light_probes for s in stats], float)
    ms = np.array([s.light_ms for s in stats], float)
    ach = float(b.mean() / (ms.mean() * 1e-3) / 1e9)
    rate = float(r.mean() / (ms.mean() * 1e-3))
    return {"kernel": STREAM_KERNEL, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
            "bytes_model": "8*rows_opened + 4*edges_read + 16*direct_probes (per k_stream launch; R/E/P counted in-kernel)",
            "launch_ms": float(ms.mean()), "bytes_per_launch": float(b.mean()), "launches_per_batch": 1,
            "ms_per_batch": float(ms.mean()),
            # the random-request view: one row open and one dset probe are one random line each;
            # ceiling = independent random 16-B loads/s measured by tools/randprobe.hip on MI355X
            "requests_per_launch": float(r.mean()), "request_rate": rate, "request_peak": RAND_REQ_PEAK,
            "request_frac": rate / RAND_REQ_PEAK}


def tail_roofline(stats: list, traffic_of) -> dict | None:
    """The tail tier's level kernel (kg_stats tail_*): k_grid_level (per-query grid tier; the 8d byte model
    over its counters) or k_ms_level (MS-BFS; per edge with work its 16-B adjx record + 4-B hop stamp, per
    active (edge, 64-query word) the child's 8-B VIS + 8-B TG words -- one row read per (group, node)
    entry, i.e. per 512 queries, not per query).  Launch time = the HIP-event durations of the timed
    launches (the first 64 of a batch) / their count; bytes per launch = the batch's bytes / launches."""
    st = [s for s in stats if s.tail_launches > 0 and s.tail_ms > 0]
    if not st:
        return None
    kind = max(int(s.tail_kind) for s in st)
    if kind == 2:
        b = np.array([20 * s.ms_edges_loaded + 16 * s.ms_words_active for s in st], float)
        model = ("20*ms_edges_loaded + 16*ms_words_active (k_ms_level: adjx record + hop stamp per edge with work, "
                 "child VIS + TG word per active (edge, 64-query word); counted in-kernel)")
    else:
        b = np.array([8 * s.tail_rows + 4 * s.tail_edges + 16 * s.tail_probes + 16 * s.tail_logged for s in st], float)
        model = "8*rows_opened + 4*edges_read + 16*direct_probes + 16*level_entries (grid tier share; counted in-kernel)"
    launches = np.array([s.tail_launches for s in st], float)
    timed = np.minimum(launches, 64)
    ms = np.array([s.tail_ms for s in st], float)
    launch_ms = float(ms.sum() / timed.sum())
    bpl = float(b.sum() / launches.sum())
    ach = bpl / (launch_ms * 1e-3) / 1e9
    name = TAIL_KERNELS.get(kind, "tail")
    return {"kernel": name, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": traffic_of(name), "bytes_model": model, "launch_ms": launch_ms,
            "bytes_per_launch": bpl, "launches_per_batch": float(launches.mean()),
            "ms_per_batch": float(launch_ms * launches.mean()),
            **({"ms_edges_loaded_per_batch": float(np.mean([s.ms_edges_loaded for s in st])),
                "ms_words_active_per_batch": float(np.mean([s.ms_words_active for s in st])),
                "edge_visits_per_batch": float(np.mean([s.tail_edges for s in st]))} if kind == 2 else
               {"edges_per_batch": float(np.mean([s.tail_edges for s in st]))})}


def level_events(snap, on: int) -> None:
    """kg_snapshot_tune("level_events"): HIP events around every tail-tier level launch of batches with stats
    (round 6; a library without the knob -- an A/B build -- just reports no tail roofline)."""
    from keto_amd import _lib
    try:
        snap.tune("level_events", on)
    except _lib.KetoGPUError:
        pass


def dominant(*rfs) -> dict:
    """The roofline of the kernel with the most device time per batch."""
    return max([r for r in rfs if r], key=lambda r: r["ms_per_batch"])


def pmc_traffic(kernel: str, tuples: int, batch: int, preset: int, inflight: int, tag: str = ""):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes
    (profiles/pmc_<kernel>_p<preset><tag>.json, scripts/gpu_profile.sh), if taken on this exact workload;
    else None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{kernel.split('<')[0]}_p{preset}{tag}.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if (int(d.get("tuples", -1)) == tuples and int(d.get("batch", -1)) == batch
                and int(d.get("inflight", -1)) == inflight):
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(orc: "CheckOracle", q: np.ndarray, a, cpus: dict) -> dict:
    """The C restatement of the reference engine (oracle, sequential Go-order DFS with visited sets)
    over the same rows, on a bounded sample of the same batch, timed at the CPUs this process can
    actually use (affinity mask capped by the cgroup quota), at 1 thread and at nproc; `value` is the
    best of them, every count is kept in `by_threads`."""
    from oracle.oracle import POLICY_DFS
    eff = cpus["effective"]

    def run(n, th, passes=1):
        t = time.perf_counter()
        for _ in range(passes):
            orc.run(q[:n], POLICY_DFS, th)
        return time.perf_counter() - t

    res = {}
    plan = [(eff, a.cpu_seconds / 2)]
    for th in (1, cpus["nproc"]):
        if th not in [p[0] for p in plan]:
            plan.append((th, a.cpu_seconds / 4))
    for th, budget in plan:
        n, passes = 256, 1
        t = run(n, th)
        while t < budget / 4 and n < len(q):  # grow the sample of distinct checks first
            n = min(len(q), n * 4)
            t = run(n, th)
        if t < budget / 2:  # then repeat it to reach ~budget seconds of CPU work
            passes = max(1, int(budget / max(t, 1e-6)))
            t = run(n, th, passes)
        res[th] = (n * passes / t, n, passes, t)
    best = max(res, key=lambda k: res[k][0])
    v, n, passes, t = res[best]
    return {"value": v, "unit": "checks/s", "cores": best, "kind": "port",
            "sample": f"{passes} pass(es) over the first {n} checks of the rank-0 batch on the same graph "
                      f"({t:.1f} s), sequential Go-order DFS with visited sets (oracle/keto_oracle.c POLICY_DFS), "
                      f"{best} host threads (best of {sorted(res)}; {eff} CPUs usable: affinity "
                      f"{cpus['affinity']}, cgroup quota {cpus['cgroup_quota']})",
            "by_threads": {str(k): r[0] for k, r in sorted(res.items())}, "effective_cpus": eff,
            "cpus": cpus, "value_1thread": res[1][0], "host_cpu": host_cpu()}


def host_cpu() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip() + f" (nproc {os.cpu_count()})"
    except OSError:
        pass
    return f"nproc {os.cpu_count()}"


if __name__ == "__main__":
    main()
