"""A/B of the sharded exchange protocol's knobs on one GPU: the headline's generator graph, one rank,
the N > 1 exchange protocol forced over a one-rank RCCL communicator (kg_snapshot_tune
shard_force_exchange), one batch in flight (the driver's N > 1 setting).  Every configuration runs the
same batches; its answers are compared bit-exact with the first configuration's (which bench.py's
sharded line checks against the oracle).  One JSON line per configuration.

usage: python tools/shard_ab.py [--tuples 1e9] [--batch 4000000] [--steps 6] CONFIG ...
CONFIG: comma-separated key=value kg_snapshot_tune settings, e.g. shard_budget=1024,shard_back_budget=4096
("-" = the library defaults)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tuples", type=float, default=1e9)
    ap.add_argument("--batch", type=int, default=4_000_000)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=2, help="passes over the configuration list (alternating)")
    ap.add_argument("--local", action="store_true", help="the one-rank local-first path instead of the exchange")
    ap.add_argument("configs", nargs="+")
    x = ap.parse_args()
    import torch

    import bench
    from keto_amd import _lib
    from keto_amd.sharded import LibShardedChecker
    a = bench.parse(["--tuples", str(x.tuples)])
    torch.cuda.set_device(0)
    snap, _ = bench.build_synthetic(a, a.tuples, device=0)
    L = _lib.load()
    stream = bench.inflight_streams(0, 2)[1]
    chk = LibShardedChecker(snap, 0, 1, None, stream=stream)
    if not x.local:
        snap.tune("shard_force_exchange", 1)
    B, K, W = x.batch, x.steps, x.warmup
    dqs = []
    for k in range(W + K):
        d = torch.empty((B, 7), dtype=torch.int32, device="cuda:0")
        _lib.check(L.kg_synth_queries(snap.handle, 900000 + 7919 * k, B, d.data_ptr()), "kg_synth_queries")
        dqs.append(d)
    res = torch.empty((K, B), dtype=torch.uint8, device="cuda:0")
    err = torch.empty(B, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    ref = None
    defaults = {}

    def run(cfg):
        kv = {}
        if cfg != "-":
            for item in cfg.split(","):
                k, v = item.split("=")
                kv[k] = int(v)
        for k, v in kv.items():
            snap.tune(k, v)
        try:
            for k in range(W):
                chk._check_t(L.kg_check_batch_device(snap.handle, dqs[k].data_ptr(), B, a.global_depth,
                                                     res[0].data_ptr(), err.data_ptr(), None, chk._sp), "warmup")
            stream.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                chk._check_t(L.kg_check_batch_device(snap.handle, dqs[W + k].data_ptr(), B, a.global_depth,
                                                     res[k].data_ptr(), err.data_ptr(), None, chk._sp), "timed")
            stream.synchronize()
            el = time.perf_counter() - t0
            st = chk.stats()
        finally:
            for k in kv:
                snap.tune(k, defaults.get(k, 0))
        return el, st

    # library defaults to restore (the knobs these A/Bs touch)
    defaults.update({"shard_budget": 0, "shard_back_budget": 1 << 14, "shard_vis_mode": 0, "shard_heavy": 64,
                     "shard_wgs": 8, "shard_vis": 23, "shard_local": 1, "shard_level_occ": 0, "shard_pack": 0})
    for rnd in range(x.rounds):
        for cfg in x.configs:
            el, st = run(cfg)
            r = res.cpu().numpy()
            if ref is None:
                ref = r.copy()
            mism = int((r != ref).sum())
            print(json.dumps({"cfg": cfg, "round": rnd, "checks_per_s": B * K / el, "ms_per_batch": el / K * 1e3,
                              "mismatches_vs_first": mism, "allowed": float(r.mean()), "stats": st}), flush=True)
    chk.close()
    snap.close()


if __name__ == "__main__":
    main()
