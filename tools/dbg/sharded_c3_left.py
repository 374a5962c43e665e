"""Debug: the C3 hash-sharded one-rank batch leaves records after gdepth levels -- which path."""
import os, sys, ctypes as C
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from keto_amd import _lib
from keto_amd.engine import Snapshot
from keto_amd.sharded import HipShardOps, ShardedChecker

torch.cuda.set_device(0)
n_t = float(sys.argv[1]) if len(sys.argv) > 1 else 1e8
snap = Snapshot.synthetic(int(n_t), seed=20250131, shard=(0, 1), preset=1)
L = _lib.load()
B = 1_000_000
dq = torch.empty((B, 7), dtype=torch.int32, device="cuda")
_lib.check(L.kg_synth_queries(snap.handle, 1000, B, dq.data_ptr()), "kg_synth_queries")
ops = HipShardOps(snap)
print("bad nodes", ops.errors_possible(), "slots", ops.result_slots(B), flush=True)
for heavy in (64, 4096):
    for trace in (0, 1):
        snap.tune("shard_heavy", heavy)
        os.environ["KG_SHARD_TRACE"] = str(trace)
        chk = ShardedChecker(ops, 0, 1, None, device="cuda")
        try:
            res, err = chk.check(dq, 10)
            print("heavy", heavy, "trace", trace, "ok", float(res.float().mean()), "levels", chk.level_records, flush=True)
        except Exception as e:  # noqa: BLE001
            print("heavy", heavy, "trace", trace, "FAIL", e, "levels", chk.level_records, flush=True)
