"""Diagnostic: one rank, escalation budgets (2, 16) on the C4 generator -- the in-library device loop,
the forced exchange protocol and the Python driver, two batches each, against the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from keto_amd import _lib  # noqa: E402
from keto_amd.engine import Snapshot  # noqa: E402
from oracle.oracle import POLICY_CANONICAL, Oracle  # noqa: E402
from test_shard import _checker  # noqa: E402

torch.cuda.set_device(0)
n_q, gmax = 20000, 10
full = Snapshot.synthetic(300_000, seed=20250131)
o = Oracle(full.export(), 0)
for driver in sys.argv[1:] or ["lib-loop", "lib-rccl-forced", "py"]:
    snap = Snapshot.synthetic(300_000, seed=20250131, shard=(0, 1))
    snap.tune("shard_budget", int(os.environ.get("BUDGET", "2")))
    snap.tune("shard_back_budget", int(os.environ.get("BACK", "16")))
    dq = torch.empty((n_q, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 31, n_q, dq.data_ptr()), "kg_synth_queries")
    q = dq.cpu().numpy().view(np.uint32)
    exp, _, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL, nthreads=8)
    chk = _checker(driver, snap, 0, 1, None, cap=1 << 14)
    for run in range(3):
        r, e = chk.check(dq, gmax)
        r = r.cpu().numpy()
        bad = np.nonzero(r != exp)[0]
        print(driver, "run", run, "mismatches", bad.size, "got1/exp1", int((r[bad] == 1).sum()), int((exp[bad] == 1).sum()),
              "back_levels", getattr(chk, "back_levels", None), "first", bad[:5].tolist(), flush=True)
    snap.close()
