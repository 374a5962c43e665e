# diagnostics: a hot C5 root's gather / walk times (KG_EXPAND_TRACE).  Round 5 timed the walk without its
# record emission with a temporary KG_GW_DBG switch in k_expand_gw (17 % of the walk); the switch is gone.
import ctypes as C, os, subprocess, sys
code = r'''
import ctypes as C, sys, os, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from keto_amd import _lib
from keto_amd.engine import Snapshot
from keto_amd.synth import hot_group_roots
L = _lib.load()
snap = Snapshot.synthetic(1062976915, seed=20250131)
roots = hot_group_roots(snap.synth_ids(), 100000)
big = np.ascontiguousarray(roots[[0]])
def call(rs):
    buf = _lib.kg_tree_buf()
    _lib.check(L.kg_expand_batch(snap.handle, rs.ctypes.data_as(C.c_void_p), len(rs), 5, C.byref(buf)), "expand")
    n = buf.n_nodes; ms = buf.kernel_ms
    L.kg_tree_free(C.byref(buf))
    return n, ms
sz = []
for i in range(64):
    n, _ = call(np.ascontiguousarray(roots[[i]]))
    sz.append(n)
g = int(np.argmax(sz))
for _ in range(3):
    n, ms = call(np.ascontiguousarray(roots[[g]]))
print("giant", g, n, "kernel ms %.2f" % ms, flush=True)
'''
for dbg in ("0", "1"):
    env = dict(os.environ, KG_GW_DBG=dbg, KG_EXPAND_TRACE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=280)
    print("KG_GW_DBG", dbg, "rc", r.returncode)
    print("\n".join(r.stdout.strip().splitlines()[-2:]))
    print("\n".join(l for l in r.stderr.strip().splitlines() if "gw" in l)[-600:])
