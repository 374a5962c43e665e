# diagnostics: the C5 largest root alone, gw on / off, with KG_EXPAND_TRACE timings
import ctypes as C, os, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from keto_amd import _lib
from keto_amd.engine import Snapshot
from keto_amd.synth import hot_group_roots
L = _lib.load()
snap = Snapshot.synthetic(1062976915, seed=20250131)
roots = hot_group_roots(snap.synth_ids(), 100000)
def call(rs):
    buf = _lib.kg_tree_buf()
    _lib.check(L.kg_expand_batch(snap.handle, rs.ctypes.data_as(C.c_void_p), len(rs), 5, C.byref(buf)), "expand")
    off = np.ctypeslib.as_array(buf.root_off, shape=(len(rs) + 1,)).copy()
    ms = buf.kernel_ms
    L.kg_tree_free(C.byref(buf))
    return off, ms
off, _ = call(roots)
sz = np.diff(off.astype(np.int64))
order = np.argsort(-sz)
print("largest", sz[order[:5]].tolist(), flush=True)
big = np.ascontiguousarray(roots[order[:1]])
for gw in (1, 0, 1):
    snap.tune("expand_gw", gw)
    for _ in range(2):
        o, ms = call(big)
    print("gw", gw, "giant kernel ms %.2f" % ms, flush=True)
snap.tune("expand_gw", 1)
for _ in range(2):
    o, ms = call(roots)
print("full batch kernel ms %.2f" % ms, flush=True)
