"""Builds libketogpu.so in-tree with hipcc for gfx950 (no torch types cross the C ABI)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libketogpu.so")
SOURCES = ["kg_abi.cpp", "kg_batcher.cpp", "kg_snapshot.hip", "kg_check.hip", "kg_grid.hip", "kg_msbfs.hip", "kg_interp.hip", "kg_expand.hip", "kg_shard.hip", "kg_shard_comm.hip", "kg_augment.hip", "kg_formula.hip", "kg_delta.hip", "kg_rows.hip", "kg_tree.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KG_OFFLOAD_ARCH", "gfx950")


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def stale() -> bool:
    if not os.path.exists(LIB) or not os.path.exists(os.path.join(ROOT, "tools", "lib", "libkg_loadgen.so")):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(ROOT, "include", "ketogpu.h"))
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=()) -> str:
    """out / defines: an A/B variant of the library (e.g. keto_amd/lib/ab/x.so with a -D define),
    loaded by bench.py through KG_LIB_PATH; the in-tree library is built without defines."""
    if out == LIB and not force and not stale():
        return LIB
    obj_dir = os.path.join(os.path.dirname(out), ".obj_" + os.path.basename(out))
    os.makedirs(obj_dir, exist_ok=True)
    objs = []
    jobs = []
    for src in sources():
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", "-x", "hip", src, "-o", obj,
               "-I", os.path.join(ROOT, "include"), "-Wall", "-Wno-unused-function", "-Wno-unused-result"]
        cmd += ["-D" + d for d in defines]
        jobs.append((cmd, src))
        objs.append(obj)
    procs = [(subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), s) for c, s in jobs]
    failed = False
    for p, s in procs:
        log, _ = p.communicate()
        if p.returncode != 0 or verbose:
            sys.stderr.write(log.decode(errors="replace"))
        if p.returncode != 0:
            failed = True
    if failed:
        raise RuntimeError("hipcc failed")
    tmp = out + ".tmp"
    # RCCL: the hash-sharded mode's transport over xGMI (kg_shard_comm.hip)
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs +
                   ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"], check=True)
    os.replace(tmp, out)
    for o in objs:
        os.remove(o)
    os.rmdir(obj_dir)
    if out == LIB:
        build_tools()
    return out


TOOLS_LIB = os.path.join(ROOT, "tools", "lib", "libkg_loadgen.so")


def build_tools() -> str:
    """tools/kg_loadgen.cpp (bench load generator for the batcher; links libketogpu.so)."""
    src = os.path.join(ROOT, "tools", "kg_loadgen.cpp")
    os.makedirs(os.path.dirname(TOOLS_LIB), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", src, "-o", TOOLS_LIB, "-L", LIB_DIR, "-lketogpu",
                    "-Wl,-rpath," + LIB_DIR, "-Wl,-rpath,$ORIGIN/../../keto_amd/lib", "-lpthread"], check=True)
    return TOOLS_LIB


if __name__ == "__main__":
    # python -m keto_amd.build [--force] [-v] [--out PATH -DNAME=V ...]
    av = sys.argv[1:]
    out = av[av.index("--out") + 1] if "--out" in av else LIB
    print(build(force="--force" in av, verbose="-v" in av, out=os.path.abspath(out),
                defines=[x[2:] for x in av if x.startswith("-D")]))
