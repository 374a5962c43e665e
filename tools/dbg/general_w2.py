"""Debug: the OPL full example sharded at world 2 -- which wrong answers come from the level protocol
and which from the general phase."""
import os, sys
import numpy as np
import torch
import torch.multiprocessing as mp
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))


def worker(rank, world, port, outq, general):
    sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from keto_amd.engine import Snapshot
    from keto_amd.sharded import HipShardOps, ShardedChecker
    from test_shard import _opl_full_example_graph
    os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    it, t6, q, prog, _ = _opl_full_example_graph(7)
    snap = Snapshot(t6, it, prog, 0, shard=(rank, world))
    mine = np.array_split(np.arange(len(q)), world)[rank]
    chk = ShardedChecker(HipShardOps(snap), rank, world, dist, device="cuda", cap=256, general=general)
    res, err = chk.check(torch.from_numpy(q[mine].view(np.int32).copy()).cuda(), 5)
    outq.put((rank, mine, res.cpu().numpy(), err.cpu().numpy()))
    dist.destroy_process_group()


def run(world, general):
    from test_shard import _free_port
    ctx = mp.get_context("spawn"); outq = ctx.Queue(); port = _free_port()
    ps = [ctx.Process(target=worker, args=(r, world, port, outq, general)) for r in range(world)]
    for p in ps: p.start()
    got = [outq.get(timeout=120) for _ in range(world)]
    for p in ps: p.join(60)
    from test_shard import _opl_full_example_graph
    it, t6, q, _, _ = _opl_full_example_graph(7)
    res = np.zeros(len(q), np.uint8); err = np.zeros(len(q), np.int64)
    for _, mine, r, e in got:
        res[mine], err[mine] = r, e
    return res, err


if __name__ == "__main__":
    from test_shard import _opl_full_example_graph
    from oracle.oracle import POLICY_CANONICAL, Oracle
    it, t6, q, prog, prog_ref = _opl_full_example_graph(7)
    exp, oerr, _ = Oracle(t6, it.wildcard_rel, prog_ref).check_batch(q[:, :6], q[:, 6].view(np.int32), 5, POLICY_CANONICAL)
    rels = {it.rel_id(r, create=False): r for r in ["view", "edit", "not", "rename", "viewers", "owners", "parents"]}
    for world in (1, 2):
        r0, e0 = run(world, False)
        r1, e1 = run(world, True)
        ni = (r0 == 2) & (e0 == 2)
        bad0 = np.nonzero(~ni & ((r0 != exp) | (e0 != oerr)))[0]
        bad1 = np.nonzero((r1 != exp) | (e1 != oerr))[0]
        print(f"world {world}: level-protocol answers {int((~ni).sum())} wrong {bad0.size}; NOT_IMPL {int(ni.sum())}; "
              f"with general phase wrong {bad1.size} (of them NOT_IMPL before: {int(ni[bad1].sum())})")
        for i in bad1[:10]:
            print("  ", q[i].tolist(), rels.get(int(q[i][2]), q[i][2]), "got", int(r1[i]), int(e1[i]), "exp", int(exp[i]),
                  int(oerr[i]), "level:", int(r0[i]), int(e0[i]))
