"""Test-only CPU restatement of one rank's local steps of the hash-sharded mode (the contract of
kg_shard_seed / kg_shard_level in include/ketogpu.h, keto_amd/csrc/kg_shard.hip), used to run
keto_amd.sharded.ShardedChecker's exchange protocol on CPU ranks under gloo.  Never shipped: the
product path is keto_amd.sharded.HipShardOps (GPU).  Rewrite-free graphs only.

The checkIsAllowed recursion it restates (internal/check/engine.go:87-207):
a record (q, v, d) = checkIsAllowed(v, d) -> checkDirect(d-1) on v's row, and children of v's
subject-set row (no SubjectIDs, no "..." sets, engine.go:118-136) at d-1 when d >= 2.
"""
import numpy as np
import torch

SUBJECT_ID = 0xFFFFFFFF
SET_BIT = 0x80000000
Q_BITS = 26
HIT = -1  # kg_frec.node == KG_FREC_HIT as int32
ERR = -2  # kg_frec.node == KG_FREC_ERR as int32
ERR_NOT_IMPLEMENTED = 2
M64 = (1 << 64) - 1


def mix64(x: int) -> int:  # kg_internal.h mix64
    x &= M64
    x ^= x >> 30
    x = (x * 0xbf58476d1ce4e5b9) & M64
    x ^= x >> 27
    x = (x * 0x94d049bb133111eb) & M64
    x ^= x >> 31
    return x


def shard_owner(ns: int, obj: int, n: int) -> int:  # kg_internal.h shard_owner
    return 0 if n <= 1 else (mix64((ns << 32) | obj) >> 20) % n


class CpuShardOps:
    device_counts = False  # level() takes host record counts only

    def __init__(self, tuples6: np.ndarray, wildcard_rel: int, rank: int, nranks: int, impure=()):
        """impure: (ns, rel) pairs whose relation has a rewrite or is undeclared (relflag != 0)."""
        self.rank, self.n = rank, nranks
        self.impure = set((int(a), int(b)) for a, b in impure)
        t = np.asarray(tuples6, np.int64).reshape(-1, 6)
        self.node = {}
        self.nrel = {}

        def nid(ns, obj, rel):
            k = (int(ns), int(obj), int(rel))
            if k not in self.node:
                self.node[k] = len(self.node)
                self.nrel[self.node[k]] = (k[0], k[2])
            return self.node[k]

        self.adj, self.direct, self.owner, self.held = {}, set(), {}, set()
        for ns, obj, rel, sns, sobj, srel in t:
            v = nid(ns, obj, rel)
            self.owner[v] = shard_owner(int(ns), int(obj), nranks)
            if sns == SUBJECT_ID:
                subj = int(sobj)
            else:
                c = nid(sns, sobj, srel)
                self.owner[c] = shard_owner(int(sns), int(sobj), nranks)
                subj = SET_BIT | c
                if srel != wildcard_rel and self.owner[v] == rank:
                    self.adj.setdefault(v, []).append(c)
            if self.owner[v] == rank:
                self.direct.add((v, subj))
            if sns == SUBJECT_ID:
                self.held.add(int(sobj))  # every rank's rows: the OR the driver installs (kg_shard_held)
        self.vis = set()

    def _emit(self, out, cap, counts, dest, rec):
        at = int(counts[dest])
        counts[dest] += 1
        if at < cap:
            out[dest * cap + at] = torch.tensor(rec, dtype=torch.int32)
        else:
            counts[self.n] |= 1

    def seed(self, dq, n, gdepth, out, cap, counts, res, err):
        self.vis = set()
        counts.zero_()
        res.zero_()
        err.zero_()
        qs = dq.numpy().reshape(-1, 7)
        qu = qs.view(np.uint32).astype(np.int64)
        for i in range(n):
            ns, obj, rel, sns, sobj, srel = (int(x) for x in qu[i, :6])
            md = int(qs[i, 6])
            v = self.node.get((ns, obj, rel))
            if sns == SUBJECT_ID:
                subj = int(sobj)
            else:
                c = self.node.get((sns, sobj, srel))
                subj = None if c is None else SET_BIT | c
            d = md if 0 < md <= gdepth else gdepth  # engine.go:68-70
            if (ns, rel) in self.impure:
                err[i] = ERR_NOT_IMPLEMENTED
                continue
            if v is None or (subj is None and not self.impure):
                continue
            if not self.impure and sns == SUBJECT_ID and int(sobj) not in self.held:
                continue  # no row of any rank holds the subject (kg_shard_seed's no-holder test)
            if subj is None:
                subj = 0xFFFFFFFF  # unknown subject: never held, but the query may still reach a rewrite
            self._emit(out, cap, counts, self.owner[v],
                       [(self.rank << Q_BITS) | i, v, np.uint32(subj).view(np.int32), d])

    def done_bits(self, res, n, words):
        """kg_shard_done: bit i of this rank's words = query i answered IsMember so far."""
        bits = np.zeros(words, np.uint32)
        for i in np.nonzero(res.numpy()[:n] == 1)[0]:
            bits[i >> 5] |= np.uint32(1 << (int(i) & 31))
        return torch.from_numpy(bits.view(np.int32).copy())

    def level(self, din, n_in, n_in_dev, out, cap, counts, res, err, done=None, done_words=0):
        assert n_in_dev is None
        counts.zero_()
        dn = None if done is None else done.numpy().view(np.uint32)
        for r in din[:n_in].tolist():
            q, v, subj, d = r[0], r[1], r[2] & 0xFFFFFFFF, r[3]
            home, qi = q >> Q_BITS, q & ((1 << Q_BITS) - 1)
            if v == HIT:
                if home == self.rank:
                    res[qi] = 1
                continue
            if v == ERR:
                if home == self.rank:
                    err[qi] = max(int(err[qi]), subj)
                continue
            if dn is not None and (qi >> 5) < done_words and (int(dn[home * done_words + (qi >> 5)]) >> (qi & 31)) & 1:
                continue  # answered IsMember by an earlier level
            if (q, v) in self.vis:
                continue
            self.vis.add((q, v))
            if self.nrel[v] in self.impure:
                if home == self.rank:
                    err[qi] = max(int(err[qi]), ERR_NOT_IMPLEMENTED)
                else:
                    self._emit(out, cap, counts, home, [q, ERR, ERR_NOT_IMPLEMENTED, 0])
            elif d >= 1 and (v, subj) in self.direct:
                if home == self.rank:
                    res[qi] = 1
                else:
                    self._emit(out, cap, counts, home, [q, HIT, 0, 0])
            elif d >= 2:
                for c in self.adj.get(v, []):
                    self._emit(out, cap, counts, self.owner[c], [q, c, np.uint32(subj).view(np.int32), d - 1])
            elif d == 1:  # checkIsAllowed(child, 0) still evaluates astRelationFor: impure -> error
                for c in self.adj.get(v, []):
                    if self.nrel[c] in self.impure:
                        if home == self.rank:
                            err[qi] = max(int(err[qi]), ERR_NOT_IMPLEMENTED)
                        else:
                            self._emit(out, cap, counts, home, [q, ERR, ERR_NOT_IMPLEMENTED, 0])

    def finish(self, n, res, err):
        res[:n][err[:n] != 0] = 2
