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
ESC = -3  # kg_frec.node == KG_FREC_ESC as int32 (the query escalates to the backward phase)
ESC_BIT = 0x40000000  # err marker of an escalated query while the batch runs (kg_shard.hip)
ESC2_BIT = 0x20000000  # ... and of one past the backward budget too (final forward phase)
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

    @property
    def escalates(self) -> bool:  # the backward / final forward phases run only with a forward budget
        return self.budget > 0

    def __init__(self, tuples6: np.ndarray, wildcard_rel: int, rank: int, nranks: int, impure=(), budget=0,
                 back_budget=1 << 14, program=None):
        """impure: (ns, rel) pairs whose relation has a rewrite or is undeclared (relflag != 0).
        budget: forward set edges per query on this rank before the query escalates (0 = off; only
        without impure relations, like kg_snapshot_tune "shard_budget")."""
        self.rank, self.n = rank, nranks
        self.budget = 0 if impure else int(budget)
        self.back_budget = int(back_budget)
        self.final = False
        self.impure = set((int(a), int(b)) for a, b in impure)
        t = np.asarray(tuples6, np.int64).reshape(-1, 6)
        self.wildcard_rel, self.program = wildcard_rel, program
        # rows of this rank's objects in tuple (shard) order, per (ns, obj): GetRelationTuples of the
        # general-rewrite region gather (HipShardOps.region_rows, kg_snapshot_rows)
        self.obj_rows = {}
        for k, row in enumerate(t):
            if shard_owner(int(row[0]), int(row[1]), nranks) == rank:
                self.obj_rows.setdefault((int(row[0]), int(row[1])), []).append(k)
        self.t6 = np.asarray(tuples6, np.uint32).reshape(-1, 6)
        self.node = {}
        self.nrel = {}

        def nid(ns, obj, rel):
            k = (int(ns), int(obj), int(rel))
            if k not in self.node:
                self.node[k] = len(self.node)
                self.nrel[self.node[k]] = (k[0], k[2])
            return self.node[k]

        self.adj, self.direct, self.owner, self.held, self.holders = {}, set(), {}, set(), {}
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
                self.holders.setdefault(subj, []).append(v)  # this rank's rows holding subj
            if sns == SUBJECT_ID:
                self.held.add(int(sobj))  # every rank's rows: the OR the driver installs (kg_shard_held)
        self.radj = {}  # local parents: P (owned here) -> N for every set edge P -> N of this rank's rows
        for p, cs in self.adj.items():
            for c in cs:
                self.radj.setdefault(c, []).append(p)
        self.vis = set()
        self.qcnt, self.qinfo = {}, {}

    def errors_possible(self) -> bool:  # kg_shard_bad_nodes: a relation the protocol cannot evaluate
        return bool(self.impure)

    def _emit(self, out, cap, counts, dest, rec, nb=None):
        nb = self.n if nb is None else nb  # buckets (the flags word follows them)
        at = int(counts[dest])
        counts[dest] += 1
        if at < cap:
            out[dest * cap + at] = torch.tensor(rec, dtype=torch.int32)
        else:
            counts[nb] |= 1

    def seed(self, dq, n, gdepth, out, cap, counts, res, err):
        self.vis = set()
        self.qcnt, self.qinfo = {}, {}
        self.final = False
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
            self.qinfo[i] = (v, subj, d)
            self._emit(out, cap, counts, self.owner[v],
                       [(self.rank << Q_BITS) | i, v, np.uint32(subj).view(np.int32), d])

    def done_bits(self, res, n, words, err=None, mode=1):
        """kg_shard_done: bit i of this rank's words = query i answered IsMember so far (err given:
        or escalated out of the phase: mode 1 forward, 2 backward)."""
        bits = np.zeros(words, np.uint32)
        d = res.numpy()[:n] == 1
        if err is not None and mode:
            d |= (err.numpy()[:n] & (ESC_BIT if mode == 1 else ESC2_BIT)) != 0
        for i in np.nonzero(d)[0]:
            bits[i >> 5] |= np.uint32(1 << (int(i) & 31))
        return torch.from_numpy(bits.view(np.int32).copy())

    def level_seg(self, din, n_seg, seg_cap, seg_counts, out, cap, counts, res, err, done=None, done_words=0):
        """kg_shard_level_seg: segment k = din[k * seg_cap:], min(seg_counts[k], seg_cap) records."""
        cnt = [min(int(x), seg_cap) for x in seg_counts.tolist()]
        recs = torch.cat([din[k * seg_cap: k * seg_cap + cnt[k]] for k in range(n_seg)])
        self.level(recs, int(recs.shape[0]), None, out, cap, counts, res, err, done, done_words)

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
            if v == ESC:
                if home == self.rank:
                    err[qi] = int(err[qi]) | ESC_BIT
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
                kids = self.adj.get(v, [])
                if self.budget and kids and not self.final:  # escalation: this rank's set-edge count of the query passes the budget
                    old = self.qcnt.get(q, 0)
                    add = min(len(kids), self.budget)
                    self.qcnt[q] = old + add
                    if old + add >= self.budget:  # every dropped row marks its query (kg_shard.hip k_shard_level)
                        if home == self.rank:
                            err[qi] = int(err[qi]) | ESC_BIT
                        else:
                            self._emit(out, cap, counts, home, [q, ESC, 0, 0])
                        kids = []
                for c in kids:
                    self._emit(out, cap, counts, self.owner[c], [q, c, np.uint32(subj).view(np.int32), d - 1])
            elif d == 1:  # checkIsAllowed(child, 0) still evaluates astRelationFor: impure -> error
                for c in self.adj.get(v, []):
                    if self.nrel[c] in self.impure:
                        if home == self.rank:
                            err[qi] = max(int(err[qi]), ERR_NOT_IMPLEMENTED)
                        else:
                            self._emit(out, cap, counts, home, [q, ERR, ERR_NOT_IMPLEMENTED, 0])

    # ---- backward phase (kg_shard_back_list / _seed / _level): reverse search from the holders
    def back_list(self, n, res, err, out, cap, counts):
        counts.zero_()
        self.vis = set()
        self.qcnt = {}
        for i, (v, subj, d) in sorted(self.qinfo.items()):
            if i < n and (int(err[i]) & ESC_BIT) and int(res[i]) != 1 and subj != 0xFFFFFFFF:
                self._emit(out, cap, counts, 0, [(self.rank << Q_BITS) | i, v, np.uint32(subj).view(np.int32), d], 1)

    def back_seed(self, lst, m, m_dev, out, cap, counts):
        assert m_dev is None
        counts.zero_()
        for q, root, subj, d in lst[:m].tolist():
            if d >= 2:
                for h in self.holders.get(subj & 0xFFFFFFFF, []):
                    if h != root:
                        self._emit(out, cap, counts, 0, [q, h, root, d - 1], 1)

    def back_level(self, din, n_in, n_in_dev, out, cap, counts, res, err, done=None, done_words=0):
        assert n_in_dev is None
        counts[0] = 0
        dn = None if done is None else done.numpy().view(np.uint32)
        for q, v, root, d in din[:n_in].tolist():
            home, qi = q >> Q_BITS, q & ((1 << Q_BITS) - 1)
            if v == HIT:
                if home == self.rank:
                    res[qi] = 1
                continue
            if v == ESC:
                if home == self.rank:
                    err[qi] = int(err[qi]) | ESC2_BIT
                continue
            if dn is not None and (qi >> 5) < done_words and (int(dn[home * done_words + (qi >> 5)]) >> (qi & 31)) & 1:
                continue
            if (q, v) in self.vis or d < 1:
                self.vis.add((q, v))
                continue
            self.vis.add((q, v))
            parents = self.radj.get(v, [])
            if self.back_budget and parents:  # the reverse search's budget: past it, the final forward phase
                old = self.qcnt.get(q, 0)
                add = min(len(parents), self.back_budget)
                self.qcnt[q] = old + add
                if old + add >= self.back_budget:  # every dropped row marks its query (k_shard_back_level)
                    if home == self.rank:
                        err[qi] = int(err[qi]) | ESC2_BIT
                    else:
                        self._emit(out, cap, counts, 0, [q, ESC, 0, 0], 1)
                    parents = []
            for p in parents:
                if p == root:
                    if home == self.rank:
                        res[qi] = 1
                    else:
                        self._emit(out, cap, counts, 0, [q, HIT, 0, 0], 1)
                elif d >= 2:
                    self._emit(out, cap, counts, 0, [q, p, root, d - 1], 1)

    def refwd_seed(self, n, res, err, out, cap, counts):
        counts.zero_()
        self.vis = set()
        self.final = True
        for i, (v, subj, d) in sorted(self.qinfo.items()):
            if i < n and (int(err[i]) & ESC2_BIT) and int(res[i]) != 1:
                self._emit(out, cap, counts, self.owner[v], [(self.rank << Q_BITS) | i, v, np.uint32(subj).view(np.int32), d])

    def finish(self, n, res, err):
        err[:n] = err[:n] & ~(ESC_BIT | ESC2_BIT)
        res[:n][err[:n] != 0] = 2

    # ---- general rewrites: the region gather's local steps (HipShardOps.region_rows / general_check)
    def region_rows(self, objs):
        """Rows of every relation of each held (ns, obj), grouped by relation in shard order."""
        offs, parts = [0], []
        for ns, obj in np.asarray(objs, np.int64).reshape(-1, 2).tolist():
            idx = self.obj_rows.get((ns, obj), [])
            rows = self.t6[idx] if idx else np.zeros((0, 6), np.uint32)
            rows = rows[np.argsort(rows[:, 2], kind="stable")]  # relation by relation, each in shard order
            parts.append(rows)
            offs.append(offs[-1] + rows.shape[0])
        tup = np.concatenate(parts) if parts else np.zeros((0, 6), np.uint32)
        return np.asarray(offs, np.int64), tup

    def general_check(self, region, q7, gdepth):
        """The oracle (test-only, in the role of the single-GPU engine) on the gathered region's rows."""
        from oracle.oracle import POLICY_CANONICAL, Oracle
        q7 = np.asarray(q7, np.uint32).reshape(-1, 7)
        o = Oracle(np.asarray(region, np.uint32).reshape(-1, 6), self.wildcard_rel, self.program)
        res, err, _ = o.check_batch(q7[:, :6], q7[:, 6].view(np.int32), gdepth, POLICY_CANONICAL)
        return np.asarray(res, np.uint8), np.asarray(err, np.uint32)
