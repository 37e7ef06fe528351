"""Oracle backend for the distributed algorithms of monetdb_amd/dist.py: the
same exchange logic, with every local operator computed by the CPU oracle
(oracle/, the restatement of the reference GDK operators) and the shuffles
over gloo on CPU tensors.  Test infrastructure only."""
import numpy as np
import torch

from oracle import pyoracle as ora

NP = {ora.TYPE_bit: np.int8, ora.TYPE_bte: np.int8, ora.TYPE_sht: np.int16,
      ora.TYPE_int: np.int32, ora.TYPE_lng: np.int64, ora.TYPE_oid: np.uint64}


class Col:
    """A host column: numpy values (hge: (n, 2) uint64 words) + hseqbase."""

    def __init__(self, tp, arr, hseq=0):
        self.tp = tp
        self.arr = arr
        self.hseqbase = hseq

    def ora(self):
        return ora.Bat.from_array(self.tp, self.arr, hseqbase=self.hseqbase)


def _from_ora(b, hseq=0):
    s = b.s
    if s.type == ora.TYPE_hge:
        vals = b.values()
        arr = np.array([ora.int_to_hge_words(v) for v in vals], dtype=np.uint64).reshape(-1, 2)
        return Col(ora.TYPE_hge, arr, hseq)
    tp = ora.TYPE_oid if s.type == ora.TYPE_void else s.type
    return Col(tp, np.asarray(b.values()).astype(NP[tp]), hseq)


def _hash(v, nparts):
    x = v.astype(np.uint64)
    x ^= x >> np.uint64(33)
    x *= np.uint64(0xff51afd7ed558ccd)
    x ^= x >> np.uint64(33)
    return (x % np.uint64(nparts)).astype(np.int64)


class OracleBackend:
    device = "cpu"
    TYPE_lng, TYPE_oid, TYPE_hge, TYPE_bit = ora.TYPE_lng, ora.TYPE_oid, ora.TYPE_hge, ora.TYPE_bit

    def column(self, tp, arr, hseq=0):
        if tp == ora.TYPE_hge:                  # (n, 2) words
            return Col(tp, np.asarray(arr, dtype=np.uint64).reshape(-1, 2), hseq)
        return Col(tp, np.asarray(arr).astype(NP[tp]), hseq)

    def n(self, c):
        return len(c.arr)

    def values(self, c):
        if c.tp == ora.TYPE_hge:
            return [ora.hge_to_int(r) for r in c.arr]
        return c.arr

    def widen(self, c):
        if c.tp in (ora.TYPE_lng, ora.TYPE_oid):
            return c
        a = c.arr.astype(np.int64)
        a[c.arr == np.iinfo(c.arr.dtype).min] = np.iinfo(np.int64).min
        return Col(ora.TYPE_lng, a, c.hseqbase)

    def zeros_bit(self, n):
        return Col(ora.TYPE_bit, np.zeros(n, np.int8))

    def append(self, b, n):
        b.arr = np.concatenate([b.arr, n.arr.astype(b.arr.dtype)])
        return b

    def copy(self, c):
        return Col(c.tp, c.arr.copy(), c.hseqbase)

    def slice(self, c, lo, hi):
        return Col(c.tp, c.arr[lo:hi], c.hseqbase + lo)

    def dense(self, tseq, n):
        return Col(ora.TYPE_oid, np.arange(tseq, tseq + n, dtype=np.uint64))

    def addcst(self, c, v):
        return Col(ora.TYPE_lng, c.arr.astype(np.int64) + v, c.hseqbase)

    def hashpartition(self, c, nparts):
        d = _hash(c.arr.astype(np.int64), nparts)
        pos = np.argsort(d, kind="stable")
        counts = np.bincount(d, minlength=nparts).tolist()
        return Col(ora.TYPE_oid, (pos + c.hseqbase).astype(np.uint64)), counts

    def project(self, order, c):
        idx = order.arr.astype(np.int64) - c.hseqbase
        return Col(c.tp, c.arr[idx], order.hseqbase)

    def group(self, c, histo=True):
        g, e, h = ora.BATgroup(c.ora())
        return _from_ora(g, c.hseqbase), _from_ora(e), (_from_ora(h) if histo else None)

    def groupsum(self, c, g, e, tp):
        return _from_ora(ora.BATgroupsum(c.ora(), g.ora(), e.ora(), tp))

    def group_sums(self, keys, vals, tp):
        gi, e, h = self.group(keys)
        return e, h, self.widen(self.project(e, keys)), [self.groupsum(v, gi, e, tp) for v in vals]

    def groupmin(self, c, g, e):
        co = c.ora()
        return _from_ora(ora.BATproject(ora.BATgroupminmax(co, g.ora(), e.ora(), False), co))

    def groupavg3(self, c, g, e):
        a, r, k = ora.BATgroupavg3(c.ora(), g.ora(), e.ora(), True)
        return _from_ora(a), _from_ora(r), _from_ora(k)

    def groupavg3combine(self, a, r, c, g, e):
        return _from_ora(ora.BATgroupavg3combine(a.ora(), r.ora(), c.ora(), g.ora(), e.ora(), True))

    def join(self, l, r):
        a, b = ora.BATjoin(l.ora(), r.ora())
        return _from_ora(a), _from_ora(b)

    def sort(self, c, reverse=False):
        s, o = ora.BATsort(c.ora(), reverse=reverse, nilslast=reverse)
        return _from_ora(s, c.hseqbase), _from_ora(o, c.hseqbase)

    def order_info(self, c):
        a = c.arr.astype(np.int64)
        # compare neighbours (a difference would overflow next to the nil)
        srt, rev = bool((a[1:] >= a[:-1]).all()), bool((a[1:] <= a[:-1]).all())
        return srt, rev, srt and bool((a[1:] > a[:-1]).all()), int(a[0]), int(a[-1])

    def values_at(self, c, positions):
        return [int(v) for v in c.arr.astype(np.int64)[np.asarray(positions, np.int64)]]

    def lowerbound2(self, keys, pos, qk, qp):
        k = keys.arr.astype(np.int64)
        p = pos.arr.astype(np.uint64) if pos is not None else np.arange(len(k), dtype=np.uint64)
        return [int(np.count_nonzero((k < a) | ((k == a) & (p < np.uint64(b))))) for a, b in zip(qk, qp)]

    def rangebounds(self, vals, parts, limit, preceding):
        return _from_ora(ora.rangebounds(vals.ora(), parts.ora(), limit, preceding))

    def first_start(self, parts):
        nz = np.flatnonzero(parts.arr)
        return int(nz[0]) if len(nz) else None

    def pack(self, cols):
        n = len(cols[0].arr) if cols else 0
        parts = []
        for c in cols:
            if c.tp == ora.TYPE_hge:
                parts.append(c.arr.view(np.int64).reshape(n, 2))
            else:
                parts.append(c.arr.astype(np.int64).reshape(n, 1))
        return torch.from_numpy(np.ascontiguousarray(np.concatenate(parts, axis=1)))

    def unpack(self, t, types, hseq=0):
        a = t.numpy()
        cols, j = [], 0
        for tp in types:
            if tp == ora.TYPE_hge:
                cols.append(Col(tp, np.ascontiguousarray(a[:, j:j + 2]).view(np.uint64), hseq))
                j += 2
            else:
                cols.append(Col(tp, a[:, j].astype(NP[tp]), hseq))
                j += 1
        return cols
