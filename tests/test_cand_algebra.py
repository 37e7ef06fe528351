"""Candidate-list algebra: BATmergecand, BATintersectcand, BATdiffcand
(gdk/gdk_cand.c:46, :184, :259) and BATnegcands (:1296).

No known-answer test of the reference exercises these (they are reached
through bat.mergecand / bat.intersectcand and the SQL layer's OR / NOT
plans), so the oracle's restatement of the reference's loops is checked
against an independent model -- numpy's set operations on the sorted,
duplicate-free oid sequences a candidate list stands for (parity unpinned
beyond that) -- and the device against the oracle, over every form a
candidate list takes: dense (void), materialised oid lists, cand_except
and cand_mask lists and msk BATs (the oracle gets the oid list they stand
for).  Results: the same oid sequence, void exactly when dense (virtualize,
gdk_select.c:31), sorted / key / no nils."""
import numpy as np
import pytest

from helpers import rng


def _cases():
    r = rng(1201)
    U = np.uint64
    dense = lambda s, n: ("dense", s, n)                                     # noqa: E731
    mat = lambda a: ("oids", np.unique(np.asarray(a, U)))                    # noqa: E731
    big = np.sort(r.choice(2_000_000, 600_000, replace=False)).astype(U) + 100
    yield "dense_overlap", dense(10, 100), dense(60, 100)
    yield "dense_touch", dense(10, 50), dense(60, 40)
    yield "dense_gap", dense(10, 50), dense(70, 40)
    yield "dense_inside", dense(10, 500), dense(60, 40)
    yield "dense_empty", dense(10, 50), dense(0, 0)
    yield "empty_empty", dense(0, 0), dense(5, 0)
    yield "mat_dense", mat(r.choice(1000, 300, replace=False) + 5), dense(200, 400)
    yield "dense_mat", dense(200, 400), mat(r.choice(1000, 300, replace=False) + 5)
    yield "mat_mat", mat(r.choice(5000, 2000, replace=False)), mat(r.choice(5000, 3000, replace=False))
    yield "mat_dense_run", mat(np.arange(300, 900)), mat(np.arange(500, 1200))
    yield "mat_disjoint", mat(np.arange(0, 100, 2)), mat(np.arange(1, 100, 2))
    yield "one_each", mat([7]), mat([7])
    yield "big", ("oids", big), ("oids", np.sort(r.choice(big, 250_000, replace=False)))
    yield "big_dense", ("oids", big), dense(500_000, 1_000_000)


def _model(kind, a, b):
    if kind == "merge":
        return np.union1d(a, b).astype(np.uint64)
    if kind == "intersect":
        return np.intersect1d(a, b).astype(np.uint64)
    return np.setdiff1d(a, b).astype(np.uint64)


def _oids(spec):
    if spec[0] == "dense":
        return np.arange(spec[1], spec[1] + spec[2], dtype=np.uint64)
    return spec[1]


def _ora_bat(ora, spec):
    if spec[0] == "dense":
        return ora.Bat.dense(spec[1], spec[2])
    return ora.Bat.from_array(ora.TYPE_oid, spec[1], sorted_=True, key=True, nonil=True)


def _is_dense(v):
    return len(v) == 0 or int(v[-1]) - int(v[0]) == len(v) - 1


OPS = ("merge", "intersect", "diff")


@pytest.mark.parametrize("name,a,b", list(_cases()))
@pytest.mark.parametrize("op", OPS)
def test_oracle_cand_algebra(ora, name, a, b, op):
    fa, fb = _ora_bat(ora, a), _ora_bat(ora, b)
    f = {"merge": ora.mergecand, "intersect": ora.intersectcand, "diff": ora.diffcand}[op]
    got = f(fa, fb)
    want = _model(op, _oids(a), _oids(b))
    assert np.array_equal(np.asarray(got.values(), np.uint64), want)
    if len(want):
        assert (got.s.type == ora.TYPE_void) == _is_dense(want)


@pytest.mark.parametrize("tseq,nr,dels", [(100, 1000, [5, 100, 101, 500, 1099, 1100, 5000]),
                                          (0, 50, []), (10, 20, np.arange(0, 100)), (10, 20, [3, 40]),
                                          (7, 100_000, np.arange(7, 100_007, 3))])
def test_oracle_negcands(ora, tseq, nr, dels):
    d = np.asarray(dels, np.uint64)
    got = ora.negcands(tseq, nr, ora.Bat.from_array(ora.TYPE_oid, d, sorted_=True, key=True, nonil=True))
    want = np.setdiff1d(np.arange(tseq, tseq + nr, dtype=np.uint64), d)
    assert np.array_equal(np.asarray(got.values(), np.uint64), want)


def _dev_bat(gdk, spec, form, r):
    """the device list in `form` standing for the oids of spec"""
    oids = _oids(spec)
    if spec[0] == "dense" and form == "plain":
        return gdk.BAT.dense(spec[1], spec[2])
    if form == "plain" or len(oids) == 0:
        return gdk.BAT.from_numpy(gdk.TYPE_oid, oids, sorted_=True, revsorted=len(oids) <= 1, key=True, nonil=True)
    lo, hi = int(oids[0]), int(oids[-1]) + 1
    if form == "except":
        exc = np.setdiff1d(np.arange(lo, hi, dtype=np.uint64), oids)
        return gdk.BAT.negoid_cand(lo, len(oids), exc)
    bits = np.zeros(hi - lo, bool)
    bits[(oids - lo).astype(np.int64)] = True
    if form == "mask":
        return gdk.BAT.mask_cand(lo, bits)
    return gdk.BAT.msk(bits, hseqbase=lo)          # a msk BAT: hseqbase + i for every set bit


@pytest.mark.gpu
@pytest.mark.parametrize("name,a,b", list(_cases()))
@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("forms", [("plain", "plain"), ("except", "plain"), ("plain", "mask"), ("msk", "except")])
def test_gpu_cand_algebra(gdk, ora, name, a, b, op, forms):
    r = rng(1202)
    da, db = _dev_bat(gdk, a, forms[0], r), _dev_bat(gdk, b, forms[1], r)
    f = {"merge": gdk.BATmergecand, "intersect": gdk.BATintersectcand, "diff": gdk.BATdiffcand}[op]
    got = f(da, db)
    of = {"merge": ora.mergecand, "intersect": ora.intersectcand, "diff": ora.diffcand}[op]
    want = of(_ora_bat(ora, a), _ora_bat(ora, b))
    wv = np.asarray(want.values(), np.uint64)
    assert np.array_equal(got.to_numpy().astype(np.uint64), wv)
    assert got.hseqbase == 0
    if len(wv):
        assert (got.ttype == gdk.TYPE_void) == _is_dense(wv)
        assert got.s.tsorted and got.s.tkey and got.s.tnonil


@pytest.mark.gpu
@pytest.mark.parametrize("tseq,nr,dels,void", [(100, 1000, [5, 100, 101, 500, 1099, 1100, 5000], False),
                                               (0, 50, [], False), (10, 20, np.arange(0, 100), False),
                                               (10, 20, [3, 40], False), (7, 100_000, np.arange(7, 100_007, 3), False),
                                               (50, 1000, (900, 300), True)])
def test_gpu_negcands(gdk, ora, tseq, nr, dels, void):
    if void:
        od = gdk.BAT.dense(dels[0], dels[1])
        d = np.arange(dels[0], dels[0] + dels[1], dtype=np.uint64)
    else:
        d = np.asarray(dels, np.uint64)
        od = gdk.BAT.from_numpy(gdk.TYPE_oid, d, sorted_=True, key=True, nonil=True)
    got = gdk.BATnegcands(tseq, nr, od)
    want = np.asarray(ora.negcands(tseq, nr, ora.Bat.from_array(ora.TYPE_oid, d, sorted_=True, key=True,
                                                                nonil=True)).values(), np.uint64)
    assert got.ttype == gdk.TYPE_void and got.count() == len(want)
    assert np.array_equal(gdk.cand_oids(got), want)
    # the cand_except list works as a candidate list (select through it)
    if len(want):
        n = tseq + nr + 10
        v = (np.arange(n) % 7).astype(np.int32)
        B = gdk.BAT.from_numpy(gdk.TYPE_int, v)
        s = gdk.BATthetaselect(B, got, 3, "<").to_numpy()
        assert np.array_equal(s, want[v[want.astype(np.int64)] < 3])
