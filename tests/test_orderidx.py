"""BATorderidx (gdk/gdk_orderidx.c:184) and its consumers.

The order index is a column's sort order kept with it.  What it changes
that a caller can see:
  * BATsort (gdk_batop.c:2488-2572) answers from it: an unstable sort of a
    column with a STABLE index returns the stable order (not GDKqsort's),
    a stable sort ignores an unstable index; BATsort builds an index when it
    returns an order of a column that is not a view, and views over a whole
    column use the parent's;
  * BATrangejoin (gdk_join.c:5137-5273) probes an unsorted l through it:
    the pairs come right-major, each right candidate's matches in the
    index's order -- not the nested loop's left-major order.
The oracle has no order index; the tests pin the index to the oracle's
stable / unstable BATsort and the range join to a Python model of the
reference's loop, itself checked against the oracle's nested-loop join as
a multiset (parity unpinned beyond that: the reference holds no fixture)."""
import numpy as np
import pytest

from helpers import rng


def _lower(keys, ord_, v, last):
    """ORDERfndfirst (last False) / ORDERfndlast (True) over the index"""
    a, b = 0, len(ord_)
    while a < b:
        m = (a + b) // 2
        x = keys[ord_[m]]
        if (x <= v) if last else (x < v):
            a = m + 1
        else:
            b = m
    return a


def rangejoin_oidx_model(lv, lnil, ord_, rl, rh, rnil, lcands, rcands, linc, hinc):
    """gdk_join.c:5160-5273 (hseqbase 0): per right candidate the index
    entries between the bounds that are left candidates, in index order"""
    lset = set(int(x) for x in lcands)
    keys = np.where(lnil, -np.inf, lv.astype(np.float64))
    r1, r2 = [], []
    for ro in rcands:
        if rnil[ro]:
            continue
        lo = _lower(keys, ord_, float(rl[ro]), not linc)
        hi = _lower(keys, ord_, float(rh[ro]), hinc)
        for q in range(lo, hi):
            if int(ord_[q]) in lset:
                r1.append(int(ord_[q]))
                r2.append(int(ro))
    return r1, r2


def _case(seed, n=3000, m=300):
    r = rng(seed)
    lv = r.integers(-500, 500, n).astype(np.int32)
    lv[::41] = -(1 << 31)
    a = r.integers(-520, 520, m)
    w = r.integers(0, 30, m)
    rl = a.astype(np.int32)
    rh = (a + w).astype(np.int32)
    rl[::17] = -(1 << 31)
    return lv, rl, rh


def test_model_matches_nested_loop(ora):
    lv, rl, rh = _case(1701)
    n, m = len(lv), len(rl)
    lnil = lv == -(1 << 31)
    rnil = (rl == -(1 << 31)) | (rh == -(1 << 31))
    _, o = ora.BATsort(ora.Bat.from_array(ora.TYPE_int, lv), stable=True)
    ord_ = np.asarray(o.values())
    r = rng(1702)
    lc = np.sort(r.choice(n, n // 2, replace=False))
    rc = np.sort(r.choice(m, m // 2, replace=False))
    for linc, hinc in ((True, True), (False, True), (True, False), (False, False)):
        a, b = rangejoin_oidx_model(lv, lnil, ord_, rl, rh, rnil, lc, rc, linc, hinc)
        oa, ob = ora.BATrangejoin(ora.Bat.from_array(ora.TYPE_int, lv), ora.Bat.from_array(ora.TYPE_int, rl),
                                  ora.Bat.from_array(ora.TYPE_int, rh),
                                  ora.Bat.from_array(ora.TYPE_oid, lc.astype(np.uint64), sorted_=True, key=True,
                                                     nonil=True),
                                  ora.Bat.from_array(ora.TYPE_oid, rc.astype(np.uint64), sorted_=True, key=True,
                                                     nonil=True), linc, hinc)
        assert sorted(zip(a, b)) == sorted(zip(oa.values().tolist(), ob.values().tolist()))
        # right-major, each right candidate's matches in index order
        assert b == sorted(b)
        pos = {int(x): i for i, x in enumerate(ord_)}
        for k in range(1, len(a)):
            if b[k] == b[k - 1]:
                assert pos[a[k]] > pos[a[k - 1]]


# ---- device ---------------------------------------------------------------


def _dbl_ties(seed, n=5000):
    r = rng(seed)
    v = (r.integers(0, 40, n) / 4).astype(np.float64)
    v[::97] = np.nan
    return v


def _g(gdk, tp, v):
    return gdk.BAT.from_numpy(tp, v, sorted_=False, revsorted=False, key=False)


@pytest.mark.gpu
@pytest.mark.parametrize("stable", [False, True])
def test_gpu_orderidx_is_the_sort_order(gdk, ora, stable):
    v = _dbl_ties(1703)
    b = _g(gdk, gdk.TYPE_dbl, v)
    assert not gdk.BATcheckorderidx(b)
    gdk.BATorderidx(b, stable)
    assert gdk.BATcheckorderidx(b)
    idx, st = gdk.BATorderidx_get(b)
    assert st == stable
    _, o, _ = ora.BATsort_full(ora.Bat.from_array(ora.TYPE_dbl, v), stable=stable, want_groups=False)
    assert np.array_equal(idx.to_numpy(), o.values())
    # a second call keeps the index
    gdk.BATorderidx(b, not stable)
    assert gdk.BATorderidx_get(b)[1] == stable


@pytest.mark.gpu
def test_gpu_sort_answers_from_a_stable_index(gdk, ora):
    v = _dbl_ties(1704)
    ob = ora.Bat.from_array(ora.TYPE_dbl, v)
    _, ost, _ = ora.BATsort_full(ob, stable=True)
    _, oun, _ = ora.BATsort_full(ob, stable=False)
    assert not np.array_equal(ost.values(), oun.values())     # ties: qsort's order differs
    b = _g(gdk, gdk.TYPE_dbl, v)
    gdk.BATorderidx(b, True)
    s, o, g = gdk.BATsort(b, stable=False)
    assert np.array_equal(o.to_numpy(), ost.values())
    ws, _, wg = ora.BATsort_full(ob, stable=True)
    assert np.array_equal(np.isnan(s.to_numpy()), np.isnan(ws.values()))
    assert np.array_equal(np.nan_to_num(s.to_numpy()), np.nan_to_num(ws.values()))
    assert np.array_equal(g.to_numpy(), wg.values())
    assert s.ptr.contents.tsorted == 1


@pytest.mark.gpu
def test_gpu_sort_builds_and_skips_an_unstable_index(gdk, ora):
    v = _dbl_ties(1705)
    ob = ora.Bat.from_array(ora.TYPE_dbl, v)
    b = _g(gdk, gdk.TYPE_dbl, v)
    _, o1, _ = gdk.BATsort(b, stable=False, groups=False)
    _, oun, _ = ora.BATsort_full(ob, stable=False, want_groups=False)
    assert np.array_equal(o1.to_numpy(), oun.values())
    idx, st = gdk.BATorderidx_get(b)
    assert not st and np.array_equal(idx.to_numpy(), oun.values())
    # a stable sort does not use the unstable index, and keeps it
    _, o2, _ = gdk.BATsort(b, stable=True, groups=False)
    _, ost, _ = ora.BATsort_full(ob, stable=True, want_groups=False)
    assert np.array_equal(o2.to_numpy(), ost.values())
    assert not gdk.BATorderidx_get(b)[1]
    # reverse sorts neither use nor build one
    b2 = _g(gdk, gdk.TYPE_dbl, v)
    gdk.BATsort(b2, reverse=True, nilslast=True, stable=True, groups=False)
    assert not gdk.BATcheckorderidx(b2)


@pytest.mark.gpu
def test_gpu_orderidx_lifecycle(gdk, ora):
    v = _dbl_ties(1706, 2000)
    b = _g(gdk, gdk.TYPE_dbl, v)
    gdk.BATorderidx(b, True)
    # a whole-column view sorts through the parent's index; it has none of its own
    vw = gdk.BATslice(b, 0, len(v))
    assert not gdk.BATcheckorderidx(vw)
    _, o, _ = gdk.BATsort(vw, stable=False, groups=False)
    _, ost, _ = ora.BATsort_full(ora.Bat.from_array(ora.TYPE_dbl, v), stable=True, want_groups=False)
    assert np.array_equal(o.to_numpy(), ost.values())
    # a partial view neither uses nor builds one
    pv = gdk.BATslice(b, 10, 1500)
    _, o, _ = gdk.BATsort(pv, stable=False, groups=False)
    _, oun, _ = ora.BATsort_full(ora.Bat.from_array(ora.TYPE_dbl, v[10:1500]), stable=False, want_groups=False)
    assert np.array_equal(o.to_numpy() - 10, oun.values())
    assert not gdk.BATcheckorderidx(pv)
    # a write drops it
    gdk.BATappend(b, _g(gdk, gdk.TYPE_dbl, v[:5]))
    assert not gdk.BATcheckorderidx(b)
    gdk.BATorderidx(b, False)
    gdk.OIDXdestroy(b)
    assert not gdk.BATcheckorderidx(b)
    # sorted input: no index, the column is marked sorted
    s = gdk.BAT.from_numpy(gdk.TYPE_int, np.arange(100, dtype=np.int32))
    gdk.BATorderidx(s, True)
    assert not gdk.BATcheckorderidx(s) and s.ptr.contents.tsorted == 1
    with pytest.raises(gdk.GDKError, match="No order index on void type bats"):
        gdk.BATorderidx(gdk.BAT.dense(0, 10), True)


@pytest.mark.gpu
@pytest.mark.parametrize("cands", ["none", "oids"])
def test_gpu_rangejoin_through_orderidx(gdk, ora, cands):
    lv, rl, rh = _case(1707, n=20000, m=2000)
    n, m = len(lv), len(rl)
    lnil = lv == -(1 << 31)
    rnil = (rl == -(1 << 31)) | (rh == -(1 << 31))
    L = _g(gdk, gdk.TYPE_int, lv)
    gdk.BATorderidx(L, False)
    idx = gdk.BATorderidx_get(L)[0].to_numpy()
    r = rng(1708)
    lc = np.arange(n) if cands == "none" else np.sort(r.choice(n, n // 3, replace=False))
    rc = np.arange(m) if cands == "none" else np.sort(r.choice(m, m // 2, replace=False))
    sl = sr = None
    if cands == "oids":
        sl = gdk.BAT.from_numpy(gdk.TYPE_oid, lc.astype(np.uint64), sorted_=True, key=True, nonil=True)
        sr = gdk.BAT.from_numpy(gdk.TYPE_oid, rc.astype(np.uint64), sorted_=True, key=True, nonil=True)
    for linc, hinc in ((True, True), (False, False)):
        a, b = gdk.BATrangejoin(L, _g(gdk, gdk.TYPE_int, rl), _g(gdk, gdk.TYPE_int, rh), sl, sr, linc, hinc)
        wa, wb = rangejoin_oidx_model(lv, lnil, idx, rl, rh, rnil, lc, rc, linc, hinc)
        assert a.to_numpy().tolist() == wa and b.to_numpy().tolist() == wb
        assert b.ptr.contents.tsorted == 1
    # without the index: the nested loop's left-major order (the oracle's)
    L2 = _g(gdk, gdk.TYPE_int, lv)
    a, b = gdk.BATrangejoin(L2, _g(gdk, gdk.TYPE_int, rl), _g(gdk, gdk.TYPE_int, rh), sl, sr)
    oa, ob = ora.BATrangejoin(ora.Bat.from_array(ora.TYPE_int, lv), ora.Bat.from_array(ora.TYPE_int, rl),
                              ora.Bat.from_array(ora.TYPE_int, rh),
                              None if sl is None else ora.Bat.from_array(ora.TYPE_oid, lc.astype(np.uint64),
                                                                          sorted_=True, key=True, nonil=True),
                              None if sr is None else ora.Bat.from_array(ora.TYPE_oid, rc.astype(np.uint64),
                                                                          sorted_=True, key=True, nonil=True))
    assert np.array_equal(a.to_numpy(), oa.values()) and np.array_equal(b.to_numpy(), ob.values())
