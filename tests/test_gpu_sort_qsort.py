"""Unstable BATsort on the device against the oracle's restatement of
BATsort + GDKqsort (gdk/gdk_batop.c:2266-2827, gdk/gdk_qsort_impl.h): which
runs the reference sorts with the quicksort (do_sort: bit / oid / flt / dbl
/ str, nils at the unnatural end, runs of <= 100 rows) and the order in
which it leaves equal values; the sizes cover the device's batched
insertion sorts (< 60 rows), its one-thread replay (60..160 rows) and its
level-parallel partition steps (more rows), with many and few ties."""
import numpy as np
import pytest

from helpers import rng

pytestmark = pytest.mark.gpu

DIRS = [(False, False), (False, True), (True, True), (True, False)]


def _pair(gdk, ora, tp_name, vals, nonil, hseq=0, vheap=None):
    tp = getattr(gdk, "TYPE_" + tp_name)
    kw = dict(sorted_=False, revsorted=False, key=False, nonil=nonil)
    d = gdk.BAT.from_numpy(tp, vals, hseqbase=hseq, vheap=vheap, **kw)
    o = ora.Bat.from_array(getattr(ora, "TYPE_" + tp_name), vals, hseqbase=hseq, vheap=vheap, **kw)
    return d, o


def _check(gdk, ora, D, O, o=None, g=None, reverse=False, nilslast=False, stable=False, float_vals=False):
    s, od, gd = gdk.BATsort(D, o[0] if o else None, g[0] if g else None, reverse=reverse, nilslast=nilslast,
                            stable=stable)
    os_, oo, og = ora.BATsort_full(O, o[1] if o else None, g[1] if g else None, reverse=reverse,
                                   nilslast=nilslast, stable=stable)
    what = (reverse, nilslast, stable)
    assert np.array_equal(np.asarray(od.values()), np.asarray(oo.values())), what
    sv, ov = s.to_numpy(), np.asarray(os_.values())
    if float_vals:
        assert np.array_equal(sv.view(np.uint8), ov.view(np.uint8)), what
    else:
        assert np.array_equal(sv, ov), what
    assert np.array_equal(np.asarray(gd.values()), np.asarray(og.values())), what
    assert (bool(s.s.tsorted), bool(s.s.trevsorted)) == (bool(os_.s.sorted), bool(os_.s.revsorted)), what
    return od


@pytest.mark.parametrize("n", [2, 45, 100, 101, 150, 700, 5000, 200_000, 2_000_000])
@pytest.mark.parametrize("card", [3, 1000])
def test_unstable_dbl(gdk, ora, n, card):
    r = rng(600 + n % 97 + card)
    v = (r.integers(0, card, n) / 4 - card / 8).astype(np.float64)
    v[r.random(n) < 0.03] = np.nan
    v[r.random(n) < 0.03] = -0.0
    D, O = _pair(gdk, ora, "dbl", v, nonil=False, hseq=9)
    for reverse, nilslast in DIRS:
        _check(gdk, ora, D, O, reverse=reverse, nilslast=nilslast, float_vals=True)


@pytest.mark.parametrize("n", [30, 100, 101, 5000])
def test_unstable_int_dispatch(gdk, ora, n):
    """int: the quicksort for <= 100 rows or nils at the unnatural end, the
    radix sort otherwise"""
    r = rng(610 + n)
    v = r.integers(-5, 5, n).astype(np.int32)
    v[r.random(n) < 0.1] = -(1 << 31)
    D, O = _pair(gdk, ora, "int", v, nonil=False)
    for reverse, nilslast in DIRS:
        for stable in (False, True):
            if stable and reverse != nilslast:
                continue
            _check(gdk, ora, D, O, reverse=reverse, nilslast=nilslast, stable=stable)


def test_unstable_oid_and_flt(gdk, ora):
    r = rng(620)
    n = 300_000
    v = r.integers(0, 50, n).astype(np.uint64) * 3
    D, O = _pair(gdk, ora, "oid", v, nonil=True)
    for reverse in (False, True):
        _check(gdk, ora, D, O, reverse=reverse, nilslast=reverse)
    f = (r.integers(-30, 30, n) / 8).astype(np.float32)
    f[r.random(n) < 0.02] = np.nan
    D, O = _pair(gdk, ora, "flt", f, nonil=False)
    for reverse, nilslast in DIRS:
        _check(gdk, ora, D, O, reverse=reverse, nilslast=nilslast, float_vals=True)


def test_unstable_presorted_and_constant(gdk, ora):
    """sorted inputs (the "no swap" insertion sort below 1024 rows, big
    equal-to-pivot blocks above) and a constant column"""
    for v in (np.arange(900, dtype=np.float64), np.arange(50_000, dtype=np.float64)[::-1].copy(),
              np.full(40_000, 2.5), np.tile(np.arange(7, dtype=np.float64), 9000)):
        D, O = _pair(gdk, ora, "dbl", v, nonil=True)
        for reverse in (False, True):
            _check(gdk, ora, D, O, reverse=reverse, nilslast=reverse, float_vals=True)


def test_unstable_subsort_runs(gdk, ora):
    """with o and g: runs of every size, each sorted on its own; int runs of
    <= 100 rows by the quicksort, longer ones by the radix sort"""
    r = rng(630)
    lens = np.concatenate([r.integers(2, 60, 300), r.integers(60, 170, 200), r.integers(170, 3000, 40),
                           [70_000]])
    r.shuffle(lens)
    n = int(lens.sum())
    a = np.repeat(np.arange(len(lens)), lens).astype(np.int32)
    perm = r.permutation(n)
    a = a[perm]                                      # first key, shuffled
    b = r.integers(0, 6, n).astype(np.int32)         # second key with ties
    c = (r.integers(0, 9, n) / 2).astype(np.float64)
    A, OA = _pair(gdk, ora, "int", a, nonil=True, hseq=3)
    s1, o1, g1 = gdk.BATsort(A)
    os1, oo1, og1 = ora.BATsort_full(OA)
    assert np.array_equal(o1.to_numpy(), oo1.values())
    Bd, Bo = _pair(gdk, ora, "int", b, nonil=True, hseq=3)
    OG = (o1, g1), (oo1, og1)
    _check(gdk, ora, Bd, Bo, o=(OG[0][0], OG[1][0]), g=(OG[0][1], OG[1][1]))
    Cd, Co = _pair(gdk, ora, "dbl", c, nonil=True, hseq=3)
    for reverse in (False, True):
        _check(gdk, ora, Cd, Co, o=(OG[0][0], OG[1][0]), g=(OG[0][1], OG[1][1]), reverse=reverse,
               nilslast=reverse, float_vals=True)


def test_unstable_str(gdk, ora):
    from strheap import build_heap, tail
    words = [b"", b"b", b"a", b"ab", b"\x80", b"zz", b"\xc3\xa9", b"abcdefghij", b"abcdefghik"]
    heap, offs = build_heap(words, 1)
    r = rng(640)
    for n in (80, 3000, 400_000):
        wi = r.integers(0, len(words), n)
        t = tail([offs[i][0] for i in wi], 1)
        D, O = _pair(gdk, ora, "str", t, nonil=False, vheap=heap)
        for reverse, nilslast in DIRS:
            _check(gdk, ora, D, O, reverse=reverse, nilslast=nilslast)


def test_sort_shortcuts(gdk, ora):
    """already sorted columns (gdk_batop.c:2422-2472) and a key g (:2633-2686):
    dense order, copied groups, the reference's flags"""
    v = np.arange(5000, dtype=np.int32) * 2
    kw = dict(sorted_=True, revsorted=False, key=True, nonil=True)
    D = gdk.BAT.from_numpy(gdk.TYPE_int, v, hseqbase=4, **kw)
    O = ora.Bat.from_array(ora.TYPE_int, v, hseqbase=4, **kw)
    s, o, g = gdk.BATsort(D, stable=False)
    os_, oo, og = ora.BATsort_full(O, stable=False)
    assert o.s.ttype == 0 and oo.s.type == 0 and o.s.tseqbase == oo.s.tseqbase == 4
    assert np.array_equal(g.to_numpy(), og.values()) and g.s.ttype == og.s.type
    gk = np.arange(5000, dtype=np.uint64)
    Gd = gdk.BAT.from_numpy(gdk.TYPE_oid, gk, sorted_=True, revsorted=False, key=True, nonil=True)
    Go = ora.Bat.from_array(ora.TYPE_oid, gk, sorted_=True, key=True, nonil=True)
    w = (v[::-1] % 7).astype(np.int32)
    Wd, Wo = _pair(gdk, ora, "int", w, nonil=True, hseq=4)
    s, o, g = gdk.BATsort(Wd, None, Gd, stable=False)
    os_, oo, og = ora.BATsort_full(Wo, None, Go, stable=False)
    assert np.array_equal(o.to_numpy(), oo.values())
    assert (bool(o.s.tsorted), bool(o.s.trevsorted)) == (bool(oo.s.sorted), bool(oo.s.revsorted))
    assert np.array_equal(g.to_numpy(), og.values())
