"""BATsort in the oracle (CPU): the reference's choice of sort function per
sorted run (do_sort, gdk/gdk_batop.c:2266-2304) and GDKqsort's order of
equal values (gdk/gdk_qsort.c, gdk_qsort_impl.h), cross-checked against an
independent Python restatement of GDKqsort (tests/qsort_py.py).  No
reference fixture holds an unstable sort's permutation of ties, so this
row is pinned by the two restatements agreeing."""
import numpy as np
import pytest

from helpers import rng
from qsort_py import gdk_qsort

NIL32 = -(1 << 31)
DIRS = [(False, False), (False, True), (True, True), (True, False)]


def _pyvals(vals, tname):
    if tname == "dbl":
        return [None if np.isnan(x) else float(x) for x in vals]
    return [None if int(x) == NIL32 else int(x) for x in vals]


def _arr(r, tname, n, card):
    if tname == "dbl":
        v = r.integers(0, card, n).astype(np.float64) / 4 - 3
        v[r.random(n) < 0.05] = np.nan
        v[r.random(n) < 0.05] = -0.0
        return v
    v = r.integers(-card, card, n).astype(np.int32)
    v[r.random(n) < 0.05] = NIL32
    return v


@pytest.mark.parametrize("tname", ["int", "dbl"])
@pytest.mark.parametrize("reverse,nilslast", DIRS)
def test_gdkqsort_two_restatements(ora, tname, reverse, nilslast):
    r = rng(500)
    tp = getattr(ora, "TYPE_" + tname)
    for n in (2, 7, 59, 60, 61, 100, 150, 500, 1023, 1500, 4000):
        for card in (3, 40, 100_000):
            v = _arr(r, tname, n, card)
            got = ora.GDKqsort(ora.Bat.from_array(tp, v), reverse, nilslast)
            want = gdk_qsort(_pyvals(v, tname), reverse, nilslast)
            assert list(got) == want, (n, card)


def test_gdkqsort_presorted_and_constant(ora):
    """the "no swap" shortcut (insertion sort below 1024 rows) and the
    equal-to-pivot blocks moved to the middle"""
    for v in (np.arange(800, dtype=np.int32), np.arange(3000, dtype=np.int32)[::-1].copy(),
              np.full(2000, 5, np.int32), np.tile(np.arange(7, dtype=np.int32), 300)):
        for reverse, nilslast in DIRS:
            got = ora.GDKqsort(ora.Bat.from_array(ora.TYPE_int, v), reverse, nilslast)
            assert list(got) == gdk_qsort([int(x) for x in v], reverse, nilslast)


def test_gdkqsort_str(ora):
    from strheap import build_heap, tail
    words = [b"", b"b", b"a", b"ab", b"\x80", b"zz", b"\xc3\xa9"]
    heap, offs = build_heap(words, 1)
    r = rng(501)
    for n in (50, 300, 2500):
        wi = r.integers(0, len(words), n)
        t = tail([offs[i][0] for i in wi], 2)
        b = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap)
        pv = [None if words[i] == b"\x80" else words[i] for i in wi]
        for reverse, nilslast in DIRS:
            assert list(ora.GDKqsort(b, reverse, nilslast)) == gdk_qsort(pv, reverse, nilslast)


def _stable_perm(pv, reverse, nilslast):
    import functools

    def cmp(i, j):
        x, y = pv[i], pv[j]
        if x is None or y is None:
            if x is None and y is None:
                return 0
            xn = x is None
            return (1 if xn else -1) if nilslast else (-1 if xn else 1)
        return (x < y) - (x > y) if reverse else (x > y) - (x < y)
    return sorted(range(len(pv)), key=functools.cmp_to_key(cmp))


@pytest.mark.parametrize("tname", ["int", "dbl"])
def test_batsort_dispatch(ora, tname):
    """int: n > 100 with nils at their natural end -> radix (stable); n <= 100
    or reverse != nilslast -> GDKqsort; dbl: GDKqsort whenever unstable"""
    r = rng(502)
    tp = getattr(ora, "TYPE_" + tname)
    for n in (80, 100, 101, 3000):
        v = _arr(r, tname, n, 10)
        pv = _pyvals(v, tname)
        for reverse, nilslast in DIRS:
            for stable in (False, True):
                if stable and reverse != nilslast:
                    with pytest.raises(ora.OracleError, match="stable sort cannot"):
                        ora.BATsort_full(ora.Bat.from_array(tp, v), reverse=reverse, nilslast=nilslast,
                                         stable=True)
                    continue
                s, o, g = ora.BATsort_full(ora.Bat.from_array(tp, v, hseqbase=5), reverse=reverse,
                                           nilslast=nilslast, stable=stable)
                qs = not stable and (tname == "dbl" or n <= 100 or reverse != nilslast)
                want = gdk_qsort(pv, reverse, nilslast) if qs else _stable_perm(pv, reverse, nilslast)
                assert list(o.values() - 5) == want, (n, reverse, nilslast, stable)
                sv = s.values()
                assert np.array_equal(sv, v[want]) or (tname == "dbl" and np.array_equal(
                    np.isnan(sv), np.isnan(v[want])))
                gv = g.values()
                ks = [pv[i] for i in want]
                wg = np.cumsum([0] + [ks[i] != ks[i - 1] for i in range(1, n)])
                assert np.array_equal(gv, wg)


def test_batsort_subsort_runs(ora):
    """with g: every run sorted on its own -- short runs of an int column by
    GDKqsort (unstable), long runs by the radix sort"""
    r = rng(503)
    n = 4000
    runs = np.repeat(np.arange(25), r.integers(20, 300, 25))[:n]
    n = len(runs)
    gcol = np.sort(runs).astype(np.uint64)
    v = r.integers(0, 6, n).astype(np.int32)
    G = ora.Bat.from_array(ora.TYPE_oid, gcol, sorted_=True)
    s, o, g = ora.BATsort_full(ora.Bat.from_array(ora.TYPE_int, v), None, G, stable=False)
    got = o.values()
    start = 0
    for k in range(n + 1):
        if k == n or (k > 0 and gcol[k] != gcol[k - 1]):
            seg = [int(x) for x in v[start:k]]
            want = gdk_qsort(seg) if k - start <= 100 else _stable_perm(seg, False, False)
            assert list(got[start:k] - start) == want
            start = k
