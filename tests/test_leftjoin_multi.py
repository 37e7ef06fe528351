"""The left-output join family with SEVERAL matches per left candidate:
BATleftjoin, BATouterjoin, BATsemijoin with its right output (the form
algebra.semijoin binds, monetdb5/modules/kernel/algebra.c:1792) and
BATmarkjoin with r2 (gdk/gdk_join.c:4320-4407, all through leftjoin :4049).

Which matches a left candidate has does not depend on the algorithm leftjoin
picks; their order and the one a semi join keeps do:
  selectjoin  ascending, semi the first;
  mergejoin   ascending, semi the LAST when l and r are scanned in the same
              order (both ascending, or l unordered), else the first;
  hashjoin    descending (hash chains are built by prepending), semi the last;
  swapped hashjoin (leftjoin / semi without max_one, when hashing l is
              cheaper): hashjoin(r, l)'s pairs -- right candidates in order,
              each one's left matches descending -- sorted by GDKqsort on the
              left oids; semi first reduces r to BATunique (first occurrences)
              so it keeps the first match;
  fetchjoin   (dense l) pairs in right position order -- the left candidates
              descending for a reverse-sorted r -- and no nil rows for misses.
The oracle restates the choice (oracle/gdk_oracle_join.c ora_leftjoin_ex);
here it is checked against a Python model of those orders (the swapped
join's tie order through the independent Python GDKqsort restatement,
tests/qsort_py.py), and the device against the oracle on every shape and
candidate form.  No reference fixture holds these results: parity unpinned
beyond the model."""
import numpy as np
import pytest

from helpers import rng
from qsort_py import gdk_qsort

NI = -(1 << 31)
NL = -(1 << 63)
ONIL = 1 << 63


def _shapes():
    """(name, type, l values, r values, flags, expected algorithm, equal_order)"""
    r = rng(1401)
    i32 = np.int32
    lk = r.integers(0, 5000, 20_000).astype(i32)
    lk[::101] = NI
    rk = r.integers(0, 6000, 8000).astype(i32)
    rk[5] = NI
    yield "hash", "int", lk, rk, {}, "hashjoin", True
    # r of ten values, 2000 rows each; l 3000 distinct values: hashing l wins
    ls = r.choice(100_000, 3000, replace=False).astype(i32)
    ls[:40] = np.arange(40) % 10
    yield "swap", "int", ls, r.integers(0, 10, 20_000).astype(i32), {}, "hashjoin_swapped", True
    yield "merge_eq", "int", np.sort(lk), np.sort(rk), {}, "mergejoin", True
    yield "merge_rev", "int", np.sort(lk), np.sort(rk)[::-1].copy(), {}, "mergejoin", False
    yield "merge_lunsorted", "int", r.integers(0, 300, 900).astype(i32), np.sort(r.integers(0, 400, 3000)).astype(i32), \
        {}, "mergejoin", True
    yield "select", "int", np.full(3000, 77, i32), r.integers(0, 100, 5000).astype(i32), {}, "selectjoin", True
    yield "select_miss", "int", np.full(300, 1234, i32), r.integers(0, 100, 500).astype(i32), {}, "selectjoin", True
    ll, rl = lk.astype(np.int64) * 1_000_003, rk.astype(np.int64) * 1_000_003
    ll[lk == NI] = NL
    rl[rk == NI] = NL
    yield "lng_hash", "lng", ll, rl, {}, "hashjoin", True


def _fetch_shapes():
    """l dense (void), r a sorted / reverse-sorted oid column with repeats"""
    r = rng(1402)
    v = np.sort(r.integers(50, 2600, 6000)).astype(np.uint64)
    return [("fetch_asc", v, False), ("fetch_desc", v[::-1].copy(), True)]


def _cands(r, n, form):
    if form == "none" or n == 0:
        return None
    if form == "dense":
        return ("dense", 3, max(0, n - 7))
    return ("oids", np.sort(r.choice(n, (2 * n) // 3, replace=False)).astype(np.uint64))


def _oids(c, n):
    if c is None:
        return np.arange(n, dtype=np.uint64)
    if c[0] == "dense":
        return np.arange(c[1], c[1] + c[2], dtype=np.uint64)
    return c[1]


def _ora_c(ora, c):
    if c is None:
        return None
    if c[0] == "dense":
        return ora.Bat.dense(c[1], c[2])
    return ora.Bat.from_array(ora.TYPE_oid, c[1], sorted_=True, key=True, nonil=True)


def _gdk_c(gdk, c, form="plain"):
    if c is None:
        return None
    if c[0] == "dense":
        return gdk.BAT.dense(c[1], c[2])
    if form == "except" and len(c[1]):
        lo, hi = int(c[1][0]), int(c[1][-1]) + 1
        exc = np.setdiff1d(np.arange(lo, hi, dtype=np.uint64), c[1])
        return gdk.BAT.negoid_cand(lo, len(c[1]), exc)
    return gdk.BAT.from_numpy(gdk.TYPE_oid, c[1], sorted_=True, key=True, nonil=True)


def _matches(lv, rv, lc, rc, nilv):
    """per left candidate: its right candidates with an equal value, ascending"""
    from collections import defaultdict
    pos = defaultdict(list)
    for o in rc:
        if rv[o] != nilv:
            pos[rv[o]].append(int(o))
    return [(int(o), pos.get(lv[o], []) if lv[o] != nilv else []) for o in lc]


def _model(algo, eqo, m, rv, rc, mode):
    """(r1, r2) of leftjoin in `mode` (left / outer / semi) per the rules above"""
    if algo == "hashjoin_swapped" and mode == "left":
        byl = {o: ms for o, ms in m}
        inv = {}
        for o, ms in m:
            for x in ms:
                inv.setdefault(x, []).append(o)
        pairs = [(lo, int(ro)) for ro in rc for lo in sorted(inv.get(int(ro), []), reverse=True)]
        del byl
        perm = gdk_qsort([p[0] for p in pairs])
        # GDKqsort moves the payload with its key
        return [pairs[k][0] for k in perm], [pairs[k][1] for k in perm]
    a, b = [], []
    for o, ms in m:
        if not ms:
            if mode == "outer":
                a.append(o)
                b.append(ONIL)
            continue
        if mode == "semi":
            last = algo == "hashjoin" or (algo == "mergejoin" and eqo)
            a.append(o)
            b.append(ms[-1] if last else ms[0])
            continue
        for x in (ms[::-1] if algo == "hashjoin" else ms):
            a.append(o)
            b.append(x)
    return a, b


@pytest.mark.parametrize("name,tname,lv,rv,kw,algo,eqo", list(_shapes()))
@pytest.mark.parametrize("mode", ["left", "outer", "semi"])
def test_oracle_leftjoin_multi_model(ora, name, tname, lv, rv, kw, algo, eqo, mode):
    tp = getattr(ora, "TYPE_" + tname)
    nilv = {"int": NI, "lng": NL}[tname]
    L, R = ora.Bat.from_array(tp, lv), ora.Bat.from_array(tp, rv)
    m = _matches(lv, rv, range(len(lv)), range(len(rv)), nilv)
    a, b, _, got_algo = ora.leftjoin_ex(L, R, nil_on_miss=mode == "outer", semi=mode == "semi")
    # the swapped join is leftjoin's / semi's only: outer joins hash r
    want_algo = "hashjoin" if algo == "hashjoin_swapped" and mode == "outer" else algo
    assert got_algo == want_algo
    wa, wb = _model(want_algo, eqo, m, rv, range(len(rv)), mode)
    assert [int(x) for x in a.values()] == wa
    assert [int(x) for x in b.values()] == wb


@pytest.mark.parametrize("name,v,rev", _fetch_shapes())
def test_oracle_fetchjoin_order(ora, name, v, rev):
    """dense l against a sorted / reverse-sorted oid column: fetchjoin's rows
    in right position order, misses dropped even for an outer join"""
    L = ora.Bat.dense(100, 3000)
    R = ora.Bat.from_array(ora.TYPE_oid, v, nonil=True)
    for outer in (False, True):
        a, b, _, al = ora.leftjoin_ex(L, R, nil_on_miss=outer)
        assert al == "fetchjoin"
        want = [(int(x), p) for p, x in enumerate(v) if 100 <= x < 3100]
        assert [int(x) for x in a.values()] == [x - 100 for x, _ in want]
        assert [int(x) for x in b.values()] == [p for _, p in want]


def test_oracle_select_min_one(ora):
    """BATouterjoin(match_one) raises 'not enough matches' only on selectjoin"""
    L = ora.Bat.from_array(ora.TYPE_int, np.full(50, 999, np.int32))
    R = ora.Bat.from_array(ora.TYPE_int, np.arange(100, dtype=np.int32))
    with pytest.raises(Exception, match="not enough matches"):
        ora.leftjoin_ex(L, R, nil_on_miss=True, max_one=True, min_one=True)
    L = ora.Bat.from_array(ora.TYPE_int, np.array([999, 5, 7] * 20, np.int32))
    a, b, _, al = ora.leftjoin_ex(L, R, nil_on_miss=True, max_one=True, min_one=True)
    assert al != "selectjoin" and b.values()[0] == ONIL


def test_oracle_diff_sorted_l_skips_nils(ora):
    """BATdiff over a sorted l with nils: mergejoin skips them (gdk_join.c:
    2093-2100), the hash path lists them"""
    lv = np.array([NI, NI, 1, 2, 3, 5, 8, 9] * 200, np.int32)
    rv = np.sort(np.array([2, 3, 4] * 100, np.int32))
    got = ora.BATdiff(ora.Bat.from_array(ora.TYPE_int, np.sort(lv)), ora.Bat.from_array(ora.TYPE_int, rv))
    s = np.sort(lv)
    assert [int(x) for x in got.values()] == [i for i, x in enumerate(s) if x not in (NI, 2, 3)]
    # unsorted l, unsorted r of many rows: the hash path lists the nils
    rr = rng(7).permutation(np.repeat(np.arange(0, 3000, dtype=np.int32), 2))
    got = ora.BATdiff(ora.Bat.from_array(ora.TYPE_int, lv), ora.Bat.from_array(ora.TYPE_int, rr))
    assert [int(x) for x in got.values()] == [i for i, x in enumerate(lv) if not (0 <= x < 3000)]


def _gdk_out(x):
    return np.asarray(x.to_numpy()).astype(np.uint64)


def _ora_out(x):
    return np.asarray(x.values()).astype(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("name,tname,lv,rv,kw,algo,eqo", list(_shapes()))
@pytest.mark.parametrize("cform", ["none", "dense", "oids", "except"])
def test_gpu_leftjoin_multi(gdk, ora, name, tname, lv, rv, kw, algo, eqo, cform):
    r = rng(1403)
    tg, to = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    lcs = _cands(r, len(lv), "oids" if cform == "except" else cform)
    rcs = _cands(r, len(rv), "dense" if cform == "except" else cform)
    sort_l = name.startswith("merge") and name != "merge_lunsorted"
    mk = lambda v, s: gdk.BAT.from_numpy(tg, v, sorted_=False, revsorted=False, key=False)  # noqa: E731
    L, R = mk(lv, sort_l), mk(rv, False)
    OL, OR = ora.Bat.from_array(to, lv), ora.Bat.from_array(to, rv)
    gl, gr, ol, orr = _gdk_c(gdk, lcs, cform), _gdk_c(gdk, rcs, cform), _ora_c(ora, lcs), _ora_c(ora, rcs)
    a, b = gdk.BATleftjoin(L, R, gl, gr)
    wa, wb, _, _ = ora.leftjoin_ex(OL, OR, ol, orr)
    assert np.array_equal(_gdk_out(a), _ora_out(wa)) and np.array_equal(_gdk_out(b), _ora_out(wb))
    a, b = gdk.BATouterjoin(L, R, gl, gr)
    wa, wb, _, _ = ora.leftjoin_ex(OL, OR, ol, orr, nil_on_miss=True)
    assert np.array_equal(_gdk_out(a), _ora_out(wa)) and np.array_equal(_gdk_out(b), _ora_out(wb))
    assert bool(b.s.tnil) == bool((_ora_out(wb) == ONIL).any())
    a, b = gdk.BATsemijoin(L, R, gl, gr, want_r2=True)
    wa, wb, _, _ = ora.leftjoin_ex(OL, OR, ol, orr, semi=True)
    assert np.array_equal(_gdk_out(a), _ora_out(wa)) and np.array_equal(_gdk_out(b), _ora_out(wb))
    a, b, c = gdk.BATmarkjoin(L, R, gl, gr)
    wa, wb, wc, _ = ora.leftjoin_ex(OL, OR, ol, orr, nil_on_miss=True, want_r3=True)
    assert np.array_equal(_gdk_out(a), _ora_out(wa)) and np.array_equal(_gdk_out(b), _ora_out(wb))
    assert np.array_equal(c.to_numpy().astype(np.int8), np.asarray(wc.values()).astype(np.int8))
    # the left output alone is unchanged by the algorithm
    assert np.array_equal(_gdk_out(gdk.BATsemijoin(L, R, gl, gr)), _ora_out(ora.BATintersect(OL, OR, ol, orr)))
    if (_ora_out(wb) == ONIL).any() or len(set(_ora_out(wa).tolist())) < len(wa.values()):
        with pytest.raises(gdk.GDKError, match="more than one match|not enough matches"):
            gdk.BATouterjoin(L, R, gl, gr, match_one=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name,v,rev", _fetch_shapes())
def test_gpu_fetchjoin_order(gdk, ora, name, v, rev):
    L = gdk.BAT.dense(100, 3000)
    R = gdk.BAT.from_numpy(gdk.TYPE_oid, v, sorted_=False, revsorted=False, key=False, nonil=True)
    OL, OR = ora.Bat.dense(100, 3000), ora.Bat.from_array(ora.TYPE_oid, v, nonil=True)
    for outer in (False, True):
        a, b = (gdk.BATouterjoin if outer else gdk.BATleftjoin)(L, R)
        wa, wb, _, al = ora.leftjoin_ex(OL, OR, nil_on_miss=outer)
        assert al == "fetchjoin"
        assert np.array_equal(_gdk_out(a), _ora_out(wa)) and np.array_equal(_gdk_out(b), _ora_out(wb))
        assert bool(a.s.trevsorted) == rev or a.count() <= 1


@pytest.mark.gpu
def test_gpu_select_min_one(gdk):
    L = gdk.BAT.from_numpy(gdk.TYPE_int, np.full(50, 999, np.int32))
    R = gdk.BAT.from_numpy(gdk.TYPE_int, np.arange(100, dtype=np.int32))
    with pytest.raises(gdk.GDKError, match="not enough matches"):
        gdk.BATouterjoin(L, R, match_one=True)


@pytest.mark.gpu
def test_gpu_diff_sorted_l_skips_nils(gdk, ora):
    lv = np.sort(np.array([NI, NI, 1, 2, 3, 5, 8, 9] * 200, np.int32))
    rv = np.sort(np.array([2, 3, 4] * 100, np.int32))
    got = gdk.BATdiff(gdk.BAT.from_numpy(gdk.TYPE_int, lv, sorted_=False, revsorted=False, key=False),
                      gdk.BAT.from_numpy(gdk.TYPE_int, rv, sorted_=False, revsorted=False, key=False))
    want = ora.BATdiff(ora.Bat.from_array(ora.TYPE_int, lv), ora.Bat.from_array(ora.TYPE_int, rv))
    assert np.array_equal(_gdk_out(got), _ora_out(want))
    assert not (lv[_gdk_out(got).astype(np.int64)] == NI).any()


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["flt", "dbl", "str"])
def test_gpu_leftjoin_float_str_keys(gdk, ora, tname):
    """flt / dbl / str keys through BATjoin's integer images: -0.0 == +0.0,
    NaN the nil; strings by content"""
    r = rng(1404)
    if tname == "str":
        from strheap import ELIMLIMIT, build_heap, tail
        words = [b"w%03d" % k for k in range(300)] + [b"\x80"]
        heap, offs = build_heap(words, 3, pad_to=ELIMLIMIT + 512, rng=r)

        def side(n, hi):
            wi = r.integers(0, hi, n)
            t = tail([offs[w][c] for w, c in zip(wi, r.integers(0, 3, n))], 4)
            return (gdk.BAT.from_numpy(gdk.TYPE_str, t, vheap=heap, sorted_=False, revsorted=False, key=False,
                                       nonil=False),
                    ora.Bat.from_array(ora.TYPE_str, t, vheap=heap))
        (L, OL), (R, OR) = side(5000, len(words)), side(3000, 250)
    else:
        dt = np.float32 if tname == "flt" else np.float64
        lv = (r.integers(-300, 300, 6000) / 4).astype(dt)
        rv = (r.integers(-300, 300, 4000) / 4).astype(dt)
        lv[::97] = np.nan
        rv[::131] = -0.0
        lv[::89] = 0.0
        tg, to = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
        L = gdk.BAT.from_numpy(tg, lv, sorted_=False, revsorted=False, key=False)
        R = gdk.BAT.from_numpy(tg, rv, sorted_=False, revsorted=False, key=False)
        OL, OR = ora.Bat.from_array(to, lv), ora.Bat.from_array(to, rv)
    for mode in ("left", "outer", "semi"):
        if mode == "semi":
            a, b = gdk.BATsemijoin(L, R, want_r2=True)
        else:
            a, b = (gdk.BATouterjoin if mode == "outer" else gdk.BATleftjoin)(L, R)
        wa, wb, _, _ = ora.leftjoin_ex(OL, OR, nil_on_miss=mode == "outer", semi=mode == "semi")
        assert np.array_equal(_gdk_out(a), _ora_out(wa)), mode
        assert np.array_equal(_gdk_out(b), _ora_out(wb)), mode
