"""The left-output join family: BATintersect, BATsemijoin (candidate
output), BATdiff (with SQL NOT IN semantics), BATleftjoin and BATouterjoin
(gdk/gdk_join.c:4320-4407, all through leftjoin :4049).

Their results do not depend on which of leftjoin's algorithms runs: the
left candidates in order, with or without a match among the right
candidates (and the match).  The oracle restates that definition with the
reference's nil rules (a nil matches only with nil_matches; NOT IN drops
nil left values and returns nothing when a right candidate is nil, except
on the dense-right path mergejoin_void, which has no not_in; empty sides
give nomatch; max_one / match_one raise "more than one match"); it is
checked against a brute-force pair model here, and the device against the
oracle on every shape that selects a different leftjoin algorithm (single
left value, dense right, dense left, both sorted, hash), with candidate
lists in every form.  No reference fixture holds these (parity unpinned
beyond the pair model).  Several matches per left candidate:
test_leftjoin_multi.py."""
import numpy as np
import pytest

from helpers import rng

NI, NL = -(1 << 31), -(1 << 63)
ONIL = 1 << 63


def _shapes():
    r = rng(1301)
    i32 = np.int32
    rk = r.choice(50_000, 20_000, replace=False).astype(i32)                 # unique right keys
    lk = r.integers(0, 60_000, 80_000).astype(i32)
    lk[::97] = NI
    rkn = rk.copy()
    rkn[7] = NI                                                              # a nil on the right
    yield "hash_unique", "int", lk, rk, {}
    yield "hash_unique_rnil", "int", lk, rkn, {}
    yield "hash_dups", "int", lk, r.integers(0, 60_000, 30_000).astype(i32), {"dups": True}
    yield "sorted_both", "int", np.sort(lk), np.sort(rk), {}
    yield "single_left", "int", np.full(5000, 4242, i32), np.append(rk, np.int32(4242)), {}
    yield "lng_cands", "lng", lk.astype(np.int64), rk.astype(np.int64), {"cands": True}
    yield "small", "sht", r.integers(-50, 50, 3000).astype(np.int16), r.choice(np.arange(-60, 60), 80,
                                                                             replace=False).astype(np.int16), {}
    yield "empty_right", "int", lk[:1000], np.zeros(0, i32), {}
    yield "empty_left", "int", np.zeros(0, i32), rk, {}


def _dense_right_shape():
    """oid keys against a dense (void) right side: mergejoin_void"""
    r = rng(1302)
    lv = r.integers(0, 3000, 20_000).astype(np.uint64)
    lv[::53] = ONIL
    return lv, (1000, 1200)


def _cands(r, n, form):
    if form == "none":
        return None
    if form == "dense":
        return ("dense", 5, max(0, n - 9))
    return ("oids", np.sort(r.choice(n, n // 2, replace=False)).astype(np.uint64)) if n else None


def _model(lv, rv, lc, rc, nil_matches, nilv):
    """per left candidate (in order): the right candidate oids with an equal value"""
    from collections import defaultdict
    pos = defaultdict(list)
    for o in rc:
        v = rv[o]
        if v == nilv and not nil_matches:
            continue
        pos[v].append(o)
    return [(o, pos.get(lv[o], []) if not (lv[o] == nilv and not nil_matches) else []) for o in lc]


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


@pytest.mark.parametrize("name,tname,lv,rv,kw", list(_shapes()))
@pytest.mark.parametrize("nil_matches", [False, True])
def test_oracle_join_kinds_model(ora, name, tname, lv, rv, kw, nil_matches):
    r = rng(1303)
    tp = getattr(ora, "TYPE_" + tname)
    nilv = {"int": NI, "lng": NL, "sht": -(1 << 15)}[tname]
    lcs = _cands(r, len(lv), "oids") if kw.get("cands") else None
    rcs = _cands(r, len(rv), "dense") if kw.get("cands") else None
    L, R = ora.Bat.from_array(tp, lv), ora.Bat.from_array(tp, rv)
    m = _model(lv, rv, _oids(lcs, len(lv)), _oids(rcs, len(rv)), nil_matches, nilv)
    semi = [o for o, ms in m if ms]
    got = ora.BATintersect(L, R, _ora_c(ora, lcs), _ora_c(ora, rcs), nil_matches)
    assert [int(x) for x in got.values()] == semi
    # mergejoin over a sorted l skips l's nils before its scan (gdk_join.c:
    # 2093-2100): BATdiff does not list them there (test_leftjoin_multi.py)
    skipnil = name == "sorted_both" and not nil_matches
    anti = [o for o, ms in m if not ms and not (skipnil and lv[o] == nilv)]
    assert [int(x) for x in ora.BATdiff(L, R, _ora_c(ora, lcs), _ora_c(ora, rcs), nil_matches).values()] == anti
    # NOT IN: nil left values dropped; a nil right candidate empties it
    rnil = any(rv[o] == nilv for o in _oids(rcs, len(rv)))
    notin = [] if rnil else [o for o, ms in m if not ms and lv[o] != nilv]
    if len(lv) and len(rv):
        got = ora.BATdiff(L, R, _ora_c(ora, lcs), _ora_c(ora, rcs), nil_matches, not_in=True)
        assert [int(x) for x in got.values()] == notin
    res = ora.BATleftjoin(L, R, _ora_c(ora, lcs), _ora_c(ora, rcs), nil_matches, outer=True)
    if any(len(ms) > 1 for _, ms in m):
        assert res is None
        with pytest.raises(Exception, match="more than one match"):
            ora.BATleftjoin(L, R, _ora_c(ora, lcs), _ora_c(ora, rcs), nil_matches, outer=True, match_one=True)
    else:
        a, b = res
        assert [int(x) for x in a.values()] == [o for o, _ in m]
        assert [int(x) for x in b.values()] == [ms[0] if ms else ONIL for _, ms in m]


def test_oracle_not_in_dense_right(ora):
    """mergejoin_void has no not_in: nil left values stay misses"""
    lv, (seq, n) = _dense_right_shape()
    L, R = ora.Bat.from_array(ora.TYPE_oid, lv), ora.Bat.dense(seq, n)
    got = [int(x) for x in ora.BATdiff(L, R, None, None, False, not_in=True).values()]
    assert got == [i for i in range(len(lv)) if not (seq <= lv[i] < seq + n)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,tname,lv,rv,kw", list(_shapes()))
@pytest.mark.parametrize("nil_matches", [False, True])
@pytest.mark.parametrize("cform", ["plain", "except"])
def test_gpu_join_kinds(gdk, ora, name, tname, lv, rv, kw, nil_matches, cform):
    r = rng(1304)
    tg, to = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    lcs = _cands(r, len(lv), "oids") if kw.get("cands") else None
    rcs = _cands(r, len(rv), "dense") if kw.get("cands") else None
    mk = lambda v: gdk.BAT.from_numpy(tg, v, sorted_=False, revsorted=False, key=False)   # noqa: E731
    L, R = mk(lv), mk(rv)
    OL, OR = ora.Bat.from_array(to, lv), ora.Bat.from_array(to, rv)
    gl, gr, ol, orr = _gdk_c(gdk, lcs, cform), _gdk_c(gdk, rcs, cform), _ora_c(ora, lcs), _ora_c(ora, rcs)
    eq = lambda g, o: np.array_equal(g.to_numpy().astype(np.uint64), np.asarray(o.values(), np.uint64))  # noqa
    assert eq(gdk.BATintersect(L, R, gl, gr, nil_matches), ora.BATintersect(OL, OR, ol, orr, nil_matches))
    assert eq(gdk.BATsemijoin(L, R, gl, gr, nil_matches), ora.BATintersect(OL, OR, ol, orr, nil_matches))
    for not_in in (False, True):
        assert eq(gdk.BATdiff(L, R, gl, gr, nil_matches, not_in), ora.BATdiff(OL, OR, ol, orr, nil_matches, not_in))
    res = ora.BATleftjoin(OL, OR, ol, orr, nil_matches, outer=True)
    if res is None:
        with pytest.raises(gdk.GDKError, match="more than one match"):
            gdk.BATouterjoin(L, R, gl, gr, nil_matches, match_one=True)
        with pytest.raises(gdk.GDKError, match="more than one match"):
            gdk.BATintersect(L, R, gl, gr, nil_matches, max_one=True)
        # several matches: the order leftjoin's algorithm gives them
        # (tests/test_leftjoin_multi.py)
        a, b = gdk.BATleftjoin(L, R, gl, gr, nil_matches)
        wa, wb, _, _ = ora.leftjoin_ex(OL, OR, ol, orr, nil_matches)
        assert eq(a, wa) and eq(b, wb)
        a, b = gdk.BATouterjoin(L, R, gl, gr, nil_matches)
        wa, wb, _, _ = ora.leftjoin_ex(OL, OR, ol, orr, nil_matches, nil_on_miss=True)
        assert eq(a, wa) and eq(b, wb)
    else:
        a, b = gdk.BATouterjoin(L, R, gl, gr, nil_matches)
        assert eq(a, res[0]) and eq(b, res[1])
        a, b = gdk.BATleftjoin(L, R, gl, gr, nil_matches)
        wa, wb = ora.BATleftjoin(OL, OR, ol, orr, nil_matches, outer=False)
        assert eq(a, wa) and eq(b, wb)


@pytest.mark.gpu
def test_gpu_not_in_dense_right(gdk, ora):
    lv, (seq, n) = _dense_right_shape()
    L = gdk.BAT.from_numpy(gdk.TYPE_oid, lv, sorted_=False, revsorted=False, key=False)
    got = gdk.BATdiff(L, gdk.BAT.dense(seq, n), None, None, False, True).to_numpy()
    want = ora.BATdiff(ora.Bat.from_array(ora.TYPE_oid, lv), ora.Bat.dense(seq, n), None, None, False, True)
    assert np.array_equal(got.astype(np.uint64), np.asarray(want.values(), np.uint64))


def _mark_model(lv, rv, lc, rc, nilv):
    """BATmarkjoin's mark per left candidate -- SQL's three-valued IN: TRUE on
    a match; else nil when the left value or a right candidate is nil; FALSE;
    no right candidates at all: FALSE (gdk_join.c:4144, nomatch defmark 0)"""
    m = _model(lv, rv, lc, rc, False, nilv)
    if len(rc) == 0:
        return [0] * len(m)
    rnil = any(rv[o] == nilv for o in rc)
    return [1 if ms else (-128 if (lv[o] == nilv or rnil) else 0) for o, ms in m]


@pytest.mark.parametrize("name,tname,lv,rv,kw", list(_shapes()))
def test_oracle_markjoin_model(ora, name, tname, lv, rv, kw):
    r = rng(1305)
    tp = getattr(ora, "TYPE_" + tname)
    nilv = {"int": NI, "lng": NL, "sht": -(1 << 15)}[tname]
    lcs = _cands(r, len(lv), "oids") if kw.get("cands") else None
    rcs = _cands(r, len(rv), "dense") if kw.get("cands") else None
    L, R = ora.Bat.from_array(tp, lv), ora.Bat.from_array(tp, rv)
    lc, rc = _oids(lcs, len(lv)), _oids(rcs, len(rv))
    m = _model(lv, rv, lc, rc, False, nilv)
    marks = _mark_model(lv, rv, lc, rc, nilv)
    a, c = ora.BATmarkjoin(L, R, _ora_c(ora, lcs), _ora_c(ora, rcs), want_r2=False)
    assert [int(x) for x in a.values()] == [int(o) for o in lc]
    assert [int(x) for x in c.values()] == marks
    assert bool(c.s.nil) == (-128 in marks)
    res = ora.BATmarkjoin(L, R, _ora_c(ora, lcs), _ora_c(ora, rcs))
    if any(len(ms) > 1 for _, ms in m):
        assert res is None
    else:
        a, b, c = res
        assert [int(x) for x in b.values()] == [ms[0] if ms else ONIL for _, ms in m]
        assert [int(x) for x in c.values()] == marks


@pytest.mark.gpu
@pytest.mark.parametrize("name,tname,lv,rv,kw", list(_shapes()))
@pytest.mark.parametrize("cform", ["plain", "except"])
def test_gpu_markjoin(gdk, ora, name, tname, lv, rv, kw, cform):
    r = rng(1306)
    tg, to = getattr(gdk, "TYPE_" + tname), getattr(ora, "TYPE_" + tname)
    lcs = _cands(r, len(lv), "oids") if kw.get("cands") else None
    rcs = _cands(r, len(rv), "dense") if kw.get("cands") else None
    mk = lambda v: gdk.BAT.from_numpy(tg, v, sorted_=False, revsorted=False, key=False)   # noqa: E731
    L, R = mk(lv), mk(rv)
    OL, OR = ora.Bat.from_array(to, lv), ora.Bat.from_array(to, rv)
    gl, gr, ol, orr = _gdk_c(gdk, lcs, cform), _gdk_c(gdk, rcs, cform), _ora_c(ora, lcs), _ora_c(ora, rcs)

    def eq(g, o, dt=np.uint64):
        return np.array_equal(g.to_numpy().astype(dt), np.asarray(o.values()).astype(dt))

    a, c = gdk.BATmarkjoin(L, R, gl, gr, want_r2=False)
    wa, wc = ora.BATmarkjoin(OL, OR, ol, orr, want_r2=False)
    assert eq(a, wa) and eq(c, wc, np.int8)
    assert bool(c.s.tnil) == bool(wc.s.nil)
    res = ora.BATmarkjoin(OL, OR, ol, orr)
    if res is None:
        a, b, c = gdk.BATmarkjoin(L, R, gl, gr)
        wa, wb, wc, _ = ora.leftjoin_ex(OL, OR, ol, orr, nil_on_miss=True, want_r3=True)
        assert eq(a, wa) and eq(b, wb) and eq(c, wc, np.int8)
    else:
        a, b, c = gdk.BATmarkjoin(L, R, gl, gr)
        assert eq(a, res[0]) and eq(b, res[1]) and eq(c, res[2], np.int8)


@pytest.mark.gpu
def test_gpu_markjoin_dense_right(gdk, ora):
    """oid keys against a dense right side (mergejoin_void): nil left values
    give a nil mark, the rest TRUE / FALSE"""
    lv, (seq, n) = _dense_right_shape()
    L = gdk.BAT.from_numpy(gdk.TYPE_oid, lv, sorted_=False, revsorted=False, key=False)
    a, b, c = gdk.BATmarkjoin(L, gdk.BAT.dense(seq, n))
    wa, wb, wc = ora.BATmarkjoin(ora.Bat.from_array(ora.TYPE_oid, lv), ora.Bat.dense(seq, n))
    assert np.array_equal(b.to_numpy().astype(np.uint64), np.asarray(wb.values(), np.uint64))
    assert np.array_equal(c.to_numpy().astype(np.int8), np.asarray(wc.values()).astype(np.int8))
