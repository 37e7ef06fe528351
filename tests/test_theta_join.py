"""BATthetajoin (gdk/gdk_join.c:4409, the nested loop thetajoin :3699) and
BATbandjoin (:4626): the pairs in left-candidate order, each left
candidate's matches in right-candidate order.

The oracle restates the reference's nested loops (ATOMcompare with nil
smallest and -0.0 == +0.0 for theta; the per-type band arithmetic with its
widening and, for dbl, SUBF / ADDF_WITH_CHECK's goto rules) and is checked
here against a brute-force numpy model; the device is checked against the
oracle on every operator, nil rule, candidate form and type -- including the
float band cases the device evaluates pair by pair.  No reference fixture
holds thetajoin / bandjoin answers (parity unpinned beyond the model)."""
import numpy as np
import pytest

from helpers import rng

OPS = {"lt": -1, "le": -2, "gt": 1, "ge": 2, "ne": -3}
NILS = {"int": -(1 << 31), "lng": -(1 << 63), "sht": -(1 << 15)}


def _col(r, n, tname, lo=-60, hi=60, nil_frac=0.05):
    if tname in ("flt", "dbl"):
        v = np.round(r.uniform(lo, hi, n) * 4) / 4
        v[r.random(n) < nil_frac] = np.nan
        v[r.random(n) < 0.03] = -0.0
        return v.astype(np.float32 if tname == "flt" else np.float64)
    v = r.integers(lo, hi, n).astype(np.int64)
    v[r.random(n) < nil_frac] = NILS[tname]
    return v.astype({"int": np.int32, "lng": np.int64, "sht": np.int16}[tname])


def _isnil(v):
    return np.isnan(v) if v.dtype.kind == "f" else v == np.iinfo(v.dtype).min


def _model_theta(lv, rv, lo, ro, op, nil_matches):
    out1, out2 = [], []
    for i in lo:
        a = lv[i]
        an = bool(_isnil(np.array([a]))[0])
        if an and not nil_matches:
            continue
        for j in ro:
            b = rv[j]
            bn = bool(_isnil(np.array([b]))[0])
            if bn and not nil_matches:
                continue
            c = 0 if (an and bn) else (-1 if an else (1 if bn else (int(a > b) - int(a < b))))
            ok = {"lt": c < 0, "le": c <= 0, "gt": c > 0, "ge": c >= 0, "ne": c != 0}[op]
            if ok:
                out1.append(i)
                out2.append(j)
    return out1, out2


def _mk(mod, tname, v):
    tp = getattr(mod, "TYPE_" + tname)
    if hasattr(mod, "Bat"):
        return mod.Bat.from_array(tp, v)
    return mod.BAT.from_numpy(tp, v, sorted_=False, revsorted=False, key=False)


@pytest.mark.parametrize("tname", ["int", "dbl"])
@pytest.mark.parametrize("op", list(OPS))
@pytest.mark.parametrize("nil_matches", [False, True])
def test_oracle_thetajoin_model(ora, tname, op, nil_matches):
    r = rng(1601)
    lv, rv = _col(r, 70, tname), _col(r, 50, tname)
    a, b = ora.BATthetajoin(_mk(ora, tname, lv), _mk(ora, tname, rv), None, None, OPS[op], nil_matches)
    w1, w2 = _model_theta(lv, rv, range(len(lv)), range(len(rv)), op, nil_matches)
    assert [int(x) for x in a.values()] == w1 and [int(x) for x in b.values()] == w2


def test_oracle_bandjoin_model(ora):
    r = rng(1602)
    lv, rv = _col(r, 80, "int"), _col(r, 60, "int")
    for c1, c2, li, hi in ((3, 5, True, True), (3, 5, False, True), (0, 0, True, True), (7, -2, True, False)):
        a, b = ora.BATbandjoin(_mk(ora, "int", lv), _mk(ora, "int", rv), c1, c2, linc=li, hinc=hi)
        w1, w2 = [], []
        for i, x in enumerate(lv):
            if x == NILS["int"]:
                continue
            for j, y in enumerate(rv):
                if y == NILS["int"]:
                    continue
                lo_ok = x >= y - c1 if li else x > y - c1
                hi_ok = x <= y + c2 if hi else x < y + c2
                if lo_ok and hi_ok:
                    w1.append(i)
                    w2.append(j)
        assert [int(v) for v in a.values()] == w1 and [int(v) for v in b.values()] == w2, (c1, c2, li, hi)


def _cands(gdk, ora, r, n, form):
    if form == "none":
        return None, None
    if form == "dense":
        return gdk.BAT.dense(3, n - 7), ora.Bat.dense(3, n - 7)
    c = np.sort(r.choice(n, n // 2, replace=False)).astype(np.uint64)
    return (gdk.BAT.from_numpy(gdk.TYPE_oid, c, sorted_=True, key=True, nonil=True),
            ora.Bat.from_array(ora.TYPE_oid, c, sorted_=True, key=True, nonil=True))


def _eq(g, o):
    return np.array_equal(g.to_numpy().astype(np.uint64), np.asarray(o.values(), np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["sht", "int", "lng", "flt", "dbl"])
@pytest.mark.parametrize("op", list(OPS))
@pytest.mark.parametrize("form", ["none", "dense", "oids"])
def test_gpu_thetajoin(gdk, ora, tname, op, form):
    r = rng(1603)
    nl, nr = 900, 700
    lv, rv = _col(r, nl, tname), _col(r, nr, tname)
    if form == "none" and op == "lt":
        rv = np.sort(rv)                 # right side already in value order: no final sort
    gl, gr, ol, orr = _mk(gdk, tname, lv), _mk(gdk, tname, rv), _mk(ora, tname, lv), _mk(ora, tname, rv)
    gsl, osl = _cands(gdk, ora, r, nl, form)
    gsr, osr = _cands(gdk, ora, r, nr, "dense" if form == "oids" else form)
    for nil_matches in (False, True):
        a, b = gdk.BATthetajoin(gl, gr, gsl, gsr, OPS[op], nil_matches)
        wa, wb = ora.BATthetajoin(ol, orr, osl, osr, OPS[op], nil_matches)
        assert _eq(a, wa) and _eq(b, wb), nil_matches


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["sht", "int", "lng", "flt", "dbl"])
def test_gpu_bandjoin(gdk, ora, tname):
    r = rng(1604)
    nl, nr = 3000, 2500
    lv, rv = _col(r, nl, tname, -5000, 5000), _col(r, nr, tname, -5000, 5000)
    gl, gr, ol, orr = _mk(gdk, tname, lv), _mk(gdk, tname, rv), _mk(ora, tname, lv), _mk(ora, tname, rv)
    cases = [(3, 5, True, True), (3, 5, False, False), (0, 0, True, True), (10, -2, True, True),
             (2, -2, True, False), (-3, 1, True, True)]
    if tname == "dbl":
        cases += [(1e308, 1e308, True, True), (-1e308, 1e308, True, True), (0.25, 0.5, False, True)]
    for c1, c2, li, hi in cases:
        for form in ("none", "oids"):
            gsl, osl = _cands(gdk, ora, r, nl, form)
            a, b = gdk.BATbandjoin(gl, gr, c1, c2, gsl, None, li, hi)
            wa, wb = ora.BATbandjoin(ol, orr, c1, c2, osl, None, li, hi)
            assert _eq(a, wa) and _eq(b, wb), (c1, c2, li, hi, form)


@pytest.mark.gpu
def test_gpu_thetajoin_large(gdk, ora):
    """a large left side against a small sorted / unsorted right side"""
    r = rng(1605)
    lv = r.integers(0, 1 << 20, 200_000).astype(np.int32)
    rv = r.integers(0, 1 << 20, 64).astype(np.int32)
    for op in ("lt", "ge", "ne"):
        a, b = gdk.BATthetajoin(_mk(gdk, "int", lv), _mk(gdk, "int", rv), None, None, OPS[op])
        wa, wb = ora.BATthetajoin(_mk(ora, "int", lv), _mk(ora, "int", rv), None, None, OPS[op])
        assert _eq(a, wa) and _eq(b, wb), op


def _model_range(lv, lo_, hi_, lc, rc, linc, hinc, anti, symmetric, right_major):
    def b3(v, a, b, ai, bi):
        if np.isnan(a) if isinstance(a, float) else a is None:
            pass
        g = None if a is None else (a < v or (ai and v == a))
        l_ = None if b is None else (v < b or (bi and v == b))
        if g is False or l_ is False:
            return 0
        if g is None or l_ is None:
            return -1
        return 1
    pairs = []
    for i in lc:
        v = lv[i]
        if v is None:
            continue
        for j in rc:
            m = b3(v, lo_[j], hi_[j], linc, hinc)
            if symmetric:
                m2 = b3(v, hi_[j], lo_[j], hinc, linc)
                m = 1 if (m == 1 or m2 == 1) else (-1 if (m < 0 or m2 < 0) else 0)
            if anti:
                m = -1 if m < 0 else int(not m)
            if m == 1:
                pairs.append((i, j))
    if right_major:
        pairs.sort(key=lambda p: (p[1], p[0]))
    return [p[0] for p in pairs], [p[1] for p in pairs]


@pytest.mark.parametrize("sorted_l", [False, True])
@pytest.mark.parametrize("flags", [(True, True, False, False), (False, True, False, False), (True, False, True, False),
                                   (True, True, False, True), (False, False, True, True)])
def test_oracle_rangejoin_model(ora, sorted_l, flags):
    linc, hinc, anti, symmetric = flags
    r = rng(1606)
    lv = _col(r, 60, "int")
    if sorted_l:
        lv = np.sort(lv)
    lo_, hi_ = _col(r, 40, "int"), _col(r, 40, "int")
    hi_ = np.where(hi_ == NILS["int"], hi_, np.maximum(hi_, lo_ + r.integers(-5, 20, 40)).astype(np.int32))
    a, b = ora.BATrangejoin(_mk(ora, "int", lv), _mk(ora, "int", lo_), _mk(ora, "int", hi_), None, None,
                            linc, hinc, anti, symmetric)
    nz = lambda x: None if x == NILS["int"] else int(x)   # noqa: E731
    w1, w2 = _model_range([nz(x) for x in lv], [nz(x) for x in lo_], [nz(x) for x in hi_], range(60), range(40),
                          linc, hinc, anti, symmetric, sorted_l and not anti and not symmetric)
    assert [int(x) for x in a.values()] == w1 and [int(x) for x in b.values()] == w2


@pytest.mark.gpu
@pytest.mark.parametrize("tname", ["int", "lng", "dbl"])
@pytest.mark.parametrize("lform", ["shuffled", "sorted", "revsorted"])
@pytest.mark.parametrize("flags", [(True, True, False, False), (False, True, False, False), (True, False, True, False),
                                   (True, True, False, True)])
def test_gpu_rangejoin(gdk, ora, tname, lform, flags):
    linc, hinc, anti, symmetric = flags
    r = rng(1607)
    nl, nr = 2500, 900
    lv = _col(r, nl, tname, -3000, 3000)
    if lform == "sorted":
        lv = np.sort(lv)
    elif lform == "revsorted":
        lv = np.sort(lv)[::-1].copy()
        if tname == "dbl":
            lv = np.concatenate([lv[~np.isnan(lv)], lv[np.isnan(lv)]])   # nils last in descending order
        else:
            lv = np.concatenate([lv[lv != NILS[tname]], lv[lv == NILS[tname]]])
    lo_ = _col(r, nr, tname, -3000, 3000)
    hi_ = (lo_ + r.integers(-50, 400, nr)).astype(lo_.dtype)
    if tname != "dbl":
        hi_[lo_ == NILS[tname]] = lo_[lo_ == NILS[tname]]
    gm = lambda v: _mk(gdk, tname, v)   # noqa: E731
    om = lambda v: _mk(ora, tname, v)   # noqa: E731
    for form in ("none", "oids"):
        gsl, osl = _cands(gdk, ora, r, nl, form)
        a, b = gdk.BATrangejoin(gm(lv), gm(lo_), gm(hi_), gsl, None, linc, hinc, anti, symmetric)
        wa, wb = ora.BATrangejoin(om(lv), om(lo_), om(hi_), osl, None, linc, hinc, anti, symmetric)
        assert _eq(a, wa) and _eq(b, wb), form
        for g, w in ((a, wa), (b, wb)):
            assert (bool(g.s.tsorted), bool(g.s.trevsorted), bool(g.s.tkey)) == \
                (bool(w.s.sorted), bool(w.s.revsorted), bool(w.s.key)), form
