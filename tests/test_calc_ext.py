"""The rest of gdk_calc.c's element-wise operators: BATcalcnegate / absolute /
iszero / sign / isnil / isnotnil (gdk/gdk_calc.c:233-920), min / max and
their _no_nil and constant forms (:976-2436), and / or / xor (:2439-3030;
bit columns three-valued, or3 / and3 :2590 / :2826), lsh / rsh (:3059-3760)
and ifthenelse (:4376-4760) -- the CASE / COALESCE / LEAST / GREATEST and
bitwise operators of SQL plans (batcalc.*).

The oracle (oracle/gdk_oracle_calc.c) restates them; it is checked here
against numpy / Python models of the same rules (nil propagation, the tie
rule of each min / max form: p1 < p2 ? p1 : p2 keeps p2 on a tie, the
_no_nil form keeps p1, which matters for -0.0 / +0.0; the overflow of an
integer AND / XOR whose result is the nil bit pattern; the shift checks),
and the device against the oracle with candidate lists.  No reference
fixture covers them (parity unpinned beyond the models)."""
import math

import numpy as np
import pytest

from helpers import rng

NI = -(1 << 31)
ONIL = 1 << 63


def _cols():
    r = rng(1601)
    a = r.integers(-50, 50, 3000).astype(np.int32)
    b = r.integers(-50, 50, 3000).astype(np.int32)
    a[::37] = NI
    b[::41] = NI
    f = (r.integers(-40, 40, 3000) / 8).astype(np.float64)
    g = (r.integers(-40, 40, 3000) / 8).astype(np.float64)
    f[::29] = np.nan
    g[::31] = np.nan
    f[7], g[7] = -0.0, 0.0
    f[8], g[8] = 0.0, -0.0
    return a, b, f, g


def _cand(r, n):
    return np.sort(r.choice(n, n // 2, replace=False)).astype(np.uint64)


def _nil_of(dt):
    return np.nan if dt.kind == "f" else np.iinfo(dt).min


def _isnil(x):
    return np.isnan(x) if x.dtype.kind == "f" else x == np.iinfo(x.dtype).min


def _same(got, want):
    """bit-exact, every NaN counting as the same nil"""
    got, want = np.asarray(got), np.asarray(want)
    if got.dtype.kind == "f":
        want = want.astype(got.dtype)
        nan = np.isnan(got)
        return np.array_equal(nan, np.isnan(want)) and \
            np.array_equal(got[~nan].view(np.uint8), want[~nan].view(np.uint8))
    return np.array_equal(got.astype(np.int64), want.astype(np.int64))


def _ora(ora, x):
    tp = {np.dtype(np.int32): ora.TYPE_int, np.dtype(np.float64): ora.TYPE_dbl, np.dtype(np.int8): ora.TYPE_bit,
          np.dtype(np.int64): ora.TYPE_lng}[x.dtype]
    return ora.Bat.from_array(tp, x)


@pytest.mark.parametrize("name", ["negate", "absolute", "iszero", "sign", "isnil", "isnotnil"])
def test_oracle_unary_model(ora, name):
    a, _, f, _ = _cols()
    for x in (a, f):
        got = ora.BATcalcunary(name, _ora(ora, x)).values()
        nil = _isnil(x)
        xv = np.where(nil, 0, x)
        if name == "negate":
            w = np.where(nil, _nil_of(x.dtype), -xv)
        elif name == "absolute":
            w = np.where(nil, _nil_of(x.dtype), np.abs(xv))
        elif name == "iszero":
            w = np.where(nil, -128, xv == 0)
        elif name == "sign":
            w = np.where(nil, -128, np.sign(xv))
        elif name == "isnil":
            w = nil
        else:
            w = ~nil
        assert _same(np.asarray(got), w.astype(np.asarray(got).dtype) if name in ("negate", "absolute") else w), \
            (name, x.dtype)


def _minmax_model(name, p, q):
    pn, qn = _isnil(p), _isnil(q)
    out = []
    for x, y, xn, yn in zip(p, q, pn, qn):
        if name in ("min", "max"):
            if xn or yn:
                out.append(_nil_of(p.dtype))
            else:
                out.append(x if (x < y if name == "min" else x > y) else y)
        else:
            if xn:
                out.append(y)
            else:
                out.append(y if (not yn and (y < x if name == "min_no_nil" else y > x)) else x)
    return np.array(out, dtype=p.dtype)


@pytest.mark.parametrize("name", ["min", "max", "min_no_nil", "max_no_nil"])
def test_oracle_minmax_model(ora, name):
    a, b, f, g = _cols()
    for p, q in ((a, b), (f, g)):
        got = np.asarray(ora.BATcalcminmax(name, _ora(ora, p), _ora(ora, q)).values())
        w = _minmax_model(name, p, q)
        assert _same(got, w), (name, p.dtype)
        # the constant forms: p1 OP c ? p1 : c (ties keep the constant)
        c = p.dtype.type(-0.0 if p.dtype.kind == "f" else 7)
        tp = ora.TYPE_dbl if p.dtype.kind == "f" else ora.TYPE_int
        got = np.asarray(ora.BATcalcminmax(name, _ora(ora, p), None, c=c, ct=tp).values())
        pn = _isnil(p)
        if name in ("min", "max"):
            w = np.array([_nil_of(p.dtype) if n else (x if (x < c if name == "min" else x > c) else c)
                          for x, n in zip(p, pn)], p.dtype)
        else:
            w = np.array([c if n else (x if (x < c if name == "min_no_nil" else x > c) else c)
                          for x, n in zip(p, pn)], p.dtype)
        assert _same(got, w), (name, "cst", p.dtype)


def test_oracle_bits_model(ora):
    r = rng(1602)
    b1 = r.integers(-1, 2, 500).astype(np.int8)      # bit: 0, 1, nil (-1 -> nil)
    b2 = r.integers(-1, 2, 500).astype(np.int8)
    b1[b1 == -1] = -128
    b2[b2 == -1] = -128
    B1, B2 = ora.Bat.from_array(ora.TYPE_bit, b1), ora.Bat.from_array(ora.TYPE_bit, b2)

    def or3(x, y):
        return 1 if x == 1 or y == 1 else (-128 if x == -128 or y == -128 else 0)

    def and3(x, y):
        return 0 if x == 0 or y == 0 else (-128 if x == -128 or y == -128 else 1)
    assert list(ora.BATcalcbits("or", "BATcalcor", B1, B2).values()) == [or3(x, y) for x, y in zip(b1, b2)]
    assert list(ora.BATcalcbits("and", "BATcalcand", B1, B2).values()) == [and3(x, y) for x, y in zip(b1, b2)]
    assert list(ora.BATcalcbits("xor", "BATcalcxor", B1, B2).values()) == \
        [-128 if -128 in (x, y) else int((x == 0) != (y == 0)) for x, y in zip(b1, b2)]
    a, b, _, _ = _cols()
    A, Bb = _ora(ora, a), _ora(ora, b)
    for nm, op in (("and", np.bitwise_and), ("or", np.bitwise_or), ("xor", np.bitwise_xor)):
        got = np.asarray(ora.BATcalcbits(nm, "BATcalc" + nm, A, Bb).values())
        w = np.where(_isnil(a) | _isnil(b), NI, op(a, b))
        assert np.array_equal(got, w), nm
    with pytest.raises(Exception, match="overflow in calculation 2147483647XOR-1"):
        ora.BATcalcbits("xor", "BATcalcxor", ora.Bat.from_array(ora.TYPE_int, np.array([1, 2147483647], np.int32)),
                        ora.Bat.from_array(ora.TYPE_int, np.array([1, -1], np.int32)))
    s = np.array([0, 3, 30, 5], np.int32)
    v = np.array([1, -8, 1, 1000], np.int32)
    assert list(ora.BATcalcbits("rsh", "BATcalcrsh", _ora(ora, v), _ora(ora, s)).values()) == [1, -1, 0, 31]
    with pytest.raises(Exception, match="shift operand too large in LSH"):
        ora.BATcalcbits("lsh", "BATcalclsh", _ora(ora, v), _ora(ora, s))
    assert list(ora.BATcalcbits("lsh", "BATcalclsh", _ora(ora, np.array([1, 3], np.int32)),
                                _ora(ora, np.array([30, 4], np.int32))).values()) == [1 << 30, 48]


def test_oracle_ifthenelse_model(ora):
    r = rng(1603)
    n = 400
    c = r.integers(-1, 2, n).astype(np.int8)
    c[c == -1] = -128
    x = r.integers(0, 100, n).astype(np.int32)
    y = r.integers(0, 100, n).astype(np.int32)
    C = ora.Bat.from_array(ora.TYPE_bit, c)
    take = (c != 0) & (c != -128)
    assert np.array_equal(np.asarray(ora.BATcalcifthenelse(C, _ora(ora, x), _ora(ora, y)).values()),
                          np.where(take, x, y))
    assert np.array_equal(np.asarray(ora.BATcalcifthenelse(C, _ora(ora, x), None, c2=-5, ct=ora.TYPE_int).values()),
                          np.where(take, x, -5))
    got = ora.BATcalcifthenelse(C, ora.Bat.dense(10, n), ora.Bat.dense(1000, n)).values()
    assert [int(v) for v in got] == [10 + i if t else 1000 + i for i, t in enumerate(take)]


# ---- device ---------------------------------------------------------------


def _gdk(gdk, x):
    tp = {np.dtype(np.int32): gdk.TYPE_int, np.dtype(np.float64): gdk.TYPE_dbl, np.dtype(np.int8): gdk.TYPE_bit,
          np.dtype(np.int64): gdk.TYPE_lng}[x.dtype]
    return gdk.BAT.from_numpy(tp, x, sorted_=False, revsorted=False, key=False, nonil=False)


def _eqbat(g, o):
    gv, ov = g.to_numpy(), np.asarray(o.values())
    if gv.dtype.kind == "f":
        return np.array_equal(gv.view(np.uint8), ov.astype(gv.dtype).view(np.uint8))
    return np.array_equal(gv.astype(np.int64), ov.astype(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["negate", "absolute", "iszero", "sign", "isnil", "isnotnil"])
@pytest.mark.parametrize("cands", [False, True])
def test_gpu_unary(gdk, ora, name, cands):
    a, _, f, _ = _cols()
    r = rng(1604)
    for x in (a, f, a.astype(np.int64)):
        s = _cand(r, len(x)) if cands else None
        gs = gdk.BAT.from_numpy(gdk.TYPE_oid, s, sorted_=True, key=True, nonil=True) if cands else None
        os_ = ora.Bat.from_array(ora.TYPE_oid, s, sorted_=True, key=True, nonil=True) if cands else None
        g = gdk.BATcalcunary(name, _gdk(gdk, x), gs)
        o = ora.BATcalcunary(name, _ora(ora, x), os_)
        assert _eqbat(g, o), (name, x.dtype)
        assert bool(g.s.tnil) == bool(o.s.nil) and bool(g.s.tsorted) == bool(o.s.sorted)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["min", "max", "min_no_nil", "max_no_nil"])
def test_gpu_minmax(gdk, ora, name):
    a, b, f, g = _cols()
    r = rng(1605)
    for p, q in ((a, b), (f, g)):
        assert _eqbat(gdk.BATcalcbin(name, _gdk(gdk, p), _gdk(gdk, q)),
                      ora.BATcalcminmax(name, _ora(ora, p), _ora(ora, q)))
        s = _cand(r, len(p))
        gs = gdk.BAT.from_numpy(gdk.TYPE_oid, s, sorted_=True, key=True, nonil=True)
        os_ = ora.Bat.from_array(ora.TYPE_oid, s, sorted_=True, key=True, nonil=True)
        assert _eqbat(gdk.BATcalcbin(name, _gdk(gdk, p), _gdk(gdk, q), gs, gs),
                      ora.BATcalcminmax(name, _ora(ora, p), _ora(ora, q), os_, os_))
        tg = gdk.TYPE_dbl if p.dtype.kind == "f" else gdk.TYPE_int
        to = ora.TYPE_dbl if p.dtype.kind == "f" else ora.TYPE_int
        for c in ((-0.0, 1.5, float("nan")) if p.dtype.kind == "f" else (7, -3, NI)):
            for first in (False, True):
                got = gdk.BATcalcbincst(name, _gdk(gdk, p), c, tg, gs, cst_first=first)
                want = ora.BATcalcminmax(name, _ora(ora, p), None, os_, None, c=c, ct=to)
                assert _eqbat(got, want), (name, c, first)
    # oid / void columns
    v1 = gdk.BAT.dense(100, 500)
    v2 = gdk.BAT.from_numpy(gdk.TYPE_oid, rng(3).integers(0, 1000, 500).astype(np.uint64))
    o2 = ora.Bat.from_array(ora.TYPE_oid, v2.to_numpy())
    assert _eqbat(gdk.BATcalcbin(name, v1, v2), ora.BATcalcminmax(name, ora.Bat.dense(100, 500), o2))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["and", "or", "xor"])
def test_gpu_bits(gdk, ora, name):
    r = rng(1606)
    b1 = r.integers(-1, 2, 5000).astype(np.int8)
    b2 = r.integers(-1, 2, 5000).astype(np.int8)
    b1[b1 == -1] = -128
    b2[b2 == -1] = -128
    for x, y in ((b1, b2), _cols()[:2]):
        tg = gdk.TYPE_bit if x.dtype == np.int8 else gdk.TYPE_int
        to = ora.TYPE_bit if x.dtype == np.int8 else ora.TYPE_int
        G1 = gdk.BAT.from_numpy(tg, x, sorted_=False, revsorted=False, key=False, nonil=False)
        G2 = gdk.BAT.from_numpy(tg, y, sorted_=False, revsorted=False, key=False, nonil=False)
        O1, O2 = ora.Bat.from_array(to, x), ora.Bat.from_array(to, y)
        assert _eqbat(gdk.BATcalcbin(name, G1, G2), ora.BATcalcbits(name, "BATcalc" + name, O1, O2))
        c = 1 if tg == gdk.TYPE_bit else 6
        assert _eqbat(gdk.BATcalcbincst(name, G1, c, tg),
                      ora.BATcalcbits(name, "BATcalc" + name + "cst", O1, None, c2=c, t2=to))
    with pytest.raises(gdk.GDKError, match="overflow in calculation 2147483647XOR-1"):
        gdk.BATcalcbin("xor", gdk.BAT.from_numpy(gdk.TYPE_int, np.array([1, 2147483647], np.int32)),
                       gdk.BAT.from_numpy(gdk.TYPE_int, np.array([1, -1], np.int32)))


@pytest.mark.gpu
def test_gpu_shifts(gdk, ora):
    r = rng(1607)
    v = r.integers(0, 1 << 20, 4000).astype(np.int32)
    s = r.integers(0, 11, 4000).astype(np.int32)
    v[::53] = NI
    for nm in ("lsh", "rsh"):
        assert _eqbat(gdk.BATcalcbin(nm, _gdk(gdk, v), _gdk(gdk, s)),
                      ora.BATcalcbits(nm, "BATcalc" + nm, _ora(ora, v), _ora(ora, s)))
        assert _eqbat(gdk.BATcalcbincst(nm, _gdk(gdk, v), 3, gdk.TYPE_int),
                      ora.BATcalcbits(nm, "BATcalc" + nm + "cst", _ora(ora, v), None, c2=3, t2=ora.TYPE_int))
    bad = np.array([1, 3, 5], np.int32)
    with pytest.raises(gdk.GDKError, match=r"BATcalclsh: shift operand too large in LSH\(3,40\)"):
        gdk.BATcalcbin("lsh", _gdk(gdk, bad), _gdk(gdk, np.array([2, 40, 1], np.int32)))
    with pytest.raises(gdk.GDKError, match="shift operand too large in RSH"):
        gdk.BATcalcbin("rsh", _gdk(gdk, bad), _gdk(gdk, np.array([2, -1, 1], np.int32)))


@pytest.mark.gpu
def test_gpu_ifthenelse(gdk, ora):
    r = rng(1608)
    n = 100_000
    c = r.integers(-1, 2, n).astype(np.int8)
    c[c == -1] = -128
    x = r.integers(-1000, 1000, n).astype(np.int64)
    y = r.integers(-1000, 1000, n).astype(np.int64)
    C = gdk.BAT.from_numpy(gdk.TYPE_bit, c)
    OC = ora.Bat.from_array(ora.TYPE_bit, c)
    gx, gy = _gdk(gdk, x), _gdk(gdk, y)
    ox, oy = _ora(ora, x), _ora(ora, y)
    assert _eqbat(gdk.BATcalcifthenelse(C, gx, gy), ora.BATcalcifthenelse(OC, ox, oy))
    assert _eqbat(gdk.BATcalcifthenelse(C, gx, 42, gdk.TYPE_lng),
                  ora.BATcalcifthenelse(OC, ox, None, c2=42, ct=ora.TYPE_lng))
    assert _eqbat(gdk.BATcalcifthenelse(C, -1, gy, gdk.TYPE_lng),
                  ora.BATcalcifthenelse(OC, None, oy, c1=-1, ct=ora.TYPE_lng))
    assert _eqbat(gdk.BATcalcifthenelse(C, 5, 6, gdk.TYPE_lng),
                  ora.BATcalcifthenelse(OC, None, None, c1=5, c2=6, ct=ora.TYPE_lng))
    f = (r.integers(-9, 9, n) / 4).astype(np.float64)
    f[::7] = np.nan
    assert _eqbat(gdk.BATcalcifthenelse(C, _gdk(gdk, f), -0.0, gdk.TYPE_dbl),
                  ora.BATcalcifthenelse(OC, _ora(ora, f), None, c2=-0.0, ct=ora.TYPE_dbl))
    assert _eqbat(gdk.BATcalcifthenelse(C, gdk.BAT.dense(10, n), gdk.BAT.dense(7, n)),
                  ora.BATcalcifthenelse(OC, ora.Bat.dense(10, n), ora.Bat.dense(7, n)))


# ---- ifthenelse on str (gdk_calc.c:4407-4459) ------------------------------


def _strings(gdk, b):
    """the strings of a device str BAT (its offsets and heap read back)"""
    import ctypes as C
    s = b.ptr.contents
    heap = (C.c_uint8 * max(1, s.tvheapsize))()
    assert gdk.lib().mgdk_BATdownload_vheap(b.ptr, C.cast(heap, C.c_void_p)) == 0
    hb = bytes(heap)
    offs = b.to_numpy().astype(np.uint64)
    w = s.twidth
    out = []
    for o in offs:
        o = int(o) + (8192 if w < 4 else 0)
        out.append(hb[o:hb.index(b"\0", o)])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("forms", ["bat_bat", "bat_cst", "cst_bat", "cst_cst", "same_heap"])
def test_gpu_ifthenelse_str(gdk, forms):
    from strheap import NIL, WORDS, sample, content_groups
    r = rng(1609)
    n = 20_000
    c = r.integers(-1, 2, n).astype(np.int8)
    c[c == -1] = -128
    C_ = gdk.BAT.from_numpy(gdk.TYPE_bit, c)
    t1, h1, w1 = sample(r, n, 2)
    t2, h2, w2 = sample(r, n, 8, words=WORDS[::-1])
    if forms == "same_heap":
        t2, h2, w2 = sample(r, n, 4)
        h2 = h1
        w2 = [WORDS[i] for i in w2]
        t2 = None
    words1 = [WORDS[i] for i in w1]
    words2 = [WORDS[::-1][i] for i in w2] if forms != "same_heap" else w2
    B1 = gdk.BAT.from_numpy(gdk.TYPE_str, t1, vheap=h1, sorted_=False, revsorted=False, key=False, nonil=False)
    if forms == "same_heap":
        # the else side: other rows of the then side's column (a projection shares its heap)
        perm = r.permutation(n).astype(np.uint64)
        B2 = gdk.BATproject(gdk.BAT.from_numpy(gdk.TYPE_oid, perm), B1)
        words2 = [words1[i] for i in perm]
    else:
        B2 = gdk.BAT.from_numpy(gdk.TYPE_str, t2, vheap=h2, sorted_=False, revsorted=False, key=False, nonil=False)
    take = (c != 0) & (c != -128)
    if forms in ("bat_bat", "same_heap"):
        got = gdk.BATcalcifthenelse(C_, B1, B2)
        want = [a if t else b for a, b, t in zip(words1, words2, take)]
    elif forms == "bat_cst":
        got = gdk.BATcalcifthenelse(C_, B1, b"other", gdk.TYPE_str)
        want = [a if t else b"other" for a, t in zip(words1, take)]
    elif forms == "cst_bat":
        got = gdk.BATcalcifthenelse(C_, NIL, B2, gdk.TYPE_str)
        want = [NIL if t else b for b, t in zip(words2, take)]
    else:
        got = gdk.BATcalcifthenelse(C_, b"yes", b"no", gdk.TYPE_str)
        want = [b"yes" if t else b"no" for t in take]
    assert _strings(gdk, got) == want
    if forms == "same_heap":
        assert got.ptr.contents.tvheap == B1.ptr.contents.tvheap      # shared, not copied
    # grouping the result compares strings (a copied heap may repeat one)
    g, e, h = gdk.BATgroup(got)
    wg, we, wh = content_groups(want)
    assert np.array_equal(g.to_numpy().astype(np.uint64), wg) and np.array_equal(e.to_numpy().astype(np.uint64), we)


# ---- every value type through the device kernels ---------------------------


def _typed(r, tn, n):
    if tn in ("flt", "dbl"):
        v = (r.integers(-60, 60, n) / 4).astype(np.float32 if tn == "flt" else np.float64)
        v[::23] = np.nan
        v[5] = -0.0
        return v
    if tn == "hge":
        lo = r.integers(-1000, 1000, n, dtype=np.int64)
        lo[::23] = 0
        a = np.stack([lo.view(np.uint64), (lo >> 63).view(np.uint64)], axis=1)
        a[::23] = [0, 1 << 63]      # hge nil
        return a
    dt = {"bte": np.int8, "sht": np.int16, "int": np.int32, "lng": np.int64}[tn]
    v = r.integers(-100, 100, n).astype(dt)
    v[::23] = np.iinfo(dt).min
    return v


def _eq_any(g, o, tn):
    if tn == "hge":
        return list(g.values()) == [int(x) for x in o.values()] if g.ttype == 11 else \
            np.array_equal(g.to_numpy().astype(np.int64), np.asarray(o.values()).astype(np.int64))
    return _eqbat(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("tn", ["bte", "sht", "int", "lng", "hge", "flt", "dbl"])
def test_gpu_calc_ext_types(gdk, ora, tn):
    r = rng(1610)
    n = 3000
    a, b = _typed(r, tn, n), _typed(r, tn, n)
    tg, to = getattr(gdk, "TYPE_" + tn), getattr(ora, "TYPE_" + tn)
    G = lambda x: gdk.BAT.from_numpy(tg, x, sorted_=False, revsorted=False, key=False, nonil=False)   # noqa: E731
    O = lambda x: ora.Bat.from_array(to, x)   # noqa: E731
    for name in ("negate", "absolute", "iszero", "sign", "isnil", "isnotnil"):
        assert _eq_any(gdk.BATcalcunary(name, G(a)), ora.BATcalcunary(name, O(a)), tn), name
    for name in ("min", "max", "min_no_nil", "max_no_nil"):
        assert _eq_any(gdk.BATcalcbin(name, G(a), G(b)), ora.BATcalcminmax(name, O(a), O(b)), tn), name
    if tn in ("flt", "dbl"):
        return
    def same_outcome(dev, orf, name):
        # a result with the nil pattern (and / or / xor) or that does not fit
        # (lsh) is the reference's error: both sides raise the same message,
        # or neither raises and the columns agree
        try:
            want = orf()
        except Exception as e:   # noqa: BLE001
            with pytest.raises(gdk.GDKError) as ei:
                dev()
            assert str(ei.value).strip() == str(e).strip(), name
            return
        assert _eq_any(dev(), want, tn), name
    for name in ("and", "or", "xor"):
        same_outcome(lambda: gdk.BATcalcbin(name, G(a), G(b)),
                     lambda: ora.BATcalcbits(name, "BATcalc" + name, O(a), O(b)), name)
    sh = np.abs(_typed(r, "bte", n).astype(np.int32)) % 5
    sh[::23] = 1
    S = gdk.BAT.from_numpy(gdk.TYPE_int, sh.astype(np.int32))
    OS = ora.Bat.from_array(ora.TYPE_int, sh.astype(np.int32))
    pos = a.copy()
    if tn == "hge":
        pos[:, 1] = 0
        pos[:, 0] = pos[:, 0] % 1000
    else:
        pos = np.where(pos == np.iinfo(pos.dtype).min, pos, np.abs(pos) % 16).astype(a.dtype)
    for name in ("lsh", "rsh"):
        same_outcome(lambda: gdk.BATcalcbin(name, G(pos), S),
                     lambda: ora.BATcalcbits(name, "BATcalc" + name, O(pos), OS), name)
    small = pos.copy()
    if tn != "hge":
        small = np.where(small == np.iinfo(small.dtype).min, small, small % 4).astype(a.dtype)
        sh1 = (sh % 3).astype(np.int32)
        assert _eq_any(gdk.BATcalcbin("lsh", G(small), gdk.BAT.from_numpy(gdk.TYPE_int, sh1)),
                       ora.BATcalcbits("lsh", "BATcalclsh", O(small), ora.Bat.from_array(ora.TYPE_int, sh1)), tn)
