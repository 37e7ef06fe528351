"""BATcalc comparisons, between, BATconvert, NOT, division and modulo: the
oracle against the reference's batcalc MAL tests (tst901 / tst906 / tst908,
expected as the sqllogictest md5 of the printed rows), and the device against
the oracle on random inputs (values and result properties)."""
import hashlib
import json
import os

import numpy as np
import pytest

from helpers import rng

HERE = os.path.dirname(os.path.abspath(__file__))
FX = json.load(open(os.path.join(HERE, "golden", "maltest_fixtures.json")))["batcalc"]


def _md5_rowsort(prints):
    """io.print of each BAT = (oid, value) rows; `query II rowsort` sorts the
    rows as strings and hashes value + '\\n' (testing/sqllogictest.py:492-620);
    bit values print as true / false and are converted to 1 / 0."""
    rows = []
    for vals in prints:
        for i, v in enumerate(vals):
            rows.append((str(i), str(int(v))))
    m = hashlib.md5()
    for r in sorted(rows):
        for c in r:
            m.update(c.encode() + b"\n")
    return len(rows) * 2, m.hexdigest()


def replay_batcalc(name, mk, calc, calccst, divcst, eq, notf, vals):
    """Replay the MAL function of tst901 / tst906 over 0..9: every io.print
    in order, then the md5 of the rows."""
    fx = FX[name]
    b = mk(np.arange(10))
    env = {"b": b, "c": mk(np.arange(10))}
    prints = [vals(env["c"])]
    for dst, op, a1, a2 in fx["ops"]:
        if op in "+*" and a2 in env:
            env[dst] = calc(op, env[a1], env[a2])
        elif op == "+":
            env[dst] = calccst(op, env[a1], int(a2.split(":")[0]))
        elif op == "/":
            env[dst] = divcst(env[a1], int(a2.split(":")[0]))
        elif op == "==":
            env[dst] = eq(env[a1], env[a2])
        else:
            env[dst] = notf(env[a1])
        prints.append(vals(env[dst]))
    return _md5_rowsort(prints)


def test_batcalc_maltest_oracle(ora):
    for name, tp in (("tst901", ora.TYPE_int), ("tst906", ora.TYPE_lng)):
        mk = lambda a, tp=tp: ora.Bat.from_array(tp, a, sorted_=True, key=True, nonil=True)
        got = replay_batcalc(
            name, mk,
            lambda op, x, y, tp=tp: ora.BATcalc(op, x, y, tp),
            lambda op, x, c, tp=tp: ora.BATcalc(op, x, None, tp, c2=c, t2=tp),
            lambda x, c, tp=tp: ora.BATcalcdivmod("/", x, None, tp, c2=c, t2=tp),
            lambda x, y: ora.BATcalccmp("==", x, y),
            lambda x: ora.BATcalcnot(x),
            lambda x: x.values())
        assert got == (FX[name]["nvalues"], FX[name]["md5"]), name
    b = ora.Bat.from_array(ora.TYPE_lng, np.arange(10), sorted_=True, key=True, nonil=True)
    r = ora.BATcalcdivmod("/", b, None, ora.TYPE_lng, c2=1, t2=ora.TYPE_lng)
    assert [[i, int(v)] for i, v in enumerate(r.values())] == FX["tst908"]["expected"]


@pytest.mark.gpu
def test_batcalc_maltest_device(gdk):
    for name, tp in (("tst901", gdk.TYPE_int), ("tst906", gdk.TYPE_lng)):
        mk = lambda a, tp=tp: gdk.BAT.from_numpy(tp, a)
        got = replay_batcalc(
            name, mk,
            lambda op, x, y, tp=tp: (gdk.BATcalcadd if op == "+" else gdk.BATcalcmul)(x, y, tp),
            lambda op, x, c, tp=tp: gdk.BATcalcaddcst(x, c, tp, tp),
            lambda x, c, tp=tp: gdk.BATcalcdivmod("/", x, None, tp, c2=c, t2=tp),
            lambda x, y: gdk.BATcalccmp("==", x, y),
            lambda x: gdk.BATcalcnot(x),
            lambda x: x.values())
        assert got == (FX[name]["nvalues"], FX[name]["md5"]), name
    b = gdk.BAT.from_numpy(gdk.TYPE_lng, np.arange(10))
    r = gdk.BATcalcdivmod("/", b, None, gdk.TYPE_lng, c2=1, t2=gdk.TYPE_lng)
    assert [[i, int(v)] for i, v in enumerate(r.values())] == FX["tst908"]["expected"]


def test_oracle_calccmp_semantics(ora):
    """C's conversions: int vs flt compares in flt (2^24 + 1 == 2^24f);
    nil_matches; cmp's -1/0/1; a nil-free input compares NaN raw."""
    a = ora.Bat.from_array(ora.TYPE_int, np.array([16777217, 5, -(1 << 31)], np.int32))
    f = ora.Bat.from_array(ora.TYPE_flt, np.array([16777216.0, 5.5, 1.0], np.float32))
    assert list(ora.BATcalccmp("==", a, f).values()) == [1, 0, -128]
    assert list(ora.BATcalccmp("cmp", a, f).values()) == [0, -1, -128]
    assert list(ora.BATcalccmp("==", a, f, nil_matches=True).values()) == [1, 0, 0]
    d = ora.Bat.from_array(ora.TYPE_dbl, np.array([np.nan, 1.0]), nonil=True)
    assert list(ora.BATcalccmp("!=", d, None, c2=1.0, t2=ora.TYPE_dbl).values()) == [1, 0]


def test_oracle_convert_semantics(ora):
    dbl = ora.Bat.from_array(ora.TYPE_dbl, np.array([1.005, -2.5, 3.49999]))
    assert list(ora.BATconvert(dbl, None, ora.TYPE_lng, 0, 2, 0).values()) == [100, -250, 350]
    lng = ora.Bat.from_array(ora.TYPE_lng, np.array([1005, -2550, 349999]))
    assert list(ora.BATconvert(lng, None, ora.TYPE_int, 3, 1, 0).values()) == [10, -26, 3500]
    with pytest.raises(ora.OracleError, match=r"22003!overflow in conversion of 300000 to sht\."):
        ora.BATconvert(ora.Bat.from_array(ora.TYPE_lng, np.array([1005, 300000])), None, ora.TYPE_sht)
    with pytest.raises(ora.OracleError, match=r"22003!overflow in conversion to DECIMAL\(7,2\)\."):
        ora.BATconvert(ora.Bat.from_array(ora.TYPE_lng, np.array([1005, 300000])), None, ora.TYPE_int, 0, 2, 7)


# ---- device against the oracle ------------------------------------------------

NUM = ["bte", "sht", "int", "lng", "hge", "flt", "dbl"]


def values_of(tp, n, r, nilfrac=0.1):
    """random values of a type that make the conversions matter (ints near
    2^24 / 2^53, floats equal to integers, halves) with nils"""
    if tp in ("flt", "dbl"):
        a = np.concatenate([r.integers(-50, 50, n // 2).astype(np.float64),
                            r.integers(-400, 400, n - n // 2) / 4.0])
        if tp == "dbl":
            a[::7] = 2.0 ** 53 + r.integers(-3, 4, a[::7].size)
        else:
            a[::7] = 2.0 ** 24 + r.integers(-3, 4, a[::7].size)
        a = a.astype(np.float32 if tp == "flt" else np.float64)
        a[r.random(n) < nilfrac] = np.nan
        return a
    lim = {"bte": 127, "sht": 32767, "int": 2 ** 31 - 1, "lng": 2 ** 63 - 1, "hge": 2 ** 63 - 1}[tp]
    a = r.integers(-min(lim, 60), min(lim, 60) + 1, n).astype(object)
    if tp in ("int", "lng", "hge"):
        big = 2 ** 24 if tp == "int" else 2 ** 53
        a[::5] = [big + int(x) for x in r.integers(-3, 4, a[::5].size)]
    if tp == "hge":
        a[::11] = [int(x) * 2 ** 70 for x in r.integers(-5, 6, a[::11].size)]
    nil = -(1 << ({"bte": 7, "sht": 15, "int": 31, "lng": 63, "hge": 127}[tp]))
    a[r.random(n) < nilfrac] = nil
    if tp == "hge":
        return np.array([[v & (2 ** 64 - 1), (v >> 64) & (2 ** 64 - 1)] for v in (int(x) for x in a)], np.uint64)
    return np.array(a, dtype={"bte": np.int8, "sht": np.int16, "int": np.int32, "lng": np.int64}[tp])


def scalar_of(tp, arr, i):
    if tp == "hge":
        lo, hi = int(arr[i][0]), int(arr[i][1])
        v = (hi << 64) | lo
        return v - (1 << 128) if v >= 1 << 127 else v
    return arr[i].item()


def mkpair(gdk, ora, tp, a, hseq=0, nonil=False):
    d = gdk.BAT.from_numpy(getattr(gdk, "TYPE_" + tp), a, hseqbase=hseq, sorted_=False, revsorted=False,
                           key=False, nonil=nonil)
    o = ora.Bat.from_array(getattr(ora, "TYPE_" + tp), a, hseqbase=hseq, nonil=nonil)
    o.s.nil = d.s.tnil
    return d, o


def same(d, o, what):
    dv, ov = np.asarray(d.values()), np.asarray(o.values())
    if dv.dtype.kind == "f":
        assert np.array_equal(dv, ov, equal_nan=True), what
    else:
        assert np.array_equal(dv, ov), what
    ds, os_ = d.s, o.s
    assert (ds.ttype, ds.count, ds.hseqbase) == (os_.type, os_.count, os_.hseqbase), what
    assert (bool(ds.tsorted), bool(ds.trevsorted), bool(ds.tkey), bool(ds.tnonil), bool(ds.tnil)) == \
        (bool(os_.sorted), bool(os_.revsorted), bool(os_.key), bool(os_.nonil), bool(os_.nil)), what


def both_or_error(fd, fo, what):
    """run device and oracle; both fail with the same message or agree"""
    try:
        o = fo()
    except Exception as e:  # oracle error: the device must fail the same way
        with pytest.raises(Exception) as ei:
            fd()
        assert str(ei.value).strip() == str(e).strip(), what
        return
    same(fd(), o, what)


@pytest.mark.gpu
@pytest.mark.parametrize("t1,t2", [("bte", "bte"), ("int", "int"), ("int", "flt"), ("lng", "dbl"), ("lng", "flt"),
                                   ("hge", "lng"), ("hge", "dbl"), ("flt", "dbl"), ("sht", "hge"), ("dbl", "dbl"),
                                   ("bte", "lng"), ("flt", "flt")])
def test_calccmp_parity(gdk, ora, t1, t2):
    r = rng(hash((t1, t2)) & 0xffff)
    n = 3001
    a, b = values_of(t1, n, r), values_of(t2, n, r)
    # equal values in both columns for a third of the rows (as the other type)
    da, oa = mkpair(gdk, ora, t1, a, hseq=5)
    db, ob = mkpair(gdk, ora, t2, b, hseq=5)
    cand = np.sort(r.choice(np.arange(5, 5 + n), 1200, replace=False)).astype(np.uint64)
    dc = gdk.BAT.from_numpy(gdk.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    oc = ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    T1, T2 = getattr(gdk, "TYPE_" + t1), getattr(gdk, "TYPE_" + t2)
    c2 = scalar_of(t2, b, 3)
    for op in ("<", "<=", ">", ">=", "==", "!=", "cmp"):
        for nm in ((False, True) if op in ("==", "!=") else (False,)):
            w = f"{t1} {op} {t2} nm={nm}"
            same(gdk.BATcalccmp(op, da, db, nil_matches=nm), ora.BATcalccmp(op, oa, ob, nil_matches=nm), w)
            same(gdk.BATcalccmp(op, da, db, s1=dc, s2=dc, nil_matches=nm),
                 ora.BATcalccmp(op, oa, ob, s1=oc, s2=oc, nil_matches=nm), w + " cand")
            same(gdk.BATcalccmp(op, da, None, c2=c2, t2=T2, nil_matches=nm),
                 ora.BATcalccmp(op, oa, None, c2=c2, t2=T2, nil_matches=nm), w + " cst")
            same(gdk.BATcalccmp(op, None, db, s1=dc, c1=scalar_of(t1, a, 4), t1=T1, nil_matches=nm),
                 ora.BATcalccmp(op, None, ob, s1=oc, c1=scalar_of(t1, a, 4), t1=T1, nil_matches=nm), w + " cstbat")


@pytest.mark.gpu
def test_calccmp_nonil_and_oid(gdk, ora):
    """nil-free inputs compare raw (NaN != x is true); oid / void operands;
    the two-void constant shortcut; unsupported types"""
    x = np.array([np.nan, 1.0, 2.0, np.nan])
    d, o = mkpair(gdk, ora, "dbl", x, nonil=True)
    for op in ("<", "==", "!=", "cmp"):
        same(gdk.BATcalccmp(op, d, None, c2=1.0, t2=gdk.TYPE_dbl), ora.BATcalccmp(op, o, None, c2=1.0, t2=ora.TYPE_dbl),
             "nonil " + op)
    oids = np.array([3, 7, 1 << 63, 9, 4], np.uint64)
    dd, oo = mkpair(gdk, ora, "oid", oids)
    dv, ov = gdk.BAT.dense(5, 5), ora.Bat.dense(5, 5)
    for op in ("<", ">=", "==", "!="):
        for nm in (False, True):
            same(gdk.BATcalccmp(op, dd, dv, nil_matches=nm), ora.BATcalccmp(op, oo, ov, nil_matches=nm), "oid-void " + op)
            same(gdk.BATcalccmp(op, dv, dd, nil_matches=nm), ora.BATcalccmp(op, ov, oo, nil_matches=nm), "void-oid " + op)
            same(gdk.BATcalccmp(op, dd, dd, nil_matches=nm), ora.BATcalccmp(op, oo, oo, nil_matches=nm), "oid-oid " + op)
            same(gdk.BATcalccmp(op, dv, gdk.BAT.dense(3, 5), nil_matches=nm),
                 ora.BATcalccmp(op, ov, ora.Bat.dense(3, 5), nil_matches=nm), "void-void " + op)
    di, oi = mkpair(gdk, ora, "int", np.arange(5, dtype=np.int32))
    both_or_error(lambda: gdk.BATcalccmp("<", dd, di), lambda: ora.BATcalccmp("<", oo, oi), "oid-int")


@pytest.mark.gpu
@pytest.mark.parametrize("tp", ["bte", "int", "lng", "hge", "flt", "dbl"])
def test_calcbetween_parity(gdk, ora, tp):
    r = rng(7 + len(tp))
    n = 2000
    v, lo, hi = values_of(tp, n, r, 0.05), values_of(tp, n, r, 0.05), values_of(tp, n, r, 0.05)
    dv, ov = mkpair(gdk, ora, tp, v)
    dl, ol = mkpair(gdk, ora, tp, lo)
    dh, oh = mkpair(gdk, ora, tp, hi)
    T = getattr(gdk, "TYPE_" + tp)
    cl, ch = scalar_of(tp, lo, 1), scalar_of(tp, hi, 2)
    for sym in (False, True):
        for linc in (False, True):
            for hinc in (False, True):
                for nf in (False, True):
                    for anti in (False, True):
                        f = dict(symmetric=sym, linc=linc, hinc=hinc, nils_false=nf, anti=anti)
                        w = f"{tp} {f}"
                        same(gdk.BATcalcbetween(dv, dl, dh, **f), ora.BATcalcbetween(ov, ol, oh, **f), w)
                        same(gdk.BATcalcbetween(dv, None, None, clo=cl, chi=ch, ct=T, **f),
                             ora.BATcalcbetween(ov, None, None, clo=cl, chi=ch, ct=T, **f), w + " cstcst")
                        same(gdk.BATcalcbetween(dv, dl, None, chi=ch, ct=T, **f),
                             ora.BATcalcbetween(ov, ol, None, chi=ch, ct=T, **f), w + " batcst")
                        same(gdk.BATcalcbetween(dv, None, dh, clo=cl, ct=T, **f),
                             ora.BATcalcbetween(ov, None, oh, clo=cl, ct=T, **f), w + " cstbat")


@pytest.mark.gpu
def test_calcbetween_void(gdk, ora):
    oids = np.array([2, 9, 1 << 63, 4, 6, 8], np.uint64)
    dd, oo = mkpair(gdk, ora, "oid", oids)
    for f in (dict(), dict(symmetric=True), dict(anti=True, nils_false=True)):
        same(gdk.BATcalcbetween(gdk.BAT.dense(3, 6), dd, gdk.BAT.dense(5, 6), **f),
             ora.BATcalcbetween(ora.Bat.dense(3, 6), oo, ora.Bat.dense(5, 6), **f), f"void {f}")
        same(gdk.BATcalcbetween(gdk.BAT.dense(3, 6), gdk.BAT.dense(1, 6), gdk.BAT.dense(5, 6), **f),
             ora.BATcalcbetween(ora.Bat.dense(3, 6), ora.Bat.dense(1, 6), ora.Bat.dense(5, 6), **f), f"3void {f}")


CONV = [("bte", "int", 0, 0, 0), ("int", "bte", 0, 0, 0), ("lng", "int", 3, 1, 0), ("int", "lng", 0, 4, 9),
        ("lng", "hge", 2, 10, 0), ("hge", "lng", 6, 2, 18), ("sht", "bte", 1, 0, 2), ("int", "flt", 2, 0, 0),
        ("lng", "dbl", 3, 0, 0), ("hge", "flt", 0, 0, 0), ("hge", "dbl", 5, 0, 0), ("dbl", "lng", 0, 2, 0),
        ("flt", "int", 0, 3, 9), ("dbl", "hge", 0, 18, 0), ("dbl", "flt", 0, 0, 0), ("flt", "dbl", 0, 0, 0),
        ("dbl", "sht", 0, 1, 4), ("int", "bit", 0, 0, 0), ("dbl", "bit", 0, 0, 0), ("int", "oid", 0, 0, 0),
        ("dbl", "oid", 0, 0, 0), ("lng", "lng", 0, 0, 0), ("int", "int", 2, 0, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("st,dt,s1,s2,prec", CONV)
def test_convert_parity(gdk, ora, st, dt, s1, s2, prec):
    r = rng(len(st) * 31 + len(dt) + s1 + s2 + prec)
    n = 3000
    a = values_of(st, n, r, 0.05)
    if st in ("flt", "dbl"):
        a[3::9] = (r.integers(-10 ** 6, 10 ** 6, a[3::9].size) + 0.5) / 10 ** r.integers(0, 4, a[3::9].size)
    if dt == "oid" and st != "dbl":
        a = np.abs(a) if st != "hge" else a
    da, oa = mkpair(gdk, ora, st, a, hseq=3)
    T = getattr(gdk, "TYPE_" + dt)
    cand = np.sort(r.choice(np.arange(3, 3 + n), 1000, replace=False)).astype(np.uint64)
    dc = gdk.BAT.from_numpy(gdk.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    oc = ora.Bat.from_array(ora.TYPE_oid, cand, sorted_=True, key=True, nonil=True)
    w = f"{st}->{dt} ({s1},{s2},{prec})"
    both_or_error(lambda: gdk.BATconvert(da, None, T, s1, s2, prec), lambda: ora.BATconvert(oa, None, T, s1, s2, prec), w)
    both_or_error(lambda: gdk.BATconvert(da, dc, T, s1, s2, prec), lambda: ora.BATconvert(oa, oc, T, s1, s2, prec),
                  w + " cand")
    # a range without overflow: small magnitudes only
    small = np.zeros(n, bool)
    if st == "hge":
        vals = [scalar_of(st, a, i) for i in range(n)]
        small = np.array([abs(v) < 100 or v == -(1 << 127) for v in vals])
        b = a[small]
    else:
        fin = np.nan_to_num(a.astype(np.float64), nan=0.0)
        small = np.abs(fin) < 100
        b = a[small]
    db, ob = mkpair(gdk, ora, st, b)
    both_or_error(lambda: gdk.BATconvert(db, None, T, s1, s2, prec), lambda: ora.BATconvert(ob, None, T, s1, s2, prec),
                  w + " small")


@pytest.mark.gpu
def test_convert_void_and_errors(gdk, ora):
    for dt in ("bit", "bte", "int", "lng", "dbl", "oid"):
        T = getattr(gdk, "TYPE_" + dt)
        both_or_error(lambda: gdk.BATconvert(gdk.BAT.dense(100, 50), None, T),
                      lambda: ora.BATconvert(ora.Bat.dense(100, 50), None, T), "void->" + dt)
    both_or_error(lambda: gdk.BATconvert(gdk.BAT.dense(120, 50), None, gdk.TYPE_bte),
                  lambda: ora.BATconvert(ora.Bat.dense(120, 50), None, ora.TYPE_bte), "void->bte overflow")
    d, o = mkpair(gdk, ora, "dbl", np.array([1.0, 2.5, 1e300]))
    for dt in ("int", "lng", "flt", "oid"):
        T = getattr(gdk, "TYPE_" + dt)
        both_or_error(lambda: gdk.BATconvert(d, None, T), lambda: ora.BATconvert(o, None, T), "dbl overflow " + dt)
    d, o = mkpair(gdk, ora, "int", np.array([5, -3, 12], np.int32))
    both_or_error(lambda: gdk.BATconvert(d, None, gdk.TYPE_oid), lambda: ora.BATconvert(o, None, ora.TYPE_oid),
                  "negative oid")
    both_or_error(lambda: gdk.BATconvert(d, None, gdk.TYPE_sht, 0, 3, 4),
                  lambda: ora.BATconvert(o, None, ora.TYPE_sht, 0, 3, 4), "decimal precision")


@pytest.mark.gpu
@pytest.mark.parametrize("tp", ["bit", "bte", "sht", "int", "lng", "hge"])
def test_calcnot_parity(gdk, ora, tp):
    r = rng(3)
    a = values_of("bte" if tp == "bit" else tp, 1000, r)
    if tp == "bit":
        a = np.where(a == -128, -128, np.abs(a) % 2).astype(np.int8)
    d, o = mkpair(gdk, ora, tp, a)
    both_or_error(lambda: gdk.BATcalcnot(d), lambda: ora.BATcalcnot(o), "not " + tp)
    if tp in ("int", "lng"):
        mx = np.iinfo(np.int32 if tp == "int" else np.int64).max
        d, o = mkpair(gdk, ora, tp, np.array([1, mx, 3], a.dtype))
        both_or_error(lambda: gdk.BATcalcnot(d), lambda: ora.BATcalcnot(o), "not overflow " + tp)


DIVMOD = [("/", "int", "int", "int"), ("/", "lng", "int", "dbl"), ("/", "int", "dbl", "dbl"), ("/", "flt", "int", "flt"),
          ("/", "hge", "lng", "hge"), ("/", "dbl", "flt", "dbl"), ("/", "bte", "flt", "flt"), ("/", "sht", "int", "lng"),
          ("%", "int", "int", "int"), ("%", "lng", "bte", "bte"), ("%", "hge", "int", "int"), ("%", "int", "flt", "flt"),
          ("%", "dbl", "lng", "dbl"), ("%", "sht", "lng", "sht"), ("/", "int", "int", "bte"), ("%", "int", "sht", "bte")]


@pytest.mark.gpu
@pytest.mark.parametrize("op,t1,t2,tp", DIVMOD)
def test_divmod_parity(gdk, ora, op, t1, t2, tp):
    r = rng(11)
    n = 2000
    a, b = values_of(t1, n, r), values_of(t2, n, r)
    # no zero divisors except where checked below
    if t2 in ("flt", "dbl"):
        b[b == 0] = 3
    elif t2 == "hge":
        pass
    else:
        b[b == 0] = 7
    da, oa = mkpair(gdk, ora, t1, a)
    db, ob = mkpair(gdk, ora, t2, b)
    T, T1, T2 = (getattr(gdk, "TYPE_" + t) for t in (tp, t1, t2))
    w = f"{t1} {op} {t2} -> {tp}"
    both_or_error(lambda: gdk.BATcalcdivmod(op, da, db, T), lambda: ora.BATcalcdivmod(op, oa, ob, T), w)
    c = scalar_of(t2, b, 2)
    both_or_error(lambda: gdk.BATcalcdivmod(op, da, None, T, c2=c, t2=T2),
                  lambda: ora.BATcalcdivmod(op, oa, None, T, c2=c, t2=T2), w + " cst")
    c1 = scalar_of(t1, a, 5)
    both_or_error(lambda: gdk.BATcalcdivmod(op, None, db, T, c1=c1, t1=T1),
                  lambda: ora.BATcalcdivmod(op, None, ob, T, c1=c1, t1=T1), w + " cstbat")
    z = b.copy()
    z[n // 2] = 0
    dz, oz = mkpair(gdk, ora, t2, z)
    both_or_error(lambda: gdk.BATcalcdivmod(op, da, dz, T), lambda: ora.BATcalcdivmod(op, oa, oz, T), w + " zero")
