"""BATselect / BATthetaselect on str columns (gdk/gdk_select.c:1342 generic
part with strCmp -- nil before every string, then strcmp -- and
fullscan_any :449-605; fullscan_str's string-elimination path :608-760
gives the same oids).  The CPU tests pin the oracle's restatement against
a Python model of the same rules; the -m gpu tests compare the device with
the oracle over every li / hi / anti / nil_matches combination, nil bounds,
candidate lists (dense, materialised, msk) and 1- / 2- / 4- / 8-byte offsets."""
import itertools

import numpy as np
import pytest

from helpers import rng
from strheap import NIL, WORDS, sample

BOUNDS = [b"A", b"N", b"abcdefgh", b"zz", b"", b"B", NIL, None]


def _cmp(a, b):
    """strCmp: nil first, then bytewise"""
    if a == NIL or b == NIL:
        return -int(b != NIL) if a == NIL else 1
    return (a > b) - (a < b)


def _model(words, tl, th, li, hi, anti, nil_matches):
    """BATselect's normalisation (gdk_select.c:1342-1520) + fullscan_any"""
    lnil = _cmp(tl, NIL) == 0
    lval = not lnil or th is None
    equi = th is None or (lval and _cmp(tl, th) == 0)
    if lnil and nil_matches and (th is None or _cmp(th, NIL) == 0):
        equi = lval = True
    if equi:
        if th is None:
            hi = li
        th = tl
        hval = True
        if not anti and (not li or not hi):
            return []
    else:
        nil_matches = False
        hval = _cmp(th, NIL) != 0
    abn = False
    if anti:
        if lval != hval:
            li, hi, tl, th, lval, hval = not hi, not li, th, tl, hval, lval
            lnil = _cmp(tl, NIL) == 0
            anti = False
        elif not lval and not hval:
            return []
        elif (equi and (lnil or not (li and hi))) or _cmp(tl, th) > 0:
            if equi and not lnil and nil_matches and not (li and hi):
                return list(range(len(words)))
            abn = True
        else:
            equi = False
    if not abn and hval and ((not li or not hi) if equi else _cmp(tl, th) > 0):
        return []
    out = []
    for i, v in enumerate(words):
        isnil = v == NIL
        if abn:
            ok = not isnil
        elif equi:
            ok = _cmp(tl, v) == 0
        elif anti:
            ok = (nil_matches and isnil) or (not isnil and ((lval and (_cmp(tl, v) > 0 or (not li and _cmp(tl, v) == 0)))
                                                          or (hval and (_cmp(th, v) < 0 or (not hi and _cmp(th, v) == 0)))))
        else:
            ok = not isnil and (not lval or _cmp(tl, v) < 0 or (li and _cmp(tl, v) == 0)) and \
                (not hval or _cmp(th, v) > 0 or (hi and _cmp(th, v) == 0))
        if ok:
            out.append(i)
    return out


CASES = [(tl, th, li, hi, anti, nm)
         for tl, th in [(b"A", b"N"), (b"N", b"A"), (b"abcdefgh", None), (NIL, None), (NIL, b"N"), (b"B", NIL),
                        (NIL, NIL), (b"", b"zz"), (b"zz", b"zz")]
         for li, hi, anti, nm in itertools.product([False, True], repeat=4)]


def test_oracle_str_select_model(ora):
    r = rng(31)
    t, heap, wi = sample(r, 3000, 4)
    words = [WORDS[i] for i in wi]
    b = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap, hseqbase=5)
    for tl, th, li, hi, anti, nm in CASES:
        got = list(np.asarray(ora.BATselect(b, None, tl, th, li, hi, anti, nm).values()) - 5)
        assert got == _model(words, tl, th, li, hi, anti, nm), (tl, th, li, hi, anti, nm)


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 2, 4, 8])
def test_str_select_device(gdk, ora, width):
    r = rng(40 + width)
    n = 60_000 if width != 1 else 5_000
    # 1-byte offsets reach 255 bytes past the header: one copy of each word
    t, heap, wi = sample(r, n, width, copies=1 if width == 1 else 6)
    D = gdk.BAT.from_numpy(gdk.TYPE_str, t, vheap=heap, hseqbase=7, sorted_=False, revsorted=False, key=False,
                           nonil=False)
    O = ora.Bat.from_array(ora.TYPE_str, t, vheap=heap, hseqbase=7)
    cands = np.sort(r.choice(n, n // 3, replace=False)).astype(np.uint64) + 7
    SD = gdk.BAT.from_numpy(gdk.TYPE_oid, cands, sorted_=True, key=True, nonil=True)
    SO = ora.Bat.from_array(ora.TYPE_oid, cands, sorted_=True, key=True, nonil=True)
    bits = r.random(n) < 0.5
    MD, MO = gdk.BAT.msk(bits, hseqbase=7), ora.Bat.msk(bits, hseqbase=7)
    for tl, th, li, hi, anti, nm in CASES:
        for sd, so in ((None, None), (SD, SO), (MD, MO)):
            got = gdk.BATselect(D, sd, tl, th, li, hi, anti, nm).to_numpy()
            want = np.asarray(ora.BATselect(O, so, tl, th, li, hi, anti, nm).values())
            assert np.array_equal(got, want), (tl, th, li, hi, anti, nm, sd is not None)
    for op in ("<", "<=", ">", ">=", "==", "!=", "<>", "eq", "ne"):
        for v in (b"N", b"abcdefgi", NIL):
            got = gdk.BATthetaselect(D, None, v, op).to_numpy()
            want = np.asarray(ora.BATthetaselect(O, None, v, op).values())
            assert np.array_equal(got, want), (op, v)
