"""msk (bit) BATs as candidate lists and BATmaskedcands.

A TYPE_msk BAT stands for the oid list BATunmask makes of it (hseqbase + i
for every set bit i < count, gdk/gdk_cand.c:1464 / :1549-1599): BATjoin and
BATproject2 unmask msk inputs first (gdk_join.c:4500-4517,
gdk_project.c:652-660); canditer_init's own msk branch is an assert(0)
(gdk_cand.c:468), so every operator takes a msk s as that list.
BATmaskedcands (gdk_cand.c:1366) turns a msk BAT into a cand_mask list.
The CPU tests pin the oracle's restatement against numpy; the -m gpu tests
compare the device with the oracle on select, thetaselect, project,
groupsum, sum, join and BATmaskedcands."""
import numpy as np
import pytest

from helpers import rng


def _bits(seed, n, p=0.3):
    return rng(seed).random(n) < p


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 1000, 4097])
def test_oracle_unmask(ora, n):
    bits = _bits(n + 1, n)
    got = ora.unmask(ora.Bat.msk(bits, hseqbase=70)).values()
    assert np.array_equal(np.asarray(got, np.uint64), (70 + np.flatnonzero(bits)).astype(np.uint64))


@pytest.mark.parametrize("nr,count,selected", [(100, 100, True), (100, 100, False), (150, 100, True),
                                               (150, 100, False), (64, 100, True), (33, 7, False),
                                               (40, 0, True)])
def test_oracle_maskedcands(ora, nr, count, selected):
    bits = _bits(nr * 7 + count, count)
    got = np.asarray(ora.maskedcands(5, nr, ora.Bat.msk(bits), selected).values(), np.uint64)
    if count == 0:
        want = np.zeros(0, np.uint64)
    else:
        sel = np.ones(nr, bool)
        k = min(nr, count)
        sel[:k] = bits[:k] if selected else ~bits[:k]
        want = (5 + np.flatnonzero(sel)).astype(np.uint64)
    assert np.array_equal(got, want)


def test_oracle_select_msk_equals_list(ora):
    r = rng(5)
    v = r.integers(-50, 50, 3000).astype(np.int32)
    bits = _bits(6, 2500)
    B = ora.Bat.from_array(ora.TYPE_int, v, hseqbase=10)
    S = ora.Bat.msk(bits, hseqbase=300)
    L = ora.Bat.from_array(ora.TYPE_oid, 300 + np.flatnonzero(bits), sorted_=True, key=True, nonil=True)
    a = ora.BATselect(B, S, -10, 20, True, False, False).values()
    b = ora.BATselect(B, L, -10, 20, True, False, False).values()
    assert np.array_equal(np.asarray(a), np.asarray(b))


@pytest.mark.gpu
@pytest.mark.parametrize("hseq,n", [(0, 50_000), (100, 50_000), (7, 33), (0, 1_000_000)])
def test_msk_cand_operators(gdk, ora, hseq, n):
    r = rng(n + hseq)
    v = r.integers(-1000, 1000, 60_000).astype(np.int32)
    v[::97] = gdk.NIL[gdk.TYPE_int]
    B, OB = gdk.BAT.from_numpy(gdk.TYPE_int, v, hseqbase=100), ora.Bat.from_array(ora.TYPE_int, v, hseqbase=100)
    bits = _bits(hseq + 3, n, 0.4)
    S, OS = gdk.BAT.msk(bits, hseqbase=hseq), ora.Bat.msk(bits, hseqbase=hseq)
    got = gdk.BATselect(B, S, -100, 300, True, False, False).to_numpy()
    want = np.asarray(ora.BATselect(OB, OS, -100, 300, True, False, False).values())
    assert np.array_equal(got, want)
    got = gdk.BATthetaselect(B, S, 0, ">=").to_numpy()
    want = np.asarray(ora.BATthetaselect(OB, OS, 0, ">=").values())
    assert np.array_equal(got, want)
    assert gdk.BATsum(gdk.TYPE_lng, B, s=S) == ora.BATsum(ora.TYPE_lng, OB, s=OS)
    # groupsum with the msk as candidates
    # (g holds one id per candidate, its head at the first candidate:
    # BATgroupaggrinit, gdk_aggr.c:76-80)
    cands = hseq + np.flatnonzero(bits)
    cands = cands[(cands >= 100) & (cands < 100 + v.size)]
    if cands.size:
        gk = (cands % 17).astype(np.int32)
        G = gdk.BAT.from_numpy(gdk.TYPE_int, gk, hseqbase=int(cands[0]))
        g, e, _ = gdk.BATgroup(G)
        og, oe, _ = ora.BATgroup(ora.Bat.from_array(ora.TYPE_int, gk, hseqbase=int(cands[0])))
        got = gdk.BATgroupsum(B, g, e, gdk.TYPE_lng, s=S).values()
        want = ora.BATgroupsum(OB, og, oe, ora.TYPE_lng, s=OS).values()
        assert list(got) == list(want)
    # join with the msk as left candidates, and a msk joined as a value column
    rk = r.permutation(2000).astype(np.int32) - 1000
    R = gdk.BAT.from_numpy(gdk.TYPE_int, rk)
    OR = ora.Bat.from_array(ora.TYPE_int, rk, key=True, nonil=True)
    r1, r2 = gdk.BATjoin(B, R, sl=S)
    o1, o2 = ora.BATjoin(OB, OR, sl=OS)
    assert np.array_equal(r1.to_numpy(), np.asarray(o1.values()))
    assert np.array_equal(r2.to_numpy(), np.asarray(o2.values()))
    # projection through a msk left (BATproject2's BATunmask)
    if hseq + n <= 100 + v.size and hseq >= 100:
        got = gdk.BATproject(S, B).to_numpy()
        want = np.asarray(ora.BATproject(OS, OB).values())
        assert np.array_equal(got, want)


@pytest.mark.gpu
def test_msk_project_and_join_values(gdk, ora):
    r = rng(9)
    bits = _bits(10, 5000)
    v = r.integers(0, 10**6, 5000).astype(np.int64)
    B, OB = gdk.BAT.from_numpy(gdk.TYPE_lng, v, hseqbase=0), ora.Bat.from_array(ora.TYPE_lng, v)
    S, OS = gdk.BAT.msk(bits), ora.Bat.msk(bits)
    got = gdk.BATproject(S, B).to_numpy()
    want = np.asarray(ora.BATproject(OS, OB).values())
    assert np.array_equal(got, want)
    # a msk as a join input: its unmasked oids joined with an oid column
    oids = np.sort(r.choice(5000, 800, replace=False)).astype(np.uint64)
    O, OO = gdk.BAT.from_numpy(gdk.TYPE_oid, oids), ora.Bat.from_array(ora.TYPE_oid, oids, sorted_=True,
                                                                         key=True, nonil=True)
    a1, a2 = gdk.BATjoin(S, O)
    b1, b2 = ora.BATjoin(OS, OO)
    assert np.array_equal(a1.to_numpy(), np.asarray(b1.values()))
    assert np.array_equal(a2.to_numpy(), np.asarray(b2.values()))


@pytest.mark.gpu
@pytest.mark.parametrize("nr,count,selected", [(100, 100, True), (100, 100, False), (150, 100, True),
                                               (150, 100, False), (64, 100, True), (40, 0, True),
                                               (3_000_017, 3_000_000, False)])
def test_maskedcands_device(gdk, ora, nr, count, selected):
    """BATmaskedcands: the void + ccand_t mask list (firstbit, count,
    tseqbase = hseq + firstbit, no vheap when empty) holds exactly the
    oracle's candidates; operators read it as such."""
    bits = _bits(nr + count, count)
    M = gdk.BATmaskedcands(11, nr, gdk.BAT.msk(bits), selected)
    want = np.asarray(ora.maskedcands(11, nr, ora.Bat.msk(bits), selected).values(), np.uint64)
    assert M.count() == want.size
    if want.size:
        assert M.s.tseqbase == int(want[0])
        hdr = np.zeros(M.s.tvheapsize, np.uint8)
        gdk.lib().mgdk_BATdownload_vheap(M.ptr, hdr.ctypes.data)
        h = int(hdr[:8].view(np.uint64)[0])
        assert h & 1 == 1 and (h >> 1) == int(want[0]) - 11
        words = hdr[8:].view(np.uint32)
        cand = 11 + np.flatnonzero(np.unpackbits(words.view(np.uint8), bitorder="little"))
        assert np.array_equal(cand.astype(np.uint64), want)
        # an operator sees the same candidates
        v = np.arange(nr + 20, dtype=np.int32)
        B = gdk.BAT.from_numpy(gdk.TYPE_int, v, hseqbase=11)
        got = gdk.BATthetaselect(B, M, -1, ">").to_numpy()
        assert np.array_equal(got, want)
    else:
        assert M.s.tvheapsize == 0
