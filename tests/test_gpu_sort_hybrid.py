"""BATsort's MSD-then-local path (sort.hip `radix_hybrid`: a stable scatter by
the top varying digit, a stable scatter by the next one inside its buckets,
then every (d1, d2) bucket sorted by its remaining bits in one workgroup's
LDS) against the oracle's stable sort (gdk_batop.c:2342 -> GDKrsort) at
sizes that take it (>= 2^22 rows of a 4-byte type with >= 3 varying key
digits): full-range and 30-bit int32 with nils, both directions; 3 varying
digits; floats (order + gathered values + groups from the key images);
correlated top digits whose (d1, d2) buckets overflow the LDS capacity and
are sorted by the host fallback."""
import numpy as np
import pytest

from helpers import rng, with_nils

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hybrid_on(monkeypatch):
    """the path is off by default (slower than the LSD passes at 100M int32,
    DESIGN §9); the library reads the switch on every call"""
    monkeypatch.setenv("MGDK_SORT_HYBRID", "1")

N = (1 << 22) + 12_345


def _mk(G, tp, vals, **kw):
    return G.BAT.from_numpy(tp, np.asarray(vals), sorted_=False, revsorted=False, key=False, **kw)


def _groups(sv):
    return np.concatenate([[0], np.cumsum(sv[1:] != sv[:-1])]).astype(np.uint64)


def _check_int(gdk, ora, vals, reverse=False, hseq=7):
    s, o, g = gdk.BATsort(_mk(gdk, gdk.TYPE_int, vals, hseqbase=hseq), reverse=reverse, nilslast=reverse)
    os_, oo = ora.BATsort(ora.Bat.from_array(ora.TYPE_int, vals, hseqbase=hseq), reverse=reverse,
                          nilslast=reverse)
    assert np.array_equal(o.to_numpy(), oo.values())
    assert np.array_equal(s.to_numpy(), os_.values())
    assert np.array_equal(g.to_numpy(), _groups(s.to_numpy()))


@pytest.mark.parametrize("reverse", [False, True])
def test_hybrid_int32_full_range(gdk, ora, reverse):
    r = rng(501)
    vals = with_nils(r.integers(-2**31 + 1, 2**31 - 1, N, dtype=np.int64).astype(np.int32),
                     gdk.NIL[gdk.TYPE_int], 0.02, r)
    _check_int(gdk, ora, vals, reverse)


def test_hybrid_int32_30bit_duplicates(gdk, ora):
    r = rng(502)
    pool = r.integers(0, 1 << 30, 300_000, dtype=np.int64).astype(np.int32)
    _check_int(gdk, ora, pool[r.integers(0, pool.size, N)])


def test_hybrid_three_digits(gdk, ora):
    r = rng(503)
    _check_int(gdk, ora, r.integers(0, 1 << 24, N, dtype=np.int64).astype(np.int32))


@pytest.mark.parametrize("lo,hi", [(0, 1 << 19), (-(1 << 20), 1 << 20), (5, (1 << 27) + 5)])
def test_hybrid_unaligned_digits(gdk, ora, lo, hi):
    """the MSD digits are the top 8 + 8 VARYING bits, not whole bytes (an
    extra count pass); ranges straddling the sign flip fall back to LSD"""
    r = rng(507)
    _check_int(gdk, ora, r.integers(lo, hi, N, dtype=np.int64).astype(np.int32))


def test_hybrid_overflowing_buckets(gdk, ora):
    """d1 == d2 on every row: the marginals look uniform but each (x, x)
    bucket holds n / 256 rows, far above the LDS capacity"""
    r = rng(504)
    x = r.integers(0, 256, N, dtype=np.uint64)
    v = (x * 0x01010000 + r.integers(0, 1 << 16, N, dtype=np.uint64)).astype(np.uint32).view(np.int32)
    _check_int(gdk, ora, v)
    # and a few overflowing buckets among regular ones
    v2 = r.integers(-2**31 + 1, 2**31 - 1, N, dtype=np.int64).astype(np.int32)
    v2[: N // 8] = 0x12340000 + (r.integers(0, 4096, N // 8)).astype(np.int32)
    _check_int(gdk, ora, r.permutation(v2))


@pytest.mark.parametrize("reverse", [False, True])
def test_hybrid_float(gdk, reverse):
    r = rng(505)
    vals = (r.standard_normal(N) * 1e3).astype(np.float32)
    vals[r.random(N) < 0.01] = np.nan
    vals[r.random(N) < 0.01] = -0.0
    vals[r.random(N) < 0.01] = 0.0
    s, o, g = gdk.BATsort(_mk(gdk, gdk.TYPE_flt, vals), reverse=reverse, nilslast=reverse)
    key = np.where(np.isnan(vals), -np.inf, vals).astype(np.float64)      # nil first (ascending)
    key = np.where(key == 0, 0.0, key)                                    # -0 == +0
    if reverse:
        key = -key                                                        # nil last, ties stay in input order
    perm = np.argsort(key, kind="stable")
    assert np.array_equal(o.to_numpy(), perm.astype(np.uint64))
    assert np.array_equal(s.to_numpy().view(np.uint32), vals[perm].view(np.uint32))
    ks = key[perm]
    assert np.array_equal(g.to_numpy(), _groups(ks))


def test_hybrid_stable_permutation(gdk):
    """many ties in the top digits: a sorted, stable permutation (ties in
    input order)"""
    r = rng(506)
    vals = r.integers(-2**31 + 1, 2**31 - 1, N, dtype=np.int64).astype(np.int32)
    vals[::3] = vals[::3] // 65536        # many ties in the top digits
    s, o, _ = gdk.BATsort(_mk(gdk, gdk.TYPE_int, vals))
    on = o.to_numpy().astype(np.int64)
    sv = s.to_numpy()
    assert np.array_equal(np.sort(on), np.arange(N))
    assert np.array_equal(vals[on], sv)
    assert (np.diff(sv.astype(np.int64)) >= 0).all()
    tie = sv[1:] == sv[:-1]
    assert (on[1:][tie] > on[:-1][tie]).all()
