"""Threading contract (SURVEY.md §8 b): GDK is called concurrently by the MAL
dataflow workers (mal_dataflow.c:461-500).  Every calling thread has its own
HIP stream and the HBM allocator is shared under a lock, so concurrent calls
on disjoint inputs must give the same results as sequential ones.  The
ctypes calls release the GIL, so these threads really overlap in libmgdk."""
import threading

import numpy as np
import pytest


def _worker(gdk, seed, iters, errors):
    try:
        r = np.random.default_rng(seed)
        for it in range(iters):
            n = int(r.integers(1000, 300_000))
            a = r.integers(-1000, 1000, n).astype(np.int64)
            extra = r.integers(-1000, 1000, int(r.integers(1, 50_000))).astype(np.int64)
            # BATappend grows the tail (new heap, old one released after the
            # copy) while other threads allocate and free
            b = gdk.BAT.from_numpy(gdk.TYPE_lng, a)
            gdk.BATappend(b, gdk.BAT.from_numpy(gdk.TYPE_lng, extra))
            full = np.concatenate([a, extra])
            assert np.array_equal(b.to_numpy(), full), "append"
            s = gdk.BATthetaselect(b, None, 0, "<")
            want = np.flatnonzero(full < 0).astype(np.uint64)
            assert np.array_equal(s.to_numpy(), want), "select"
            p = gdk.BATproject(s, b)
            assert np.array_equal(p.to_numpy(), full[full < 0]), "project"
            g, e, h = gdk.BATgroup(gdk.BAT.from_numpy(gdk.TYPE_int, (full % 7).astype(np.int32)))
            assert int(np.sum(h.to_numpy())) == full.size, "group"
            assert gdk.BATsum(gdk.TYPE_hge, b) == int(full.sum()), "sum"
    except Exception as ex:  # noqa: BLE001
        errors.append((seed, repr(ex)))


@pytest.mark.gpu
def test_concurrent_operators(gdk):
    errors = []
    ts = [threading.Thread(target=_worker, args=(gdk, 100 + k, 12, errors)) for k in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


@pytest.mark.gpu
def test_concurrent_append_and_alloc(gdk):
    """BATappend released the old heap to the shared cache while
    its device-to-device copy was still queued.  Many small appends racing
    with allocations of the same size class in another thread."""
    errors = []
    stop = threading.Event()

    def churn():
        r = np.random.default_rng(7)
        while not stop.is_set():
            x = gdk.BAT.from_numpy(gdk.TYPE_lng, r.integers(0, 1 << 40, 4096).astype(np.int64))
            gdk.BATcalcaddcst(x, 1, gdk.TYPE_lng, gdk.TYPE_lng)

    def appender(seed):
        try:
            r = np.random.default_rng(seed)
            b = gdk.BAT.from_numpy(gdk.TYPE_lng, np.zeros(0, np.int64))
            ref = []
            for _ in range(200):
                c = r.integers(0, 1 << 40, int(r.integers(1, 3000))).astype(np.int64)
                gdk.BATappend(b, gdk.BAT.from_numpy(gdk.TYPE_lng, c))
                ref.append(c)
            assert np.array_equal(b.to_numpy(), np.concatenate(ref))
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    ch = threading.Thread(target=churn)
    ch.start()
    ap = [threading.Thread(target=appender, args=(s,)) for s in (1, 2, 3)]
    for t in ap:
        t.start()
    for t in ap:
        t.join()
    stop.set()
    ch.join()
    assert not errors, errors


@pytest.mark.gpu
def test_qry_ctx_timeout(gdk):
    """QryCtx (gdk/gdk_system.h:187, TIMEOUT_TEST gdk.h:2367): an operator of a
    thread whose query context has expired or was interrupted fails with the
    reference's message; other threads are not affected."""
    import threading
    import time
    b = gdk.BAT.from_numpy(gdk.TYPE_int, np.arange(100_000, dtype=np.int32))
    ctx = gdk.QryCtx(0, gdk.QRY_INTERRUPT)
    gdk.set_qry_ctx(ctx)
    try:
        with pytest.raises(gdk.GDKError, match="Query interrupted!"):
            gdk.BATthetaselect(b, None, 10, "<")
        ctx.endtime = gdk.usec() + 1
        time.sleep(0.01)
        with pytest.raises(gdk.GDKError, match="Timeout was reached!"):
            gdk.BATthetaselect(b, None, 10, "<")
        assert ctx.endtime == gdk.QRY_TIMEOUT
        # data transfers still work after the timeout (the reference tests
        # the context only inside operator loops): read back, upload
        assert b.to_numpy()[5] == 5
        assert gdk.BAT.from_numpy(gdk.TYPE_int, np.arange(10, dtype=np.int32)).to_numpy()[9] == 9
        # another thread without a context runs normally meanwhile
        out = []
        t = threading.Thread(target=lambda: out.append(gdk.BATthetaselect(b, None, 10, "<").count()))
        t.start()
        t.join()
        assert out == [10]
        ctx.endtime = gdk.usec() + 60_000_000
        assert gdk.BATthetaselect(b, None, 10, "<").count() == 10
    finally:
        gdk.set_qry_ctx(None)
    assert gdk.BATthetaselect(b, None, 10, "<").count() == 10
