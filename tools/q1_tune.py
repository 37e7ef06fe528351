"""Fused Q1 main-pass layout / workgroup-count sweep (interleaved rounds in one process).

    python tools/q1_tune.py [LAYOUTS] [BLOCKS]      e.g. 0,1 512,768,1024
"""
import ctypes as C
import statistics
import sys

sys.path.insert(0, ".")
from monetdb_amd import gdk  # noqa: E402

gdk.init(0)
rows = 600_121_500
cols = gdk.tpch_lineitem(20241024, 0, rows, 20_000_000)
dmax = (((1998 + 4712) * 12 + 9 - 1) << 5) | 2
L = gdk.lib()
L.mgdk_q1_set_variant.argtypes = [C.c_int, C.c_int]
ref = gdk.q1_fused(cols, dmax)
ls = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1]
bs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [512, 768, 1024]
variants = [(lay, b) for lay in ls for b in bs]
res = {k: [] for k in variants}
gdk.prof_enable(True)
for rnd in range(3):
    for lay, b in variants:
        L.mgdk_q1_set_variant(lay, b)
        gdk.prof_reset()
        for _ in range(4):
            assert gdk.q1_fused(cols, dmax) == ref
        ms, n = gdk.prof_get("q1_fused")
        res[(lay, b)].append(ms / n)
for k in variants:
    med = statistics.median(res[k])
    print("layout %d blocks %4d: %.4f ms  %.1f GB/s" % (k[0], k[1], med, rows * 38 / med / 1e6))
