"""Q6 fused-kernel launch-variant sweep (interleaved rounds in one process)."""
import ctypes as C
import statistics
import sys
import time

sys.path.insert(0, ".")
from monetdb_amd import gdk

gdk.init(0)
import os
rows = int(os.environ.get("Q6_ROWS", "600121500"))
cols = gdk.tpch_lineitem(20241024, 0, rows, max(1, rows // 30))
mk = lambda y, m, d: (((y + 4712) * 12 + m - 1) << 5) | d
args = (cols["shipdate"], cols["discount"], cols["quantity"], cols["extendedprice"],
        mk(1994, 1, 1), mk(1995, 1, 1), 5, 7, 2400)
L = gdk.lib()
L.mgdk_q6_set_variant.argtypes = [C.c_int, C.c_int]
ref = gdk.q6_fused(*args)
vs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2, 3, 4, 5, 9, 12]
bs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [4, 8, 16]
variants = [(v, b) for v in vs for b in bs]
res = {k: [] for k in variants}
gdk.prof_enable(True)
for rnd in range(4):
    for v, b in variants:
        L.mgdk_q6_set_variant(v, b)
        gdk.prof_reset()
        for _ in range(5):
            assert gdk.q6_fused(*args) == ref
        ms, n = gdk.prof_get("q6_fused")
        res[(v, b)].append(ms / n)
L.mgdk_q6_last_sectors.restype = C.c_ulonglong
for k in variants:
    L.mgdk_q6_set_variant(*k)
    gdk.q6_fused(*args)
    sect = L.mgdk_q6_last_sectors()
    nbytes = rows * 28 if sect == 0 else rows * 4 + sect * 128   # bytes the variant reads
    med = statistics.median(res[k])
    print("variant %2d bpc %2d: %.4f ms  %.1f GB/s read (%.2f GB)  %.1f Grows/s" % (
        k[0], k[1], med, nbytes / med / 1e6, nbytes / 1e9, rows / med / 1e6))
