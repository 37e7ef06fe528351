"""Q6 op-at-a-time at SF100 (the GDK API path), a few timed runs, for a
rocprofv3 kernel trace:  rocprofv3 --kernel-trace ... -- python3 tools/q6op_trace.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from monetdb_amd import gdk  # noqa: E402

gdk.init(0)
rows = int(os.environ.get("Q6_ROWS", "600121500"))
cols = gdk.tpch_lineitem(20241024, 0, rows, max(1, rows // 30))
mk = lambda y, m, d: (((y + 4712) * 12 + m - 1) << 5) | d
args = (cols["shipdate"], cols["discount"], cols["quantity"], cols["extendedprice"],
        mk(1994, 1, 1), mk(1995, 1, 1), 5, 7, 2400)
ref = gdk.q6_fused(*args)
for _ in range(3):
    t = time.perf_counter()
    assert gdk.q6_opatatime(*args) == ref
    print("q6 op-at-a-time %.3f ms" % ((time.perf_counter() - t) * 1e3))
