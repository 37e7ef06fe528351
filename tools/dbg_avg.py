import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from helpers import rng
import test_gpu_analytic as T
from monetdb_amd import gdk
from oracle import pyoracle as ora
gdk.init(0)
r = rng(311)
_, p, o, ob = T._data(r, nparts=31, plen=900)
n = len(p)
v = T._avg_input(r, "lng", n)
for frame in (3, 4, 5):
    got = gdk.GDKanalyticalavg(gdk.BAT.from_numpy(gdk.TYPE_lng, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                               gdk.BAT.from_numpy(gdk.TYPE_bit, o), None, None, frame).values()
    want = np.asarray(ora.analyticalavg(ora.Bat.from_array(gdk.TYPE_lng, v), ora.Bat.from_array(ora.TYPE_bit, p),
                             ora.Bat.from_array(ora.TYPE_bit, o), None, None, frame).values())
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    print(frame, len(bad), [(int(i), got[i], want[i]) for i in bad[:5]])
    s = gdk.GDKanalyticalsum(gdk.BAT.from_numpy(gdk.TYPE_lng, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                               gdk.BAT.from_numpy(gdk.TYPE_bit, o), None, None, gdk.TYPE_hge, frame).values()
    c = gdk.GDKanalyticalcount(gdk.BAT.from_numpy(gdk.TYPE_lng, v), gdk.BAT.from_numpy(gdk.TYPE_bit, p),
                               gdk.BAT.from_numpy(gdk.TYPE_bit, o), None, None, True, frame).to_numpy()
    for i in bad[:5]:
        print("  sum", s[i], "cnt", c[i], "float(sum)/cnt", float(s[i]) / float(c[i]))
