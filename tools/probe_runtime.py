"""Probe coexistence of torch's bundled HIP runtime with libmgdk's (/opt/rocm)."""
import sys
import numpy as np

order = sys.argv[1] if len(sys.argv) > 1 else "torch-first"
import torch
if order == "torch-first":
    print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
    torch.cuda.set_device(0)
    x = torch.arange(10, device="cuda:0")
    print("torch op", int(x.sum()))
from monetdb_amd import gdk
gdk.init(0)
b = gdk.BAT.from_numpy(gdk.TYPE_lng, np.arange(1000, dtype=np.int64))
print("gdk roundtrip", int(b.to_numpy().sum()))
print("torch avail after", torch.cuda.is_available(), torch.cuda.device_count())
if torch.cuda.is_available():
    t = torch.empty(1000, dtype=torch.int64, device="cuda:0")
    gdk.BATdownload_device(b, t.data_ptr())
    print("download via torch ptr", int(t.sum()))
