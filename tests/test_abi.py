"""The C-ABI library loads and exports every entry point include/mgdk.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "mgdk.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mgdk_[A-Za-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    fns = header_functions()
    for f in ("mgdk_BATselect", "mgdk_BATthetaselect", "mgdk_BATproject", "mgdk_BATcalcmul",
              "mgdk_BATsum", "mgdk_BATgroup", "mgdk_BATgroupsum", "mgdk_BATgroupavg3",
              "mgdk_BATjoin", "mgdk_BATsort", "mgdk_GDKanalyticalwindowbounds"):
        assert f in fns


def test_library_exports_every_symbol():
    from monetdb_amd import gdk
    lib = ctypes.CDLL(gdk.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_python_mirror_binds_all():
    from monetdb_amd import gdk
    lib = gdk.lib()     # binds every signature in gdk._SIGS (fails on a missing symbol)
    assert set(gdk._SIGS) <= set(header_functions())


def test_no_oracle_in_product():
    """The product path never imports or links the oracle."""
    pkg = os.path.join(ROOT, "monetdb_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert "pyoracle" not in src and "liboracle" not in src and "gdk_oracle" not in src, f
