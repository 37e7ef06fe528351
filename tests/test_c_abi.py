"""The boundary from C (not ctypes): tests/c_abi/abi_test.c includes only
include/mgdk.h and links libmgdk.so.  On CPU: it compiles as strict C99
(-pedantic) and links against every entry point it uses.  On the GPU: it runs
select -> project -> sum and a forced overflow whose reference message
(22003!overflow in calculation ...) it reads from mgdk_GDKerrbuf."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
DIR = os.path.join(HERE, "c_abi")
ROOT = os.path.dirname(HERE)


def _build():
    r = subprocess.run(["make", "-s", "-C", DIR], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return os.path.join(DIR, "abi_test")


def test_c_abi_compiles_and_links():
    if not os.path.exists(os.path.join(ROOT, "monetdb_amd", "libmgdk.so")):
        pytest.skip("libmgdk.so not built")
    exe = _build()
    r = subprocess.run(["nm", "-u", exe], capture_output=True, text=True)
    used = {l.split()[-1] for l in r.stdout.splitlines() if "mgdk_" in l}
    assert {"mgdk_BATthetaselect", "mgdk_BATproject", "mgdk_BATsum", "mgdk_BATcalcmulcst",
            "mgdk_GDKerrbuf", "mgdk_GDKclrerr"} <= used
    r = subprocess.run(["ldd", exe], capture_output=True, text=True)
    assert "libmgdk.so" in r.stdout and "not found" not in r.stdout.split("libmgdk.so")[1].splitlines()[0]


@pytest.mark.gpu
def test_c_abi_runs_on_gpu():
    exe = os.path.join(DIR, "abi_test")
    if not os.path.exists(exe):
        exe = _build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1] == "abi ok"
