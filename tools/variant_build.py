"""Build a side variant of libmgdk.so with compile-time overrides for ONE source
(tuning sweeps only; the product library is monetdb_amd/libmgdk.so).

    python tools/variant_build.py NAME SOURCE.hip -DMACRO=VALUE ...
    MGDK_LIB=$PWD/tools/variants/libmgdk_NAME.so python tools/opbench.py ...
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from monetdb_amd import build as B  # noqa: E402


def main():
    name, src = sys.argv[1], sys.argv[2]
    defs = sys.argv[3:]
    B.build()
    out = os.path.join(ROOT, "tools", "variants")
    os.makedirs(out, exist_ok=True)
    vobj = os.path.join(out, name + "_" + os.path.basename(src) + ".o")
    srcp = os.path.join(B.CSRC, src)
    subprocess.run([B.HIPCC] + B.CFLAGS + defs + ["-c", srcp, "-o", vobj], check=True)
    objs = [os.path.join(B.OBJ, os.path.basename(s) + ".o")
            for s in sorted(os.listdir(B.CSRC)) if s.endswith(".hip") and s != src]
    lib = os.path.join(out, "libmgdk_%s.so" % name)
    subprocess.run([B.HIPCC, "--offload-arch=" + B.ARCH, "-shared", "-fPIC", "-o", lib] + objs + [vobj],
                   check=True)
    print(lib)


if __name__ == "__main__":
    main()
