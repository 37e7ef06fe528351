"""Build libmgdk.so (HIP, gfx950) in-tree with hipcc.

Every .hip under monetdb_amd/csrc is compiled to an object with
`hipcc --offload-arch=gfx950 -O3 -fPIC -c` (in parallel) and linked into
monetdb_amd/libmgdk.so.  Objects are rebuilt only when their source or a
header is newer.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build_obj")
LIB = os.path.join(HERE, "libmgdk.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable", "-I" + os.path.join(HERE, "..", "include")]


def _headers_mtime():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(HERE, "..", "include", "*.h"))
    return max(os.path.getmtime(h) for h in hs)


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime()):
        return obj, None
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, r.stderr
    return obj, None


def build(verbose=False, jobs=8):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    objs = []
    errors = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for obj, err in ex.map(_compile, srcs):
            objs.append(obj)
            if err:
                errors.append(err)
    if errors:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errors))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True, jobs=int(sys.argv[1]) if len(sys.argv) > 1 else 8)
