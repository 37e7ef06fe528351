# one-wave local pass: parity, per-kernel times with and without the fused group ids
set -e
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py > $O/hybrid_tests.log 2>&1
MGDK_SORT_LOCALXG=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py -k "int32 or digits" > $O/hybrid_tests_xg0.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_default -o run -- python tools/run_sort.py > $O/p_default.log 2>&1
MGDK_SORT_FUSEGID=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_nofg -o run -- python tools/run_sort.py > $O/p_nofg.log 2>&1
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench.json 2> $O/opbench.err
