# MSD-then-local sort: parity at >= 2^22 rows + the existing sort tests, op
# timings with the hybrid on / off; then the round-4 parity batch (r4c)
set -e
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py > $O/hybrid_tests.log 2>&1
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py -k "sort or order" > $O/sort_tests.log 2>&1 || echo "SORT TESTS FAILED" >> $O/sort_tests.log
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_hy.json 2> $O/opbench_hy.err
MGDK_SORT_FUSEGID=0 timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_nofg.json 2> $O/opbench_nofg.err
MGDK_SORT_XCDG=4 timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_xg4.json 2> $O/opbench_xg4.err
MGDK_SORT_XCDG=16 timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_xg16.json 2> $O/opbench_xg16.err
MGDK_SORT_XCDG=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py > $O/hybrid_tests_xg4.log 2>&1
MGDK_SORT_HYBRID=0 timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_lsd.json 2> $O/opbench_lsd.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/run_sort.py > $O/prof.log 2>&1
bash tools/gpu_r4_c.sh
bash tools/ssweep.sh w8r32 w4r64
