# MSD-then-local sort on the bench's 30-bit keys: parity, timings (hybrid /
# LSD, XCD groups), kernel trace of one sort
set -e
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_hybrid.py > $O/hybrid_tests.log 2>&1
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_hy.json 2> $O/opbench_hy.err
MGDK_SORT_XCDG=16 timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_hy_xg16.json 2> $O/opbench_hy_xg16.err
MGDK_SORT_XCDG=64 timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_hy_xg64.json 2> $O/opbench_hy_xg64.err
MGDK_SORT_HYBRID=0 MGDK_SORT_XCDG=64 timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench_lsd_xg64.json 2> $O/opbench_lsd_xg64.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/run_sort.py > $O/prof.log 2>&1
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py -k "sort or order" > $O/sort_tests.log 2>&1 || echo "SORT TESTS FAILED" >> $O/sort_tests.log
bash tools/gpu_r4_c.sh
