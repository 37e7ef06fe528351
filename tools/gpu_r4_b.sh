# group sums (LDS-staged) + window functions: parity, then kernel times
set -e
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group_sums.py tests/test_gpu_window_funcs.py tests/test_gpu_analytic.py > $O/tests.log 2>&1 || echo "TESTS FAILED" >> $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/prof_dist_group.py 600121500 > $O/prof.log 2>&1
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench.json 2>&1
