# vector group assign + project U=16: parity then op timings
set -e
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group_sums.py tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_group_sorted.py tests/test_gpu_aggr_sorted.py tests/test_gpu_window_funcs.py tests/test_select_str.py tests/test_join_str.py tests/test_join_algo.py > $O/tests.log 2>&1 || echo "TESTS FAILED" >> $O/tests.log
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/opbench.py --only other_ops > $O/prof.log 2>&1
