# parity of every radix-sort user after the per-width XCD group default, op timings
set -e
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_join_sort_window.py tests/test_gpu_sort_qsort.py tests/test_gpu_str_sort.py tests/test_gpu_sort_hybrid.py tests/test_gpu_firstn.py tests/test_gpu_group_str.py tests/test_gpu_exchange_ops.py tests/test_gpu_ops.py tests/test_join_str.py tests/test_gpu_distributed.py > $O/tests.log 2>&1 || echo "TESTS FAILED" >> $O/tests.log
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench.json 2> $O/opbench.err
