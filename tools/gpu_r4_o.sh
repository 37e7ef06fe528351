# group-path parity with 32 Ki-row assign tiles, op timings
set -e
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_group_sums.py tests/test_gpu_group_sorted.py tests/test_gpu_group_str.py tests/test_gpu_firstn.py tests/test_gpu_dict.py tests/test_gpu_aggr_sorted.py tests/test_msk_cands.py tests/test_join_str.py tests/test_gpu_distributed.py tests/test_gpu_exchange_ops.py tests/test_gpu_props.py > $O/tests.log 2>&1 || echo "TESTS FAILED" >> $O/tests.log
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench.json 2> $O/opbench.err
