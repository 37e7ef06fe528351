# fused ordered group sums + group prefix: parity, then the bench line (config-4 leg) and the op bench group row
set -e
export TMPDIR=/tmp
O=gpurun_out/gs
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group_sums.py tests/test_gpu_distributed.py tests/test_gpu_aggr_sorted.py tests/test_gpu_group_sorted.py tests/test_gpu_group_str.py tests/test_gpu_ops.py tests/test_gpu_props.py -k "group or Group or sums or dist or aggr" > $O/tests.log 2>&1 || { echo "TESTS FAILED" >> $O/tests.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python tools/opbench.py --only other_ops > $O/opbench.json 2>&1
