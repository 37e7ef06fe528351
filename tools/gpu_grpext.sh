# ordered BATgroup with extents stored by the write pass / optional histogram:
# group, aggregate and distributed parity tests, then the default bench
set -e
out=gpurun_out/grpext
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_group_sorted.py tests/test_gpu_aggr_sorted.py tests/test_gpu_distributed.py tests/test_gpu_props.py tests/test_gpu_group_str.py tests/test_gpu_ops.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
