# group / aggregate / props parity + group timing + Q1 plan breakdown; output gpurun_out/g1
set -e
out=gpurun_out/g1
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_props.py tests/test_gpu_distributed.py tests/test_gpu_firstn.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python tools/opbench.py --only other_ops > $out/ops.json 2> $out/ops.err
timeout -k 10 300 python tools/q1_breakdown.py > $out/q1.json 2>&1
