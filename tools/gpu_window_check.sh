# window-bounds parity + config-5 timing with the 32-bit-key tiles on and off; output gpurun_out/w6
set -e
out=gpurun_out/w6
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_join_sort_window.py tests/test_gpu_analytic.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python tools/opbench.py --only config5 > $out/k32.json 2> $out/k32.err
MGDK_WIN_K32=0 timeout -k 10 200 python tools/opbench.py --only config5 > $out/k64.json 2> $out/k64.err
