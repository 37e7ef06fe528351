# Round-3 closing evidence on HEAD: full GPU suite, smoke, default bench, the
# same bench under the kernel trace, op bench
set -e
out=gpurun_out/final6
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
bash tools/gpu_final.sh final6
timeout -k 10 300 python tools/opbench.py --only other_ops > $out/opbench.json 2> $out/opbench.err
