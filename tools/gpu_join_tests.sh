# Join parity tests + SF10 hash-join opbench (gt path and, for A/B, the
# radix-partitioned path) + kernel trace; output under gpurun_out/j1
set -e
out=gpurun_out/j1
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_join_algo.py tests/test_gpu_join_sort_window.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 120 python tools/opbench.py --only config3_hashjoin_sf10 > $out/gt.json 2> $out/gt.err
timeout -k 10 200 python tools/join_sweep.py > $out/sweep.json 2> $out/sweep.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/opbench.py --only config3_hashjoin_sf10 > $out/trace.json 2> $out/trace.err
