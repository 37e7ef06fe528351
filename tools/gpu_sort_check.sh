# sort parity tests + 100M int32 sort timing + its kernel trace; output under gpurun_out/s1
set -e
out=gpurun_out/s1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_join_sort_window.py tests/test_gpu_str_sort.py tests/test_gpu_firstn.py -k "sort or unique or firstn" -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python tools/opbench.py --only other_ops > $out/ops.json 2> $out/ops.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/opbench.py --only other_ops > $out/trace.json 2> $out/trace.err
