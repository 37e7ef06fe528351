# A/B of a join knob (env var $1, values $2 $3) at SF10 + join tests under the first value
set -e
out=gpurun_out/jd
mkdir -p $out
env $1=$2 timeout -k 10 300 python -u -m pytest tests/test_gpu_join_sort_window.py -k join -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
for v in $2 $3; do
env $1=$v timeout -k 10 120 python tools/opbench.py --only config3_hashjoin_sf10 > $out/v$v.json 2> $out/v$v.err
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/opbench.py --only config3_hashjoin_sf10 > $out/trace.json 2> $out/trace.err
