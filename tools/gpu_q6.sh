# Q6 parity tests + bench (same lease) + rocprof kernel trace + PMC passes
# (FETCH_SIZE, WRITE_SIZE in separate runs) of the bench; output gpurun_out/q6b
set -e
out=gpurun_out/q6b
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "q6 or q1" -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --no-cpu > $out/prof_bench.json 2> $out/prof.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --no-cpu --no-q1 --steps 3 --warmup 1 > $out/f.json 2> $out/f.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --no-cpu --no-q1 --steps 3 --warmup 1 > $out/w.json 2> $out/w.err
