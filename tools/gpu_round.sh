# Full GPU check used between milestones: parity tests, bench, rocprof stats.
set -e
mkdir -p gpurun_out/round
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/round/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/round/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/round/prof -o run -- python3 bench.py --steps 5 --no-cpu > gpurun_out/round/prof.log 2>&1
timeout -k 10 300 python tools/opbench.py > gpurun_out/round/opbench.json 2> gpurun_out/round/opbench.err
