set -e
mkdir -p gpurun_out/r3o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3o/prof -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r3o/bench.json 2> gpurun_out/r3o/bench.err
