set -e
mkdir -p gpurun_out/pmcq6
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcq6/f -o run -- python3 bench.py --no-q1 --no-dist-legs --no-cpu --steps 3 --warmup 1 > gpurun_out/pmcq6/f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcq6/w -o run -- python3 bench.py --no-q1 --no-dist-legs --no-cpu --steps 3 --warmup 1 > gpurun_out/pmcq6/w.log 2>&1
