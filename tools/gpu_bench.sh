# Bench + same-lease rocprof kernel trace of the same command (profiles/rNN).
set -e
out=gpurun_out/${1:-bench}
mkdir -p $out
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --no-cpu > $out/prof_bench.json 2> $out/prof.err
