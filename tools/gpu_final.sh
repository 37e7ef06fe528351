# Round-end evidence: smoke, default bench, same-command rocprof kernel stats.
set -e
out=gpurun_out/${1:-final}
mkdir -p $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py > $out/prof_bench.json 2> $out/prof.err
