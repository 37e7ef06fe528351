# round-4 evidence: full GPU parity suite, smoke, the default bench line, a
# kernel-trace profile of the bench, FETCH_SIZE / WRITE_SIZE passes for the
# Q6 / Q1 kernels, the op timings
set -e
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
rc=0
timeout -k 10 1100 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --no-cpu --no-parity > $O/prof.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 bench.py --no-dist-legs --no-op-legs --no-cpu --no-parity --steps 3 --warmup 1 > $O/pmc_f.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 bench.py --no-dist-legs --no-op-legs --no-cpu --no-parity --steps 3 --warmup 1 > $O/pmc_w.log 2>&1
timeout -k 10 400 python tools/opbench.py > $O/opbench.json 2> $O/opbench.err
