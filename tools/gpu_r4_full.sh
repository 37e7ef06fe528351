# full GPU parity suite, then the default bench line
set -e
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || echo "TESTS FAILED" >> $O/tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
