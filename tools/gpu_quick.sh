# Targeted GPU tests: pass test paths / -k expressions as arguments.
set -e
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/quick/tests.log 2>&1
