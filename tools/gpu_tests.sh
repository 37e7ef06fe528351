# GPU parity tests; args: pytest selection (default: the whole -m gpu suite)
set -e
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t/tests.log 2>&1
