set -e
mkdir -p gpurun_out/r3j
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base nt fr12 ntfr12; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3j/$v -o run -- python3 tools/run_window.py 1000000000 3 > gpurun_out/r3j/$v.log 2>&1
done
