set -e
mkdir -p gpurun_out/r3t
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base t32768 t131072 t262144; do
  lib=""; if [ $v != base ]; then lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t/$v -o run -- python3 tools/opbench.py --only other_ops > gpurun_out/r3t/$v.json 2> gpurun_out/r3t/$v.err
done
