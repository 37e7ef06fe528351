set -e
mkdir -p gpurun_out/r3q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base u16ns u8ns u32ns; do
  lib=""; envs=""
  if [ $v != base ]; then lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3q/$v -o run -- python3 tools/run_gsorted.py > gpurun_out/r3q/$v.log 2>&1
done
