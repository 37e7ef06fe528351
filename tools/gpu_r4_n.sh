# BATgroup assign tile size: 32 Ki / 64 Ki (default) / 128 Ki rows per workgroup
set -e
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
for v in base gt32768 gt131072; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 300 python tools/opbench.py --only other_ops > $O/$v.json 2> $O/$v.err
done
