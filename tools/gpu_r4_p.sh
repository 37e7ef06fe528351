# BATgroup assign tile 16 Ki vs the 32 Ki default
set -e
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
for v in base gt16384 base2; do
  if [ $v = gt16384 ]; then lib=$PWD/tools/variants/libmgdk_$v.so; else lib=""; fi
  MGDK_LIB=$lib timeout -k 10 300 python tools/opbench.py --only other_ops > $O/$v.json 2> $O/$v.err
done
