# BATgroup assign: nontemporal vs plain loads / stores
set -e
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
for v in base gplain gplainst; do
  if [ $v = base ]; then lib=""; else lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 300 python tools/opbench.py --only other_ops > $O/$v.json 2> $O/$v.err
done
