set -e
mkdir -p gpurun_out/r3r
for v in base cnt base cnt; do
  lib=""; if [ $v != base ]; then lib=$PWD/tools/variants/libmgdk_$v.so; fi
  MGDK_LIB=$lib timeout -k 10 200 python tools/q1_breakdown.py --reps 3 >> gpurun_out/r3r/$v.json 2>> gpurun_out/r3r/$v.err
done
