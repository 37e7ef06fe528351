# round-4 batch: group / window / str parity + op timings, then the sort tile
# shape sweep (16384- and 12288-key tiles for 4-byte keys)
set -e
bash tools/gpu_r4_c.sh
bash tools/ssweep.sh w8r32 w4r64 w4r48
