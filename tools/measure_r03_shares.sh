#!/bin/bash
# Multi-GPU prediction from one GPU (run on the GPU box through gpurun):
#   bash tools/measure_r03_shares.sh LABEL
# Every rank's share of the 2-, 4- and 8-way lattice splits of the headline frame, and of the
# 8-way split of C5 (4096^2 x 64 spp), each rendered alone on this GPU (bench.py --emulate N
# --emulate-rank r); the whole frames for reference; then the device-to-device copy time of
# one rank's packed tiles (the gather's payload) -- tools/shares_summary.py turns it into the
# slowest-rank prediction.
set -eo pipefail
L=${1:?label}
export TMPDIR=/tmp
mkdir -p gpurun_out/${L}_shares
D=gpurun_out/${L}_shares
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 > $D/head_whole.json 2> $D/head_whole.err
for N in 2 4 8; do
  for r in $(seq 0 $((N - 1))); do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --emulate $N --emulate-rank $r > $D/head_${N}_${r}.json 2> $D/head_${N}_${r}.err
    echo "head $N-way rank $r $(python3 -c "import json;print(json.load(open('$D/head_${N}_${r}.json'))['value'])")"
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 > $D/c5_whole.json 2> $D/c5_whole.err
for r in $(seq 0 7); do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 --emulate 8 --emulate-rank $r > $D/c5_8_${r}.json 2> $D/c5_8_${r}.err
  echo "c5 8-way rank $r $(python3 -c "import json;print(json.load(open('$D/c5_8_${r}.json'))['value'])")"
done
timeout -k 10 120 python3 tools/gather_cost.py $D/gather_cost.json > /dev/null
python3 tools/shares_summary.py --dir $D --out gpurun_out/${L}_shares.json --label $L
