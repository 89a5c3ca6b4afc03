#!/bin/bash
# Multi-GPU prediction from one GPU (run on the GPU box through gpurun):
#   bash tools/measure_shares.sh LABEL [DEAL] [SPLITS] [STEPS]
# Every rank's share of the N-way splits (SPLITS, default "2 4 8") of the headline frame, and
# of the 8-way split of C5 (4096^2 x 64 spp), each rendered alone on this GPU (bench.py
# --emulate N --emulate-rank r --deal DEAL, default lattice); the whole frames for
# reference (BENCH_EXTRA="..." adds bench.py arguments to every run); then the RCCL gather's fixed cost and payload estimate (tools/gather_cost.py) --
# tools/shares_summary.py turns it into the slowest-rank prediction.
source tools/gpu_steps.sh
L=${1:?label}
DEAL=${2:-lattice}
SPLITS=${3:-2 4 8}
STEPS=${4:-20}
D=gpurun_out/${L}_shares
mkdir -p $D
step ${L}_shares_head_whole.log 300 python3 bench.py --no-cpu-baseline --steps $STEPS --warmup 5 ${BENCH_EXTRA:-}
cp gpurun_out/${L}_shares_head_whole.log $D/head_whole.log; grep "^{" $D/head_whole.log > $D/head_whole.json
for N in $SPLITS; do
  for r in $(seq 0 $((N - 1))); do
    step ${L}_shares_head_${N}_${r}.log 300 python3 bench.py --no-cpu-baseline --steps $STEPS --warmup 5 --emulate $N --emulate-rank $r --deal $DEAL ${BENCH_EXTRA:-}
    grep "^{" gpurun_out/${L}_shares_head_${N}_${r}.log > $D/head_${N}_${r}.json
    echo "head $N-way rank $r $(python3 -c "import json;print(json.load(open('$D/head_${N}_${r}.json'))['value'])")"
  done
done
if [ -n "${C5:-}" ]; then
  step ${L}_shares_c5_whole.log 400 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 ${BENCH_EXTRA:-}
  grep "^{" gpurun_out/${L}_shares_c5_whole.log > $D/c5_whole.json
  for r in $(seq 0 7); do
    step ${L}_shares_c5_8_${r}.log 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 --emulate 8 --emulate-rank $r --deal $DEAL ${BENCH_EXTRA:-}
    grep "^{" gpurun_out/${L}_shares_c5_8_${r}.log > $D/c5_8_${r}.json
    echo "c5 8-way rank $r $(python3 -c "import json;print(json.load(open('$D/c5_8_${r}.json'))['value'])")"
  done
fi
step ${L}_gather.log 120 python3 tools/gather_cost.py $D/gather_cost.json
python3 tools/shares_summary.py --dir $D --out gpurun_out/${L}_shares.json --label "$L ($DEAL deal)"
