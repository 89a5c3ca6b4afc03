#!/bin/bash
# Kernel-trace profiles (rocprofv3 --kernel-trace --stats) of bench workloads on the current
# build:  bash tools/prof.sh LABEL "head em8 c3 ..."
source tools/gpu_steps.sh
L=${1:?label}
B=tests/golden/scenes/blend
for wl in ${2:-head}; do
  case "$wl" in
    head) a="--steps 3 --warmup 1" ;;
    em8) a="--steps 5 --emulate 8 --emulate-rank 7" ;;
    c2) a="--steps 5 --primary-only --spp-sqrt 1" ;;
    c3) a="--steps 3 --scene $B/Antialiasing.json" ;;
    c4) a="--steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4" ;;
    c5) a="--steps 1 --warmup 1 --res 4096 --spp-sqrt 8" ;;
  esac
  step ${L}_${wl}_kt.log 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${L}_${wl}_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline $a
  f=$(find gpurun_out/${L}_${wl}_kt -name "kt_kernel_stats.csv" | head -1)
  echo "== $wl"; cut -d, -f1-8 "$f" | head -12
done
