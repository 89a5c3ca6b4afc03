#!/bin/bash
# Knob re-sweep after the spill work (one box): refill / leaf thresholds and a seventh wave.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # label env... ; prints label workload value
  local lab=$1; shift
  for wl in head em8 c5; do
    case $wl in
      head) a="--steps 10 --warmup 2" ;;
      em8) a="--steps 10 --emulate 8 --emulate-rank 7" ;;
      c5) a="--steps 2 --warmup 1 --res 4096 --spp-sqrt 8" ;;
    esac
    env "$@" timeout -k 10 300 python3 bench.py --no-cpu-baseline $a > gpurun_out/sw_${lab}_${wl}.json 2> gpurun_out/sw_${lab}_${wl}.err
    python3 -c "import json;d=json.load(open('gpurun_out/sw_${lab}_${wl}.json'));print('$lab', '$wl', d['value'], flush=True)"
  done
}
run base RT_X=0
run refill40 RT_REFILL=40
run refill56 RT_REFILL=56
run leaf16 RT_LEAF_MIN=16
run leaf32 RT_LEAF_MIN=32
run w7 RT_LIB_DIR=ray_tracying_amd/lib_w7 RT_LDS_STACK=10
run base2 RT_X=0
