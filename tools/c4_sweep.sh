#!/bin/bash
# C4 sweep of the inline-query logic instance (r06): builds x slot counts, alternating
source tools/gpu_steps.sh
for rep in 1 2; do
  for lib in lib_i4; do
    for sl in 8388608 16777216 25165824 33554432; do
      RT_LIB_DIR=ray_tracying_amd/$lib RT_SLOTS=$sl timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 \
        --scene tests/golden/scenes/blend/glossy_reflection.json --light-radius 1.0 --light-samples 4 \
        > gpurun_out/c4s.json 2> gpurun_out/c4s.err || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/c4s.json'));r=d['roofline'];print('c4 $lib slots $sl', d['value'], d['ms_per_step'], r['launches_per_step'], flush=True)"
    done
  done
done
