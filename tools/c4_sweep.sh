#!/bin/bash
# C4 A/B of the inline-query logic builds (r06), alternating: bash tools/c4_sweep.sh "lib lib_x" REPS [ENV=VAL ...]
source tools/gpu_steps.sh
LIBS=${1:-lib}; REPS=${2:-2}; shift 2 || true
for kv in "$@"; do export "$kv"; done
for rep in $(seq 1 "$REPS"); do
  for lib in $LIBS; do
    RT_LIB_DIR=ray_tracying_amd/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 \
      --scene tests/golden/scenes/blend/glossy_reflection.json --light-radius 1.0 --light-samples 4 \
      > gpurun_out/c4s.json 2> gpurun_out/c4s.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c4s.json'));r=d['roofline'];print('c4 $lib ${RT_SLOTS:-}', d['value'], d['ms_per_step'], r['launches_per_step'], flush=True)"
  done
done
