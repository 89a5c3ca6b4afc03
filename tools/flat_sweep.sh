#!/bin/bash
# RT_FLAT_PRIMS sweep on the exported Blender scenes of a few to tens of primitives (r06):
#   bash tools/flat_sweep.sh "Distributed Test1 ..." "8 16 32" REPS
source tools/gpu_steps.sh
SCENES=${1:-"Distributed Test1"}; VALS=${2:-"8 32"}; REPS=${3:-1}
for rep in $(seq 1 "$REPS"); do
  for sc in $SCENES; do
    for v in $VALS; do
      RT_FLAT_PRIMS=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 8 --warmup 2 \
        --scene tests/golden/scenes/blend/$sc.json > gpurun_out/fs.json 2> gpurun_out/fs.err || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/fs.json'));print('$sc flat_prims $v', d['value'], d['ms_per_step'], d['config']['pipeline'][:40], flush=True)"
    done
  done
done
