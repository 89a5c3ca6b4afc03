#!/bin/bash
# Whole frames (headline, C5) with two frames in flight, with and without the deferred call's
# one-block-per-CU reserve (RT_DEFER_BPC), against one frame in flight (one box).
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "1 1" "2 1" "2 0"; do
    set -- $cfg
    RT_DEFER_BPC=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --frames-in-flight $1 > gpurun_out/fif2_head_$1_$2.json 2> gpurun_out/fif2_head_$1_$2.err
    python3 -c "import json;d=json.load(open('gpurun_out/fif2_head_$1_$2.json'));print('head F=$1 reserve=$2', d['value'], flush=True)"
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --primary-only --spp-sqrt 1 > gpurun_out/fif2_c2_auto.json 2> gpurun_out/fif2_c2_auto.err
python3 -c "import json;d=json.load(open('gpurun_out/fif2_c2_auto.json'));print('c2 auto', d['config']['frames_in_flight'], d['value'], flush=True)"
