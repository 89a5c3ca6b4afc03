#!/bin/bash
# C2 (1 spp, primary rays only) at 30 timed frames: auto frames in flight (3 for <= 4M samples) vs 2.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 30 --primary-only --spp-sqrt 1 > gpurun_out/r04_v5_c2_primary_only_bench.json 2> gpurun_out/r04_v5_c2.err
  python3 -c "import json;d=json.load(open('gpurun_out/r04_v5_c2_primary_only_bench.json'));print('c2 auto', d['config']['frames_in_flight'], d['value'], flush=True)"
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 30 --primary-only --spp-sqrt 1 --frames-in-flight 2 > gpurun_out/c2_f2.json 2> gpurun_out/c2_f2.err
  python3 -c "import json;d=json.load(open('gpurun_out/c2_f2.json'));print('c2 F=2', d['value'], flush=True)"
done
