#!/bin/bash
# Frames in flight for small calls (one box): C2 (1.05M samples) and one rank's eighth at F = 1..4.
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for F in 2 3 4; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --primary-only --spp-sqrt 1 --frames-in-flight $F > gpurun_out/fif_c2_$F.json 2> gpurun_out/fif_c2_$F.err
    python3 -c "import json;d=json.load(open('gpurun_out/fif_c2_$F.json'));print('c2 F=$F', d['value'], flush=True)"
  done
  for F in 2 3; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --emulate 8 --emulate-rank 7 --frames-in-flight $F > gpurun_out/fif_em8_$F.json 2> gpurun_out/fif_em8_$F.err
    python3 -c "import json;d=json.load(open('gpurun_out/fif_em8_$F.json'));print('em8 F=$F', d['value'], flush=True)"
  done
done
