#!/bin/bash
# C3 (Antialiasing.blend, 1024^2 x 100 spp; 28 % of its frame outside the traversal) with one
# and two frames in flight (one box).
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B=tests/golden/scenes/blend
for rep in 1 2; do
  for F in 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --scene $B/Antialiasing.json --frames-in-flight $F > gpurun_out/c3f_$F.json 2> gpurun_out/c3f_$F.err
    python3 -c "import json;d=json.load(open('gpurun_out/c3f_$F.json'));print('c3 F=$F', d['value'], flush=True)"
  done
done
