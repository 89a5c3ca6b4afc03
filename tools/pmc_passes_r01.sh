#!/bin/bash
# rocprofv3 counter passes over one bench frame (+ the instrumented frame), few counters per
# pass (gfx950 slot limits); used for the round-1 trace-kernel analysis in DESIGN.md.
export TMPDIR=/tmp; mkdir -p gpurun_out
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -k 10 90 rocprofv3 --pmc $set -d gpurun_out/pp$i -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/pp$i.err || { echo "pass $i failed: $set"; exit 1; }
done < "${1:-/dev/stdin}"
