#!/bin/bash
# rocprofv3 counter passes over one bench frame (+ the instrumented frame), one pass per line
# of SETFILE (gfx950 per-block counter limits), then a per-kernel summary.
#   bash tools/pmc_passes.sh LABEL SETFILE [bench args...]
set -o pipefail
LABEL=${1:?label}; SETS=${2:?setfile}; shift 2
export TMPDIR=/tmp; mkdir -p gpurun_out
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/${LABEL}_pp$i -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > /dev/null 2> gpurun_out/${LABEL}_pp$i.err || { echo "pass $i failed: $set"; exit 1; }
done < "$SETS"
python3 tools/pmc_summary.py gpurun_out/${LABEL}_pp* > gpurun_out/${LABEL}_pmc_summary.txt
