#!/bin/bash
# A/B sweep of one environment knob over the default bench (diagnostic):
#   bash tools/sweep_env.sh LABEL VAR "v1 v2 ..." [bench args...]
set -o pipefail
LABEL=${1:?}; VAR=${2:?}; VALS=${3:?}; shift 3
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in $VALS; do
  env "$VAR=$v" timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/${LABEL}_${VAR}_$v.json 2> gpurun_out/${LABEL}_${VAR}_$v.err || { echo "FAILED $VAR=$v"; tail -5 gpurun_out/${LABEL}_${VAR}_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step', r['avg_launch_ms'], 'ms/trace launch', r['launches_per_step'], 'launches')" gpurun_out/${LABEL}_${VAR}_$v.json "$VAR=$v"
done
