#!/bin/bash
# A/B of environment settings of one build on the GPU box (knob A/B; tools/ab.sh compares builds):
#   bash tools/ab_env.sh REPS "head em8 c5" "A:ENV=VAL,ENV=VAL" "B:" ...
# Every rep runs each workload under each setting in alternation and prints one line per run:
#   <workload> <setting> <Mrays/s> <ms/step> <avg trace launch ms>
set -eo pipefail
REPS=${1:-2}
WLS=${2:-head}
shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B=tests/golden/scenes/blend
args_for() {
  case "$1" in
    head) echo "--steps 10 --warmup 2" ;;
    em8) echo "--steps 20 --warmup 5 --emulate 8 --emulate-rank 7" ;;
    c2) echo "--steps 10 --primary-only --spp-sqrt 1" ;;
    c3) echo "--steps 3 --scene $B/Antialiasing.json" ;;
    c4) echo "--steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4" ;;
    c5) echo "--steps 2 --warmup 1 --res 4096 --spp-sqrt 8" ;;
    *) echo "unknown workload $1" >&2; return 1 ;;
  esac
}
for rep in $(seq 1 "$REPS"); do
  for wl in $WLS; do
    a=$(args_for "$wl")
    for setting in "$@"; do
      name=${setting%%:*}
      kvs=${setting#*:}
      envs=()
      IFS=',' read -ra envs <<< "$kvs"
      env "${envs[@]}" timeout -k 10 300 python3 bench.py --no-cpu-baseline $a \
        > gpurun_out/abe_${wl}_${name}.json 2> gpurun_out/abe_${wl}_${name}.err
      python3 -c "import json;d=json.load(open('gpurun_out/abe_${wl}_${name}.json'));r=d['roofline'];print('$wl', '$name', d['value'], d['ms_per_step'], r['avg_launch_ms'], flush=True)"
    done
  done
done
