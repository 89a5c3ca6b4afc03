#!/bin/bash
# Parameterised A/B comparison of library builds on the GPU box (replaces the round-2
# one-off tools/exp_r02_*.sh scripts):
#   bash tools/ab.sh "lib lib_base" REPS "head em8 c2 c3 c4 c5" [ENV=VAL ...]
# Builds are directories under ray_tracying_amd/ (make variant V=name VDEFS=...); every rep
# runs each workload on each build in alternation and prints one line per run:
#   <workload> <build> <Mrays/s> <ms/step> <avg trace launch ms> <launches/step>
# Workloads: head (bench.py default, 10 steps), em2/em4/em8 (rank N-1's share of an N-way
# split), c2 (primary only, 1 spp), c3 (Antialiasing), c4 (glossy + soft shadows), c5 (4096^2
# x 64 spp).  Extra ENV=VAL arguments are exported for every run; BENCH_EXTRA="--flag ..." adds
# bench.py arguments to every run.  Knob sweeps are ENV=VAL runs of one build, e.g.
#   bash tools/ab.sh lib 1 "head em8 c5" RT_REFILL=40     (r04: refill / leaf thresholds)
set -eo pipefail
LIBS=${1:?builds}
REPS=${2:-2}
WLS=${3:-head}
shift 3 || true
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp
mkdir -p gpurun_out
B=tests/golden/scenes/blend
args_for() {
  case "$1" in
    head) echo "--steps 10 --warmup 2" ;;
    em2) echo "--steps 20 --warmup 5 --emulate 2 --emulate-rank 1" ;;
    em4) echo "--steps 20 --warmup 5 --emulate 4 --emulate-rank 3" ;;
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
    for lib in $LIBS; do
      RT_LIB_DIR=ray_tracying_amd/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline $a ${BENCH_EXTRA:-} \
        > gpurun_out/ab_${wl}_${lib}.json 2> gpurun_out/ab_${wl}_${lib}.err
      python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_${wl}_${lib}.json'));r=d['roofline'];print('$wl', '$lib', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['launches_per_step'], flush=True)"
    done
  done
done
