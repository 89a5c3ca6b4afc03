#!/bin/bash
# Frames per rt_render_frames call (bench.py --frames-per-call B) on whole frames, alternating,
# REPS reps:  bash tools/fpc_sweep.sh REPS "head:1,4,8 c3:1,4 c2:8,16,32"
export TMPDIR=/tmp; mkdir -p gpurun_out
REPS=${1:-2}; SPEC=${2:-"head:1,2,4"}
S=tests/golden/scenes/blend
args_for() {
  case "$1" in
    head) echo "--steps 24 --warmup 4" ;;
    c2) echo "--steps 64 --warmup 16 --primary-only --spp-sqrt 1" ;;
    c3) echo "--steps 24 --warmup 4 --scene $S/Antialiasing.json" ;;
    *) echo "unknown workload $1" >&2; return 1 ;;
  esac
}
for rep in $(seq 1 "$REPS"); do
  for item in $SPEC; do
    wl=${item%%:*}; bs=${item#*:}
    for b in ${bs//,/ }; do
      timeout -k 10 300 python3 bench.py --no-cpu-baseline $(args_for "$wl") --frames-per-call "$b" \
        > gpurun_out/fpc_${wl}_$b.json 2> gpurun_out/fpc_${wl}_$b.err || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/fpc_${wl}_$b.json'));r=d['roofline'];print('$wl fpc=$b', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['launches_per_step'], flush=True)"
    done
  done
done
