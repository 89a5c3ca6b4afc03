# logic kernel occupancy targets after the split: 5 (natural) / 6 / 8 waves without frames, 3 / 4 with
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B="tests/golden/scenes/blend"
for V in lib lib_lw6 lib_lw8 lib lib_lw6 lib_lw8; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e20_h_$V.json 2> gpurun_out/e20_h_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e20_h_$V.json'));print('headline $V', d['value'], d['ms_per_step'])"
done
for V in lib lib_lwf4 lib lib_lwf4; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e20_c4_$V.json 2> gpurun_out/e20_c4_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e20_c4_$V.json'));print('C4 $V', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
bash tools/sweep_env.sh e20 RT_REFILL "40 48 56" --steps 5
bash tools/sweep_env.sh e20 RT_LEAF_MIN "8 16 24" --steps 5
bash tools/sweep_env.sh e20 RT_SLOTS "12582912 16777216 25165824" --steps 5
