# A/B on one box: lib (working tree) vs lib_base (HEAD): headline and C4; C4 with one pipeline
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B="tests/golden/scenes/blend"
for V in lib lib_base lib lib_base; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e13_h_$V.json 2> gpurun_out/e13_h_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e13_h_$V.json'));print('headline $V', d['value'], d['ms_per_step'])"
done
for V in lib lib_base; do
  for P in 1 2; do
    RT_PIPES=$P RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e13_c4_$V$P.json 2> gpurun_out/e13_c4_$V$P.err
    python3 -c "import json;d=json.load(open('gpurun_out/e13_c4_$V$P.json'));print('C4 $V pipes $P', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'])"
  done
done
echo "done $(date +%T)"
