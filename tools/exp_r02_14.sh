# A/B on one box: lib vs lib_lw1 (logic launch bounds 1) vs lib_base (HEAD); emulated 8-way share, 1 vs 2 pipelines
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for V in lib lib_lw1 lib_base lib lib_lw1 lib_base; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e14_h_$V.json 2> gpurun_out/e14_h_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e14_h_$V.json'));print('headline $V', d['value'], d['ms_per_step'])"
done
for P in 1 2 1 2; do
  RT_PIPES=$P timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 --emulate 8 --emulate-rank 3 > gpurun_out/e14_e8_$P.json 2> gpurun_out/e14_e8_$P.err
  python3 -c "import json;d=json.load(open('gpurun_out/e14_e8_$P.json'));print('8-way share, pipes $P', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
