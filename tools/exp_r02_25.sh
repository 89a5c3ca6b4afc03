# AMDGPU machine-scheduler strategy A/B: default vs max-ilp vs latency-biased (metric bias 0)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B="tests/golden/scenes/blend"
for V in lib lib_ilp lib_bias0 lib lib_ilp lib_bias0; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e25_h_$V.json 2> gpurun_out/e25_h_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e25_h_$V.json'));print('headline $V', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
for V in lib lib_ilp lib_bias0; do
  RT_LIB_DIR=ray_tracying_amd/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e25_c4_$V.json 2> gpurun_out/e25_c4_$V.err
  python3 -c "import json;d=json.load(open('gpurun_out/e25_c4_$V.json'));print('C4 $V', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
