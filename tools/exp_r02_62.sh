# node / primitive record loads: default vs four aligned 16-B node loads (RT_NODE_ALIGNED) vs
# that plus the primitive record pinned whole (RT_PRIM_ALIGNED); alternating, 3 reps (headline)
# (result: default 4803/4789/4795, node-aligned 4755/4751/4763, +prim pin 4790/4782/4785 Mrays/s; C4 equal.
#  Both defines were removed again after this negative result.)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in lib lib_na lib_nap; do
    RT_LIB_DIR=ray_tracying_amd/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/e60.json 2> gpurun_out/e60.err
    python3 -c "import json;d=json.load(open('gpurun_out/e60.json'));print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
for lib in lib lib_nap; do
  RT_LIB_DIR=ray_tracying_amd/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene tests/golden/scenes/blend/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e60c4.json 2> gpurun_out/e60c4.err
  python3 -c "import json;d=json.load(open('gpurun_out/e60c4.json'));print('C4 $lib', d['value'], d['ms_per_step'])"
done
echo "done $(date +%T)"
