set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "default $(date +%T)"; timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e4_def.json 2> gpurun_out/e4_def.err
python3 -c "import json;d=json.load(open('gpurun_out/e4_def.json'));print('def', d['value'], d['roofline']['avg_launch_ms'])"
echo "pt $(date +%T)"; RT_LIB_DIR=ray_tracying_amd/lib_pt timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e4_pt.json 2> gpurun_out/e4_pt.err
grep "rt phase" gpurun_out/e4_pt.err | tail -3
