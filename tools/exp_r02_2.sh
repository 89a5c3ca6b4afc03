set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e2_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e2_gpu_tests.log; exit 1; }
tail -2 gpurun_out/e2_gpu_tests.log
for v in bvh8 bvh4; do
  echo "$v $(date +%T)"
  if [ $v = bvh4 ]; then export RT_LIB_DIR=ray_tracying_amd/lib_bvh4; else unset RT_LIB_DIR; fi
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e2_$v.json 2> gpurun_out/e2_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/e2_$v.json'));print('$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['l2']['alg_bytes_per_ray'])"
done
