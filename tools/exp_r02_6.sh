set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e6_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e6_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e6_gpu_tests.log
for up in -1 0 1 2 3; do
  RT_SHADOW_UP=$up timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/e6_up$up.json 2> gpurun_out/e6_up$up.err
  python3 -c "import json;d=json.load(open('gpurun_out/e6_up$up.json'));print('up $up', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['l2']['alg_bytes_per_ray'])"
done
RT_SHADOW_UP=2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --emulate 8 --emulate-rank 3 > gpurun_out/e6_e8.json 2> gpurun_out/e6_e8.err
python3 -c "import json;d=json.load(open('gpurun_out/e6_e8.json'));print('e8 up2', d['value'])"
