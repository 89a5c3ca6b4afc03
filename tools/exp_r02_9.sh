# LDS top-of-tree node cache (BFS-prefix node order): parity tests, then bench sweeps of
# (RT_LDS_STACK, RT_LDS_NODES)
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e9_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e9_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e9_gpu_tests.log
for cfg in 16:0 16:128 12:256 8:384 16:0 16:128 12:256 8:384 8:0; do
  S=${cfg%%:*}; N=${cfg##*:}
  RT_LDS_STACK=$S RT_LDS_NODES=$N timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/e9_$S_$N.json 2> gpurun_out/e9_$S_$N.err
  python3 -c "import json;d=json.load(open('gpurun_out/e9_$S_$N.json'));print('stack $S nodes $N', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
echo "done $(date +%T)"
