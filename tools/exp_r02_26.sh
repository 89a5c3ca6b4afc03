# BVH2 -> BVH4 collapse: SAH-optimal dynamic programming (default) vs greedy largest-area
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e26_gpu_tests.log 2>&1 || { tail -30 gpurun_out/e26_gpu_tests.log; exit 1; }
tail -1 gpurun_out/e26_gpu_tests.log
B="tests/golden/scenes/blend"
bash tools/sweep_env.sh e26a RT_COLLAPSE "dp greedy" --steps 5
bash tools/sweep_env.sh e26b RT_COLLAPSE "dp greedy" --steps 5
bash tools/sweep_env.sh e26c3 RT_COLLAPSE "dp greedy" --steps 3 --scene $B/Antialiasing.json
bash tools/sweep_env.sh e26c4 RT_COLLAPSE "dp greedy" --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4
grep -h "instrumented" gpurun_out/e26a_RT_COLLAPSE_*.err
echo "done $(date +%T)"
