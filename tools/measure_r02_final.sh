# Final check of the default build: smoke, GPU parity suite, headline bench, rocprofv3
# kernel-trace stats of the headline bench, C4.  Outputs under gpurun_out/ (label $1).
set -eo pipefail
L=${1:?label}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${L}_smoke.log 2>&1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${L}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${L}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${L}_gpu_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/${L}_bench.json 2> gpurun_out/${L}_bench.err
cat gpurun_out/${L}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${L}_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${L}_kt_bench.json 2> gpurun_out/${L}_kt_bench.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene tests/golden/scenes/blend/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/${L}_c4_glossy_soft_bench.json 2> gpurun_out/${L}_c4.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --scene tests/golden/scenes/blend/Antialiasing.json > gpurun_out/${L}_c3_antialiasing_bench.json 2> gpurun_out/${L}_c3.err
echo "done $(date +%T)"
