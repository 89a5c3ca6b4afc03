# One GPU measurement pass (run through gpurun from the repo root): GPU tests, rocprofv3
# kernel-trace stats of the bench, the two PMC traffic passes, then the default full bench
# (with the CPU baseline).  Results land in gpurun_out/$LABEL_*; copy what is judged into profiles/.
set -eo pipefail
LABEL=${1:?label}
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "gpu tests $(date)"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${LABEL}_gpu_tests.log 2>&1
echo "rocprof kernel trace $(date)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${LABEL}_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${LABEL}_kt_bench.json 2> gpurun_out/${LABEL}_kt_bench.err
echo "pmc $(date)"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${LABEL}_pmcF -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${LABEL}_pmcF.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${LABEL}_pmcW -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${LABEL}_pmcW.err
python3 tools/pmc_traffic.py --fetch gpurun_out/${LABEL}_pmcF --write gpurun_out/${LABEL}_pmcW --out gpurun_out/${LABEL}_pmc_traffic.json --label "${LABEL}"
echo "full bench $(date)"
timeout -k 10 600 python3 bench.py --pmc-traffic gpurun_out/${LABEL}_pmc_traffic.json > gpurun_out/${LABEL}_bench_full.json 2> gpurun_out/${LABEL}_bench_full.err
echo "done $(date)"
