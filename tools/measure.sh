# One GPU measurement pass (run through gpurun from the repo root): GPU tests, rocprofv3
# kernel-trace stats of the bench, PMC passes (HBM traffic: FETCH_SIZE, WRITE_SIZE; VALU issue
# and lane utilisation), the default full bench (with the CPU baseline), then the C3 / C4 scene
# benches.  Results land in gpurun_out/$LABEL_*; copy what is judged into profiles/.
set -eo pipefail
LABEL=${1:?label}
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "gpu tests $(date)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/${LABEL}_gpu_tests.log 2>&1
echo "rocprof kernel trace $(date)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${LABEL}_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${LABEL}_kt_bench.json 2> gpurun_out/${LABEL}_kt_bench.err
echo "pmc $(date)"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${LABEL}_pmcF -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${LABEL}_pmcF.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${LABEL}_pmcW -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${LABEL}_pmcW.err
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/${LABEL}_pmcV -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${LABEL}_pmcV.err
python3 tools/pmc_traffic.py --fetch gpurun_out/${LABEL}_pmcF --write gpurun_out/${LABEL}_pmcW --out gpurun_out/${LABEL}_pmc_traffic.json --label "${LABEL}"
python3 tools/pmc_valu.py --dir gpurun_out/${LABEL}_pmcV --out gpurun_out/${LABEL}_pmc_valu.json --label "${LABEL}"
echo "full bench $(date)"
timeout -k 10 600 python3 bench.py --pmc-traffic gpurun_out/${LABEL}_pmc_traffic.json --pmc-valu gpurun_out/${LABEL}_pmc_valu.json > gpurun_out/${LABEL}_bench_full.json 2> gpurun_out/${LABEL}_bench_full.err
echo "C3 / C4 scene benches $(date)"
timeout -k 10 300 python3 bench.py --scene tests/golden/scenes/blend/Antialiasing.json > gpurun_out/${LABEL}_c3.json 2> gpurun_out/${LABEL}_c3.err
timeout -k 10 300 python3 bench.py --scene tests/golden/scenes/blend/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/${LABEL}_c4.json 2> gpurun_out/${LABEL}_c4.err
echo "done $(date)"
