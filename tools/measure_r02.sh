#!/bin/bash
# One GPU measurement pass (run on the GPU box through gpurun):
#   bash tools/measure_r02.sh LABEL [skip-tests]
# smoke + GPU parity tests, rocprofv3 kernel-trace stats of the headline bench, PMC passes
# (FETCH_SIZE, WRITE_SIZE, VALU set; one pass each), then the full bench (with the CPU
# baseline) carrying the PMC summaries just measured.  Everything lands in gpurun_out/.
set -eo pipefail
L=${1:?label}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${2:-}" != "skip-tests" ]; then
  echo "smoke $(date +%T)"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${L}_smoke.log 2>&1
  echo "gpu tests $(date +%T)"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${L}_gpu_tests.log 2>&1
fi
echo "kernel trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${L}_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${L}_kt_bench.json 2> gpurun_out/${L}_kt_bench.err
echo "pmc $(date +%T)"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${L}_pmcF -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${L}_pmcF.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${L}_pmcW -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${L}_pmcW.err
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/${L}_pmcV -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${L}_pmcV.err
python3 tools/pmc_traffic.py --fetch gpurun_out/${L}_pmcF --write gpurun_out/${L}_pmcW --kernel "trace_refill_kernel<false" --out gpurun_out/${L}_pmc_traffic.json --label "$L" > /dev/null
python3 tools/pmc_valu.py --dir gpurun_out/${L}_pmcV --out gpurun_out/${L}_pmc_valu.json --label "$L" > /dev/null
python3 tools/pmc_valu.py --dir gpurun_out/${L}_pmcV --kernel "logic_kernel" --out gpurun_out/${L}_pmc_valu_logic.json --label "$L" > /dev/null || true
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py --pmc-traffic gpurun_out/${L}_pmc_traffic.json --pmc-valu gpurun_out/${L}_pmc_valu.json > gpurun_out/${L}_bench.json 2> gpurun_out/${L}_bench.err
echo "done $(date +%T)"
