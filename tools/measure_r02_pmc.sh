# PMC passes of the headline workload on the current build (one counter set per pass), summarised
# for bench.py's roofline block; then the headline bench carrying them.  Label $1.
set -eo pipefail
L=${1:?label}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${L}_pmcF -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${L}_pmcF.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${L}_pmcW -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${L}_pmcW.err
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/${L}_pmcV -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/${L}_pmcV.err
python3 tools/pmc_traffic.py --fetch gpurun_out/${L}_pmcF --write gpurun_out/${L}_pmcW --kernel "trace_refill_kernel<false" --out gpurun_out/${L}_pmc_traffic.json --label "$L" > /dev/null
python3 tools/pmc_valu.py --dir gpurun_out/${L}_pmcV --out gpurun_out/${L}_pmc_valu.json --label "$L" > /dev/null
python3 tools/pmc_valu.py --dir gpurun_out/${L}_pmcV --kernel "logic_kernel" --out gpurun_out/${L}_pmc_valu_logic.json --label "$L" > /dev/null || true
rm -rf gpurun_out/${L}_pmcF gpurun_out/${L}_pmcW gpurun_out/${L}_pmcV
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --pmc-traffic gpurun_out/${L}_pmc_traffic.json --pmc-valu gpurun_out/${L}_pmc_valu.json > gpurun_out/${L}_bench_pmc.json 2> gpurun_out/${L}_bench_pmc.err
cat gpurun_out/${L}_bench_pmc.json
echo "done $(date +%T)"
