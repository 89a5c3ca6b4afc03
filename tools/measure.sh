#!/bin/bash
# One GPU measurement pass (run on the GPU box through gpurun):
#   bash tools/measure.sh LABEL [skip-tests]
# smoke + GPU parity tests; rocprofv3 kernel-trace stats of the headline bench; PMC passes
# (FETCH_SIZE, WRITE_SIZE, the VALU set; one pass each, dispatches serialised by the profiler)
# of the headline frame and of C5 (4096^2 x 64 spp), and the counter-measured VALU microbenchmark; the full headline bench (with the CPU
# baseline) carrying the PMC summaries just measured; the other BASELINE configs (C2, C3,
# C4, C5).  The per-rank shares of split frames: tools/measure_shares.sh.  Everything lands
# in gpurun_out/.
set -eo pipefail
L=${1:?label}
export TMPDIR=/tmp
mkdir -p gpurun_out
B=tests/golden/scenes/blend
if [ "${2:-}" != "skip-tests" ]; then
  echo "smoke $(date +%T)"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${L}_smoke.log 2>&1
  echo "gpu tests $(date +%T)"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/${L}_gpu_tests.log 2>&1
  tail -1 gpurun_out/${L}_gpu_tests.log
fi
echo "kernel trace $(date +%T)"
# (the headline renders 8 frames per rt_render_frames call: 16 timed + 8 warmup frames make every
# profiled traversal launch, the workspace-sizing call's too, an 8-frame launch like the bench's)
HP="--steps 8 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${L}_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 16 --warmup 8 > gpurun_out/${L}_kt_bench.json 2> gpurun_out/${L}_kt_bench.err
echo "pmc $(date +%T)"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${L}_pmcF -o p --output-format csv -- python3 bench.py --no-cpu-baseline $HP > /dev/null 2> gpurun_out/${L}_pmcF.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${L}_pmcW -o p --output-format csv -- python3 bench.py --no-cpu-baseline $HP > /dev/null 2> gpurun_out/${L}_pmcW.err
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/${L}_pmcV -o p --output-format csv -- python3 bench.py --no-cpu-baseline $HP > /dev/null 2> gpurun_out/${L}_pmcV.err
[ -x tools/bin/ubench_valu ] || make ubench
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${L}_ubench_pmc -o p --output-format csv -- tools/bin/ubench_valu > gpurun_out/${L}_ubench_src.txt 2>&1
python3 tools/pmc_traffic.py --fetch gpurun_out/${L}_pmcF --write gpurun_out/${L}_pmcW --kernel "trace_refill_kernel<false" --out gpurun_out/${L}_pmc_traffic.json --label "$L" --frames 8 > /dev/null
python3 tools/pmc_valu.py --dir gpurun_out/${L}_pmcV --out gpurun_out/${L}_pmc_valu.json --label "$L" > /dev/null
echo "pmc c5 $(date +%T)"
C5="--res 4096 --spp-sqrt 8"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${L}_c5_pmcF -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $C5 > /dev/null 2> gpurun_out/${L}_c5_pmcF.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${L}_c5_pmcW -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $C5 > /dev/null 2> gpurun_out/${L}_c5_pmcW.err
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/${L}_c5_pmcV -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $C5 > /dev/null 2> gpurun_out/${L}_c5_pmcV.err
python3 tools/pmc_traffic.py --fetch gpurun_out/${L}_c5_pmcF --write gpurun_out/${L}_c5_pmcW --kernel "trace_refill_kernel<false" --out gpurun_out/${L}_c5_pmc_traffic.json --label "${L} C5" > /dev/null
python3 tools/pmc_valu.py --dir gpurun_out/${L}_c5_pmcV --out gpurun_out/${L}_c5_pmc_valu.json --label "${L} C5" > /dev/null
python3 tools/pmc_ubench.py --dir gpurun_out/${L}_ubench_pmc --out gpurun_out/${L}_ubench_valu_pmc.json --label "$L" > gpurun_out/${L}_ubench_valu_pmc.txt
echo "bench $(date +%T)"
timeout -k 10 600 python3 bench.py --steps 24 --warmup 8 --pmc-traffic gpurun_out/${L}_pmc_traffic.json --pmc-valu gpurun_out/${L}_pmc_valu.json --ubench gpurun_out/${L}_ubench_valu_pmc.json > gpurun_out/${L}_bench.json 2> gpurun_out/${L}_bench.err
cat gpurun_out/${L}_bench.json
echo "issue-mix microbenchmark $(date +%T)"
timeout -k 10 200 tools/bin/ubench_mix > gpurun_out/${L}_ubench_mix.txt 2>&1
echo "configs $(date +%T)"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 128 --warmup 64 --primary-only --spp-sqrt 1 > gpurun_out/${L}_c2_primary_only_bench.json 2> gpurun_out/${L}_c2.err
timeout -k 10 300 python3 bench.py --steps 16 --warmup 8 --scene $B/Antialiasing.json > gpurun_out/${L}_c3_antialiasing_bench.json 2> gpurun_out/${L}_c3.err
timeout -k 10 300 python3 bench.py --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/${L}_c4_glossy_soft_bench.json 2> gpurun_out/${L}_c4.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --res 4096 --spp-sqrt 8 --pmc-traffic gpurun_out/${L}_c5_pmc_traffic.json --pmc-valu gpurun_out/${L}_c5_pmc_valu.json --ubench gpurun_out/${L}_ubench_valu_pmc.json > gpurun_out/${L}_c5_4096_64spp_1gpu_bench.json 2> gpurun_out/${L}_c5.err
echo "done $(date +%T)"
