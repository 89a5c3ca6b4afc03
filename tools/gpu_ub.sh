set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=r03_v9
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${L}_ubench_pmc -o p --output-format csv -- tools/bin/ubench_valu > gpurun_out/${L}_ubench_src.txt 2>&1 || exit 1
python3 tools/pmc_ubench.py --dir gpurun_out/${L}_ubench_pmc --out gpurun_out/${L}_ubench_valu_pmc.json --label "$L" > gpurun_out/${L}_ubench_valu_pmc.txt
grep "add_u32" gpurun_out/${L}_ubench_valu_pmc.txt; tail -1 gpurun_out/${L}_ubench_valu_pmc.txt
