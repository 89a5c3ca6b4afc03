set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/kt_bench.json 2> gpurun_out/kt_bench.err
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/pmcF.err
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2> gpurun_out/pmcW.err
python3 tools/pmc_traffic.py --fetch gpurun_out/pmcF --write gpurun_out/pmcW --out gpurun_out/pmc_traffic.json --label "${RT_LABEL:-r01}"
cp gpurun_out/pmc_traffic.json profiles/r01_pmc_traffic.json
echo "full bench start $(date)"
timeout -k 10 600 python3 bench.py > gpurun_out/b_full.json 2> gpurun_out/b_full.err
echo "done $(date)"
