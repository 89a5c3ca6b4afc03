# L1/L2 hit rates and request latency of trace_refill_kernel: headline frame vs the 8-way share
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
sed -n '1p;4p' tools/pmc_sets_trace.txt > gpurun_out/e32_sets.txt
bash tools/pmc_passes.sh e32_full gpurun_out/e32_sets.txt || exit 1
bash tools/pmc_passes.sh e32_share gpurun_out/e32_sets.txt --emulate 8 --emulate-rank 7 || exit 1
echo "done $(date +%T)"
