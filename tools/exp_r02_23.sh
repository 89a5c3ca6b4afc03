# one rank's eighth of the headline frame: slots in flight and pipelines re-swept after the logic split
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/sweep_env.sh e23 RT_SLOTS "16777216 8388608 6553600 4194304" --steps 10 --emulate 8 --emulate-rank 7
bash tools/sweep_env.sh e23 RT_PIPES "1 2" --steps 10 --emulate 8 --emulate-rank 7
RT_PIPES=2 bash tools/sweep_env.sh e23p RT_SLOTS "8388608 6553600" --steps 10 --emulate 8 --emulate-rank 7
echo "done $(date +%T)"
