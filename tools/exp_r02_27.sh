# trace work-fetch shards for the small C2 launch (1M queries) and the headline
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/sweep_env.sh e27c2 RT_FETCH_SHARDS "8 32 128 256" --steps 10 --primary-only --spp-sqrt 1
bash tools/sweep_env.sh e27h RT_FETCH_SHARDS "8 32 128" --steps 5
echo "done $(date +%T)"
