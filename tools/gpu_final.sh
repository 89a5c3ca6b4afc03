set -o pipefail
bash tools/measure_r03.sh r03_v8 || exit 1
bash tools/measure_r03_shares.sh r03_v8 || exit 1
