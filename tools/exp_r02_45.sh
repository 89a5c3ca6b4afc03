# C3 / C4 after the host-loop trim, with per-kernel totals for C4
set -eo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
B=tests/golden/scenes/blend
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --scene $B/Antialiasing.json > gpurun_out/e45_c3.json 2> gpurun_out/e45_c3.err
python3 -c "import json;d=json.load(open('gpurun_out/e45_c3.json'));print('C3', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'], d['roofline']['launches_per_step'])"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > gpurun_out/e45_c4.json 2> gpurun_out/e45_c4.err
python3 -c "import json;d=json.load(open('gpurun_out/e45_c4.json'));print('C4', d['value'], d['ms_per_step'], d['roofline']['trace_share_of_step'], d['roofline']['launches_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e45_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4 > /dev/null 2> gpurun_out/e45_kt.err
cut -d, -f1-5 gpurun_out/e45_kt/*kernel_stats.csv | head -12
python3 tools/timeline.py gpurun_out/e45_kt 30 > gpurun_out/e45_timeline.txt
echo "done $(date +%T)"
