# r05: kernel breakdown of C3 (one-pass, transformed shapes, fused lights) and C4 (step pipeline)
source tools/gpu_steps.sh
B=tests/golden/scenes/blend
step r05s_kt_c3.log 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05s_kt_c3 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --scene $B/Antialiasing.json
step r05s_kt_c4.log 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05s_kt_c4 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --scene $B/glossy_reflection.json --light-radius 1.0 --light-samples 4
