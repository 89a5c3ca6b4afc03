set -e
RT_LIB_DIR=ray_tracying_amd/lib_pt timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pt_head.json 2> gpurun_out/pt_head.err
RT_LIB_DIR=ray_tracying_amd/lib_pt timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --emulate 8 --emulate-rank 7 > gpurun_out/pt_em8.json 2> gpurun_out/pt_em8.err
grep "rt phase" gpurun_out/pt_head.err | tail -n 2 || true
grep "rt phase" gpurun_out/pt_em8.err | tail -n 2 || true
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r04_n_tests.log 2>&1
tail -n 2 gpurun_out/r04_n_tests.log
bash tools/ab.sh "lib lib_prev lib_sel" 2 "head em8 c5"
