# r05: where one rank's eighth (8-way share, two frames in flight) spends the time beyond
# whole-frame / 8: kernel timeline (rocprofv3 kernel trace) and the exit-timing build's queue
# exhaustion / wave exit times per call, at two frames in flight and at one
source tools/gpu_steps.sh
step r05q_kt_em8.log 200 rocprofv3 --kernel-trace -d gpurun_out/r05q_kt_em8 -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --emulate 8 --emulate-rank 7
RT_LIB_DIR=ray_tracying_amd/lib_exit step r05q_exit_em8.log 200 python3 bench.py --no-cpu-baseline --steps 6 --emulate 8 --emulate-rank 7
RT_LIB_DIR=ray_tracying_amd/lib_exit step r05q_exit_em8_f1.log 200 python3 bench.py --no-cpu-baseline --steps 6 --emulate 8 --emulate-rank 7 --frames-in-flight 1
RT_LIB_DIR=ray_tracying_amd/lib_exit step r05q_exit_head.log 200 python3 bench.py --no-cpu-baseline --steps 3
