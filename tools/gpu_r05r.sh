# r05: one rank's share with two frames in flight is bound by each stream's serial chain
# (trace 3.7 ms + shading / camera kernels of ~0.65 ms each squeezed into the reserved block):
# three frames in flight, two reserved blocks per CU, and both
source tools/gpu_steps.sh
step r05r_f2.txt 200 bash tools/ab.sh lib 2 "em8 em4"
BENCH_EXTRA="--frames-in-flight 3" step r05r_f3.txt 200 bash tools/ab.sh lib 2 "em8 em4"
step r05r_f2_bpc2.txt 200 bash tools/ab.sh lib 2 "em8 em4" RT_DEFER_BPC=2
BENCH_EXTRA="--frames-in-flight 3" step r05r_f3_bpc2.txt 200 bash tools/ab.sh lib 2 "em8 em4" RT_DEFER_BPC=2
BENCH_EXTRA="--frames-in-flight 4" step r05r_f4.txt 200 bash tools/ab.sh lib 2 "em8 em4"
