# r05 A/B: one scalar fma per plane (lib_scal) against packed fmas (lib); issue-mix microbenchmark
source tools/gpu_steps.sh
step r05d_ab.txt 900 bash tools/ab.sh "lib lib_scal" 2 "head em8 c5 c3"
step r05d_ubench_mix.txt 300 tools/bin/ubench_mix
