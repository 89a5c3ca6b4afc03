# r05: rank shares (4- and 8-way) with the 7-wave instances: frames in flight, reserved block
source tools/gpu_steps.sh
step r05l_em8_default.txt 300 bash tools/ab.sh "lib" 2 "em8 em4"
step r05l_em8_seven.txt 300 bash tools/ab.sh "lib" 2 "em8 em4" RT_TRACE_SEVEN=1
step r05l_em8_seven_defer0.txt 300 bash tools/ab.sh "lib" 2 "em8 em4" RT_TRACE_SEVEN=1 RT_DEFER_BPC=0
step r05l_em8_seven_f1.txt 300 env BENCH_EXTRA="--frames-in-flight 1" bash tools/ab.sh "lib" 2 "em8 em4" RT_TRACE_SEVEN=1
step r05l_em8_f1.txt 300 env BENCH_EXTRA="--frames-in-flight 1" bash tools/ab.sh "lib" 2 "em8 em4"
step r05l_c34.txt 300 bash tools/ab.sh "lib" 1 "c3 c4"
