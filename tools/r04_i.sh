source tools/gpu_steps.sh
step r04_i_tests.log 400 python3 -u -m pytest tests/test_gpu_one_pass.py tests/test_bench_ranks.py -x -q --timeout 200 --timeout-method thread
step r04_i_ab_base.txt 600 bash tools/ab.sh "lib" 2 "head em8 em4"
cat gpurun_out/r04_i_ab_base.txt
export BENCH_EXTRA="--frames-in-flight 2"
step r04_i_ab_f2.txt 600 bash tools/ab.sh "lib" 2 "head em8 em4"
cat gpurun_out/r04_i_ab_f2.txt
step r04_i_ab_f2r.txt 600 bash tools/ab.sh "lib" 2 "head em8 em4" RT_DEFER_BPC=1
cat gpurun_out/r04_i_ab_f2r.txt
