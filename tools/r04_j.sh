source tools/gpu_steps.sh
step r04_j_smoke.log 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step r04_j_gpu_tests.log 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step r04_j_ab_auto.txt 600 bash tools/ab.sh "lib" 2 "head em8 em4 c2"
cat gpurun_out/r04_j_ab_auto.txt
export BENCH_EXTRA="--frames-in-flight 1"
step r04_j_ab_f1.txt 600 bash tools/ab.sh "lib" 2 "em8 em4 c2"
cat gpurun_out/r04_j_ab_f1.txt
