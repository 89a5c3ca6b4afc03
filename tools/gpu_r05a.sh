source tools/gpu_steps.sh
step r05a_smoke.log 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step r05a_gpu_tests.log 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 800 --timeout-method thread
step r05a_head.json 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2
step r05a_em8.json 300 python3 bench.py --no-cpu-baseline --steps 10 --emulate 8 --emulate-rank 7
