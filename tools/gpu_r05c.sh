# r05 A/B: speculative leaf parking (lib_spec) against the current build (lib); lane use per phase
source tools/gpu_steps.sh
step r05c_ab.txt 900 bash tools/ab.sh "lib lib_spec" 2 "head em8 c5 c3"
step r05c_phase.log 200 env RT_LIB_DIR=ray_tracying_amd/lib_phspec python3 bench.py --no-cpu-baseline --steps 1 --warmup 0
step r05c_leaf.txt 600 bash tools/ab.sh "lib_spec" 1 "head em8" RT_LEAF_MIN=32
step r05c_leaf16.txt 600 bash tools/ab.sh "lib_spec" 1 "head em8" RT_LEAF_MIN=16
