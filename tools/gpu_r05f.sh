# r05 A/B: cull keys by arithmetic shift (lib_cmask), bf16-pair 80-B nodes (lib_bf16) against lib
source tools/gpu_steps.sh
step r05f_ab.txt 900 bash tools/ab.sh "lib lib_cmask lib_bf16" 2 "head em8 c5 c3"
