# r05 A/B: cull keys by shifts (fixed: negative far distances), bf16 nodes, both; seven waves
source tools/gpu_steps.sh
step r05g_ab.txt 900 bash tools/ab.sh "lib lib_cmask lib_bf16 lib_bfcm" 2 "head em8 c5"
step r05g_w7.txt 300 bash tools/ab.sh "lib_w7" 1 "head em8 c5" RT_LDS_STACK=11
