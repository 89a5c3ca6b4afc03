# r05: SAH build parameters (host build knobs) on the headline and one rank's eighth
source tools/gpu_steps.sh
step r05m_base.txt 300 bash tools/ab.sh "lib" 1 "head em8 c5"
step r05m_node025.txt 300 bash tools/ab.sh "lib" 1 "head em8 c5" RT_SAH_NODE=0.25
step r05m_node1.txt 300 bash tools/ab.sh "lib" 1 "head em8 c5" RT_SAH_NODE=1.0
step r05m_leaf2.txt 300 bash tools/ab.sh "lib" 1 "head em8 c5" RT_SAH_LEAF=2
step r05m_leaf6.txt 300 bash tools/ab.sh "lib" 1 "head em8 c5" RT_SAH_LEAF=6
step r05m_bins64.txt 300 bash tools/ab.sh "lib" 1 "head em8 c5" RT_SAH_BINS=64
