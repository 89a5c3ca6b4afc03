#!/usr/bin/env python3
"""node_visit_isa.py -- static instruction mix of one BVH4 node visit (tools/node_visit_isa.hip:
rt_hip.hip's node_visit<false, true> -- the planes instances' visit with fp16 codes -- alone in a
probe kernel, compiled with the product flags), split into the per-child instructions of the slab
and cull and the rest.  Input to the width decision.
Usage: python3 tools/node_visit_isa.py [out.txt]"""
import collections
import re
import subprocess
import sys

FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-fno-slp-vectorize", "-Wno-unused-result", "--cuda-device-only", "-S"]
subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "tools/node_visit_isa.hip", "-o", "/tmp/node_visit_isa.s"], check=True,
               capture_output=True)
txt = open("/tmp/node_visit_isa.s").read()
body = re.search(r"node_visit_probe\S*:\s*;.*?\n(.*?)\.Lfunc_end", txt, re.S).group(1)
seg = body[body.index("NODE_VISIT_BEGIN"):body.index("NODE_VISIT_END")]
ins = [ln.split(";")[0].split()[0] for ln in seg.split("\n") if ln.split(";")[0].strip() and not ln.strip().startswith(".")]
c = collections.Counter(ins)
valu = sum(v for k, v in c.items() if k.startswith("v_"))
per_child = {k: c[k] for k in ("v_fma_mix_f32", "v_perm_b32", "v_max3_i32", "v_min3_i32", "v_max_i32_e32", "v_min_i32_e32")}
lines = [f"node visit (static, hot and cold paths): {len(ins)} instructions, {valu} VALU, "
         f"{sum(v for k, v in c.items() if k.startswith('s_'))} SALU, {sum(v for k, v in c.items() if k.startswith('ds_'))} LDS, "
         f"{sum(v for k, v in c.items() if k.startswith('global_'))} VMEM",
         f"slab + cull per child (4 children): {per_child} = {sum(per_child.values())} (+ a compare and a select "
         "per child for the entry distance)",
         "mix: " + ", ".join(f"{k} {v}" for k, v in c.most_common())]
open(sys.argv[1] if len(sys.argv) > 1 else "/dev/stdout", "w").write("\n".join(lines) + "\n")
