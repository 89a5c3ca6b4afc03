#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of librt_hip (hipcc kernel-resource-usage
remarks): python3 tools/regs.py [extra hipcc defines...]"""
import re, subprocess, sys
src = "ray_tracying_amd/csrc/hip/rt_hip.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", "-fPIC", "-Wno-unused-result",
       "-shared", src, "-o", "/tmp/regs_probe.so", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)(.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    n = n.replace("(anonymous namespace)::", "")
    print(f"{n[:70]:70s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>3} vspill {r.get('VGPRs Spill','?'):>3} "
          f"sspill {r.get('SGPRs Spill','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?')} lds {r.get('LDS Size [bytes/block]','?')}")
