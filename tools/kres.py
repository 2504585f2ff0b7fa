#!/usr/bin/env python3
"""Per-kernel register use and spills of icp_kernels.hip as hipcc reports
them (-Rpass-analysis=kernel-resource-usage): `python tools/kres.py [filter]`
compiles the TU for gfx950 with the product flags (object discarded) and
prints VGPRs / AGPRs / SGPRs / spills / occupancy per kernel."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
flt = sys.argv[1] if len(sys.argv) > 1 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
       "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", f"-I{ROOT}/include",
       f"-I{ROOT}/slam-rgbd_amd/csrc", "-c", f"{ROOT}/slam-rgbd_amd/csrc/icp_kernels.hip",
       "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for ln in out.splitlines():
    m = re.search(r"remark: ([A-Za-z ]+): (.+?)\s*\[-Rpass", ln)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        cur = re.sub(r"\(anonymous namespace\)::", "", cur).split("(")[0]
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    if flt in name:
        print(f"{name:45s} VGPR {r.get('VGPRs','?'):>4s} AGPR {r.get('AGPRs','?'):>3s} "
              f"SGPR {r.get('SGPRs','?'):>4s} spillV {r.get('VGPRs Spill','?'):>4s} "
              f"spillS {r.get('SGPRs Spill','?'):>4s} occ {r.get('Occupancy','?')}")
