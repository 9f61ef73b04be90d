"""Per-kernel resource usage (VGPRs, spills, occupancy, LDS) of one csrc/*.hip file, from hipcc's
kernel-resource-usage remarks.  usage: python tools/kres.py attention.hip [name-filter]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "stable-diffusion-from-scratch_amd", "csrc")
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = ["-mno-amdgpu-ieee", "-fno-honor-nans"] if src == "attention.hip" else []
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", *extra, "-I", CS,
       "-I", os.path.join(ROOT, "include"), "-c", os.path.join(CS, src), "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)([^:\[]+): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    if flt and flt not in name:
        continue
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    print(f"{dem[:110]:110s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} vspill={r.get('VGPRs Spill')} "
          f"sspill={r.get('SGPRs Spill')} occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}")
