"""Per-kernel VGPR/AGPR/scratch/occupancy from hipcc -Rpass-analysis=kernel-resource-usage.
usage: python tools/res_usage.py file.hip [substring]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o", "/tmp/_ru.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", ln)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    if pat in k:
        print(f"{k[:70]:70s} vgpr {v.get('VGPRs')} agpr {v.get('AGPRs')} scratch {v.get('ScratchSize')} occ {v.get('Occupancy')} lds {v.get('LDS')}")
