"""Compact per-kernel register / spill / LDS table of one .hip file (hipcc -Rpass-analysis):
python scripts/kres.py localai_amd/ops/csrc/gemm_bs.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fno-slp-vectorize",
       "-I", "localai_amd/ops/csrc", "--cuda-device-only", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
r = subprocess.run(cmd, capture_output=True, text=True)
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split(" [")[0]] = int(m.group(2))
for c in rows:
    if flt in c["name"]:
        print(f"{c['name'][:90]:90s} v{c.get('VGPRs')} a{c.get('AGPRs')} spill{c.get('VGPRs Spill')} "
              f"lds{c.get('LDS Size')} occ{c.get('Occupancy')}")
if r.returncode:
    print(r.stderr[-3000:])
