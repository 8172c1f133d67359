"""Per-kernel resource usage of one HIP source (VGPRs / AGPRs / occupancy / LDS) from hipcc's
-Rpass-analysis=kernel-resource-usage remarks.  Usage: python tools/kres.py csrc/kernels/gemm.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I../include",
                    "-Icsrc", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur = {}
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).split(" ")[0], m.group(2)
    if k == "Function":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k] = v
for c in rows:
    n = c["name"].replace("wdr::", "")
    if flt in n:
        print(f"{n[:90]:90s} vgpr {c.get('VGPRs'):>4} agpr {c.get('AGPRs'):>4} occ {c.get('Occupancy'):>2} "
              f"lds {c.get('LDS'):>6} scratch {c.get('ScratchSize')}")
if r.returncode:
    print(r.stderr[-3000:])
