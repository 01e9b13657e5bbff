"""Register / LDS / occupancy summary of the gfx950 kernels in one HIP source (hipcc resource-usage remarks).

    python tools/kres.py csrc/kernels/decode_gemm.hip [name-substring]
"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(
    ["/opt/rocm/bin/hipcc", "-c", src, "-Icsrc/kernels", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
     "--offload-device-only", "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/kres.o"],
    capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    key, val = m.group(1).strip(), m.group(2).strip()
    if key == "Function Name":
        cur = {"name": val}
        rows.append(cur)
    elif cur is not None:
        cur[key] = val
for r in rows:
    if pat in r["name"]:
        print(f"{r['name'][:90]:90s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>3} "
              f"spill {r.get('VGPRs Spill', '?'):>3} occ {r.get('Occupancy [waves/SIMD]', '?'):>2} "
              f"lds {r.get('LDS Size [bytes/block]', '?')}")
