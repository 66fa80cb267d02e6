"""Per-kernel register / spill / LDS table from hipcc's kernel-resource-usage remarks.

    python tools/kres.py [filter-regex]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include", "-c",
       f"{ROOT}/simplex_method_gpu_amd/csrc/spx_kernels.hip", "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for ln in err.splitlines():
    m = re.search(r"(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\S+) \[-Rpass", ln)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
flt = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
for r in rows:
    if flt and not flt.search(r["name"]):
        continue
    print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} occ={r.get('Occupancy')} "
          f"spillV={r.get('VGPRs Spill')} spillS={r.get('SGPRs Spill')} scratch={r.get('ScratchSize')}")
