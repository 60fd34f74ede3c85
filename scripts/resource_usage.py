"""Per-kernel registers / scratch / occupancy of kernels.hip for gfx950
(clang's kernel-resource-usage remarks), one line per function."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "wiser_amd/csrc/kernels.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "--offload-device-only", "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|"
                  r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split()[0]] = v
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    name = re.sub(r"\(.*", "", name)
    print(f"{name[:48]:48s} vgpr {r.get('VGPRs','?'):>4} sgpr {r.get('TotalSGPRs','?'):>4} "
          f"scratch {r.get('ScratchSize','?'):>4} occ {r.get('Occupancy','?'):>2} lds {r.get('LDS','?')}")
