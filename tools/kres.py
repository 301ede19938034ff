"""Per-kernel VGPRs / scratch / occupancy / LDS of one HIP TU (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python tools/kres.py <file.hip> [name-filter]   (run from the csrc directory)"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-I../../include", "-munsafe-fp-atomics", "--cuda-device-only", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s*(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]|VGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).replace(' Spill', '_spill').split(' ')[0], m.group(2)
    if k == "Function":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        nm = re.sub(r"\(.*", "", r["name"])
        print(f"{nm:60s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} scratch={r.get('ScratchSize')} "
              f"occ={r.get('Occupancy')} lds={r.get('LDS')} spill={r.get('VGPRs_spill')}")
