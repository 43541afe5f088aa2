"""Per-kernel register / spill / occupancy table of a csrc file (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python scripts/kres.py <csrc file> [name regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-fno-slp-vectorize", "--offload-device-only", "-Iinclude", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark:\s+(?:Function Name: (\S+)|(\w[\w \[\]/]*?): (\S+)) \[", line)
    if not m:
        continue
    if m.group(1):
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[m.group(2).strip()] = m.group(3)
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('VGPRs Spill','?'):>3} spill {r.get('ScratchSize [bytes/lane]','?'):>4} scr "
          f"{r.get('Occupancy [waves/SIMD]','?'):>2} occ  {r['name'][:110]}")
