"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel.
    python tools/resource_usage.py <remarks.txt> [name-substring ...]"""
import re
import sys

rows, cur = [], None
for line in open(sys.argv[1]):
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0] + ("Spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
filt = sys.argv[2:]
for r in rows:
    if filt and not any(f in r["name"] for f in filt):
        continue
    print(f"{r['name'][:48]:48s} vgpr {r.get('VGPRs', '-'):>4} agpr {r.get('AGPRs', '-'):>4} "
          f"spill {r.get('VGPRsSpill', '-'):>4} scratch {r.get('ScratchSize', '-'):>4} occ {r.get('Occupancy', '-')} "
          f"lds {r.get('LDS', '-')}")
