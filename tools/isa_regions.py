"""Per-barrier-region instruction mix of one kernel in a gfx950 .s file (spill/global/LDS/VALU).
   python tools/isa_regions.py <file.s> <kernel-symbol-regex>"""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(rf"^{pat}.*:", l) and not l.startswith("\t"))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
cats = [("scr_st", r"scratch_store|buffer_store.*off, s\[0:3\]"), ("scr_ld", r"scratch_load"),
        ("g_ld", r"global_load"), ("g_st", r"global_store"), ("g_at", r"global_atomic"),
        ("ds_rd", r"ds_read"), ("ds_wr", r"ds_write"), ("valu", r"^\s+v_"), ("wait_vm", r"s_waitcnt.*vmcnt")]
region, counts = 0, {}
rows = []
for l in lines[start:end]:
    s = l.strip()
    if s.startswith(";") or not s:
        continue
    for k, rx in cats:
        if re.search(rx, l):
            counts[k] = counts.get(k, 0) + 1
    if "s_barrier" in s:
        rows.append((region, dict(counts)))
        region += 1
        counts = {}
rows.append((region, dict(counts)))
print("region " + " ".join(f"{k:>7}" for k, _ in cats))
for r, c in rows:
    if any(c.get(k, 0) for k in ("scr_st", "scr_ld", "g_ld", "g_st", "g_at")) or c.get("valu", 0) > 50:
        print(f"{r:6d} " + " ".join(f"{c.get(k, 0):7d}" for k, _ in cats))
