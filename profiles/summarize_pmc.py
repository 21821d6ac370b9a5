"""Summarise rocprofv3 PMC passes (profiles/collect_pmc.sh) per kernel and derive memory traffic.

    python profiles/summarize_pmc.py <pmc dir> [out.json]

Traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB and
come from the L2's fabric-side request counters (Infinity-Cache hits are counted, not excluded);
on gfx950 FETCH_SIZE reads exactly half of a wide (16 B/lane) coalesced stream, so the read side
is reported both raw and x2-corrected; `hbm_bytes_per_launch` uses the corrected read side plus
WRITE_SIZE (exact for 16-B stores and float atomics) — an upper estimate for mixed-width loads.
"""
import collections
import csv
import glob
import json
import os
import sys


def summarize(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pass*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "ptyx" not in k:
                continue
            k = k.split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}     # mean per dispatch
        m["dispatches"] = max(len(v) for v in cs.values())
        fetch = m.get("FETCH_SIZE", 0.0) * 1024
        write = m.get("WRITE_SIZE", 0.0) * 1024
        m["fetch_bytes_raw"] = fetch
        m["fetch_bytes_x2"] = 2 * fetch
        m["write_bytes"] = write
        m["hbm_bytes_per_launch"] = 2 * fetch + write
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            m["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"]
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0) > 0:   # L2 (per XCD) hit rate
            m["l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        if "TCC_EA0_ATOMIC_sum" in m:
            m["atomic_bytes"] = 64 * m["TCC_EA0_ATOMIC_sum"]
        out[k] = m
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1])
    for k, m in res.items():
        print(k)
        for c in sorted(m):
            print(f"    {c:28s} {m[c]:.5g}")
    if len(sys.argv) > 2:
        # short kernel name (k_fused, k_obj_gather, ...) -> HBM bytes per launch, for bench.py
        short = {}
        for k, m in res.items():
            base = k.split("<")[0].split("::")[-1]
            short[{"k_fused2": "k_fused", "k_fused1": "k_fused", "k_adjoint1": "k_adjoint",
                   "k_forward1": "k_forward"}.get(base, base)] = m["hbm_bytes_per_launch"]
        payload = {"source": sys.argv[1], "hbm_bytes_per_launch": short, "kernels": res}
        with open(sys.argv[2], "w") as f:
            json.dump(payload, f, indent=1)
