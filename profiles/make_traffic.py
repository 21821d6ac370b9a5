"""Per-config HBM traffic table for bench.py's roofline.traffic, from a tools/gpu_profile.sh run.

    python profiles/make_traffic.py <profile dir> <git head> [config ...]

For each config it reads <dir>/pmc_<c>.json (profiles/summarize_pmc.py: FETCH_SIZE x2 + WRITE_SIZE
per dispatch, MI355X_MICROARCH.md gfx950 correction) and <dir>/<c>_kernel_stats.csv (rocprofv3
--kernel-trace --stats of the same bench command) and writes profiles/traffic.json:

  {config: {"kernel": dominant kernel, "bytes_per_launch": B, "patterns_per_launch": n,
            "bytes_per_pattern": B / n, "passes": {pass: bytes per pattern} (stripe engine),
            "avg_launch_ms_rocprof": ..., "source": dir, "measured_at": head}}

The PMC passes run `bench.py --steps 1 --warmup 0`, so a kernel's dispatch count there is its
launches per step; patterns per launch = the bench's patterns per step / that count.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = {"c2": "k_fused3", "c2-strong": "k_fused3", "c4": "k_fused3ms"}
STRIPE = ("k_s1", "k_s2", "k_s3", "k_s4", "k_s5", "k_obj_gather")


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def kernel_stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Name"])
        c, avg = int(r["Calls"]), float(r["AverageNs"]) / 1e6
        if k in out:   # several template instances: merge
            c0, a0 = out[k]
            out[k] = (c0 + c, (a0 * c0 + avg * c) / (c0 + c))
        else:
            out[k] = (c, avg)
    return out


def dispatches(pmc, kernel):
    """Dispatches of `kernel` in the PMC run (one bench step), summed over template instances."""
    return sum(int(m["dispatches"]) for k, m in pmc["kernels"].items() if short(k) == kernel)


def main(d, head, configs):
    table_path = os.path.join(ROOT, "profiles", "traffic.json")
    table = json.load(open(table_path)) if os.path.exists(table_path) else {}
    rel = os.path.relpath(d, ROOT)
    for c in configs:
        pmc = json.load(open(os.path.join(d, f"pmc_{c}.json")))
        bench = json.load(open(os.path.join(d, f"bench_{c}.json")))
        per_step = bench["config"]["patterns_per_gpu_per_step"]
        stats = kernel_stats(os.path.join(d, f"{c}_kernel_stats.csv"))
        bpl = pmc["hbm_bytes_per_launch"]
        if c in DOMINANT:
            k = DOMINANT[c]
            launches = dispatches(pmc, k)
            n = per_step / launches
            table[c] = {"kernel": k, "bytes_per_launch": bpl[k], "patterns_per_launch": n,
                        "bytes_per_pattern": bpl[k] / n, "avg_launch_ms_rocprof": round(stats[k][1], 4),
                        "source": rel, "measured_at": head}
            if "k_obj_gather" in bpl:
                g = dispatches(pmc, "k_obj_gather")
                table[c]["gather_bytes_per_step"] = bpl["k_obj_gather"] * g
        else:
            launches = dispatches(pmc, "k_s3")
            n = per_step / launches
            passes = {k: bpl[k] / n for k in STRIPE if k in bpl}
            if "k_obj_gather" in passes:   # one gather launch per object mode and call
                passes["k_obj_gather"] *= dispatches(pmc, "k_obj_gather") / launches
            table[c] = {"kernel": "stripe engine k_s1..k_s5", "patterns_per_launch": n,
                        "bytes_per_pattern": sum(passes.values()), "passes": passes,
                        "avg_launch_ms_rocprof": {k: round(stats[k][1], 4) for k in STRIPE if k in stats},
                        "source": rel, "measured_at": head}
    json.dump(table, open(table_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(table, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:] or ["c3", "c4", "c5"])
