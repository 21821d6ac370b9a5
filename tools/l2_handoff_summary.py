"""Per-(W, variant) PMC summary of tools/l2_handoff --once under rocprofv3 (tools/gpu_r04_l2.sh).

    python tools/l2_handoff_summary.py <gpurun_out/<tag>> [out.json]

The --once run dispatches, for each payload size W in order, k_fused<0> (same XCD), k_fused<1>
(cross XCD), then k_produce_all + k_consume_all (two kernels); the fills / copies around them are
skipped.  FETCH_SIZE is doubled (gfx950 tallies 128-B streaming requests at 64 B,
MI355X_MICROARCH.md §HBM); L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS).
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("k_fused<0>", "k_fused<1>", "k_produce_all", "k_consume_all")


def per_dispatch(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if not any(x in k for x in KERNELS):
            continue
        e = d.setdefault(int(r["Dispatch_Id"]), {"kernel": k.split("(")[0].replace("void ", "")})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(d.values())


def main():
    base = os.path.join(sys.argv[1], "pmc_handoff")
    passes = [per_dispatch(f) for f in sorted(glob.glob(os.path.join(base, "pass_*", "*counter_collection.csv")))]
    merged = [dict(collections.ChainMap(*parts)) for parts in zip(*passes)]
    timed = [json.loads(l) for l in open(os.path.join(sys.argv[1], "l2_handoff.jsonl"))]
    sizes = sorted({t["W_bytes"] for t in timed})
    out, i = [], 0
    for W in sizes:
        for variant, n in (("fused_same_xcd", 1), ("fused_cross_xcd", 1), ("two_kernels", 2)):
            ds = merged[i:i + n]
            i += n
            fetch = 2 * 1024 * sum(x.get("FETCH_SIZE", 0) for x in ds)
            write = 1024 * sum(x.get("WRITE_SIZE", 0) for x in ds)
            hit = sum(x.get("TCC_HIT_sum", 0) for x in ds)
            miss = sum(x.get("TCC_MISS_sum", 0) for x in ds)
            t = next(x for x in timed if x["W_bytes"] == W and x["variant"] == variant)
            payload = W * t["tasks"]
            out.append({"W_bytes": W, "variant": variant, "ms": t["ms"], "GBps_moved": t["GBps_moved"],
                        "read_fetch_over_payload": round(fetch / payload, 3),
                        "write_over_payload": round(write / payload, 3),
                        "l2_hit_rate": round(hit / (hit + miss), 3) if hit + miss else None,
                        "kernels": [x["kernel"] for x in ds]})
    for o in out:
        print(json.dumps(o))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
