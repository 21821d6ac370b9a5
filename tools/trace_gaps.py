"""Kernel-timeline summary of a rocprofv3 --kernel-trace CSV: per kernel name the count and mean
duration, and the busy fraction / mean gap between consecutive kernels over the traced span.

    python tools/trace_gaps.py <kernel_trace.csv> [--last N]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if last:
        ev = ev[-last:]
    span = ev[-1][1] - ev[0][0]
    busy = sum(e - s for s, e, _ in ev)
    gaps = [ev[i + 1][0] - ev[i][1] for i in range(len(ev) - 1)]
    per = defaultdict(list)
    for s, e, n in ev:
        per[n.split("(")[0][:70]].append(e - s)
    print(f"kernels {len(ev)} span {span / 1e3:.1f} us busy {busy / 1e3:.1f} us ({100 * busy / span:.1f} %) "
          f"mean gap {sum(gaps) / max(1, len(gaps)) / 1e3:.2f} us")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(d):7d} {sum(d) / len(d) / 1e3:9.2f} us  {sum(d) / 1e3:10.1f} us  {n}")


if __name__ == "__main__":
    main()
