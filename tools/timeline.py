"""Per-pass timeline from a rocprofv3 kernel trace: kernel durations and the
gaps between consecutive kernels (the seams), averaged by kernel pair.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o tl -- python3 tools/itbench.py ...
    python tools/timeline.py OUT/.../tl_kernel_trace.csv [--skip 100]
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    m = re.search(r"spx::(k_\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--skip", type=int, default=100, help="dispatches skipped at the start (setup, warm-up)")
a = ap.parse_args()
rows = []
with open(a.csv) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
rows.sort()
rows = rows[a.skip:]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for i, (s, e, k) in enumerate(rows):
    dur[k].append(e - s)
    if i + 1 < len(rows):
        gap[(k, rows[i + 1][2])].append(rows[i + 1][0] - e)
out = {"kernels": {k: {"n": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 3),
                       "min_us": round(min(v) / 1e3, 3)} for k, v in dur.items()},
       "gaps": {f"{a_} -> {b_}": {"n": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 3),
                                  "min_us": round(min(v) / 1e3, 3)}
                for (a_, b_), v in gap.items() if len(v) >= 3}}
print(json.dumps(out, indent=1))
