"""Idle gaps of a bench run's timed steps from a rocprofv3 kernel trace,
attributed to the (previous kernel -> next kernel) pair they sit between.
Usage: python scripts/step_gaps.py <run_kernel_trace.csv> <marker regex> <warmup> [top]"""
import collections
import csv
import re
import sys

path, marker, warm = sys.argv[1], sys.argv[2], int(sys.argv[3])
top = int(sys.argv[4]) if len(sys.argv) > 4 else 25
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if re.search(marker, r["Kernel_Name"])]


def short(n):
    if "merge_sort_block_merge" in n:
        return "MERGE"
    if "radix_sort" in n:
        return "RADIXSORT"
    m = re.search(r"::(\w+)(<[^>]*>)?\(", n)
    return m.group(1) if m else n[:40]


gaps, cnt = collections.Counter(), collections.Counter()
steps = 0
for a, b in zip(marks[warm:-1], marks[warm + 1:]):
    steps += 1
    for i in range(a + 1, b + 1):
        g = int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])
        if g > 0:
            k = short(rows[i - 1]["Kernel_Name"]) + " -> " + short(rows[i]["Kernel_Name"]) + f" @{i - a}"
            gaps[k] += g
            cnt[k] += 1
print(f"gaps per step {sum(gaps.values()) / 1e3 / steps:.1f} us over {steps} steps")
for k, v in gaps.most_common(top):
    print(f"{v / 1e3 / steps:8.1f} us/step {cnt[k] / steps:4.1f}x  {k}")
