"""Per-step kernel time of a bench run's timed window from a rocprofv3
kernel trace: the window starts at the (warmup+1)-th launch of a marker
kernel (one per step) and ends at the last kernel; prints per kernel the
time per step, the busy total and the idle gaps between kernels.
Usage: python scripts/step_breakdown.py <run_kernel_trace.csv> <marker regex> <warmup> [top]"""
import collections
import csv
import re
import sys

path, marker, warm = sys.argv[1], sys.argv[2], int(sys.argv[3])
top = int(sys.argv[4]) if len(sys.argv) > 4 else 25
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if re.search(marker, r["Kernel_Name"])]
# the step runs from one marker to the next: start at the marker of the first timed step
i0 = marks[warm]
steps = len(marks) - warm
win = rows[i0:]


def short(n):
    m = re.search(r"::(\w+)(<[^>]*>)?\(", n)
    return m.group(1) if m else n[:48]


t0 = int(win[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in win)
busy = collections.Counter()
calls = collections.Counter()
last_end = t0
gap = 0
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > last_end:
        gap += s - last_end
    last_end = max(last_end, e)
    busy[short(r["Kernel_Name"])] += e - s
    calls[short(r["Kernel_Name"])] += 1
tot = sum(busy.values())
print(f"steps {steps}: window {(t1 - t0) / 1e6 / steps:.3f} ms/step, kernels {tot / 1e6 / steps:.3f}, "
      f"idle gaps {gap / 1e6 / steps:.3f}, launches {len(win) / steps:.1f}/step")
for k, v in busy.most_common(top):
    print(f"  {k[:56]:56s} {v / 1e3 / steps:8.1f} us/step  {calls[k] / steps:5.1f} calls/step")
