"""Summarize a rocprofv3 run directory tree: per kernel the mean of each
counter per dispatch (first dispatch of each kernel skipped as warm-up), and
for kernel-trace runs the per-kernel average duration.
Usage: python scripts/pmc_summary2.py gpurun_out/<tag>_pmc1 [...]"""
import collections
import csv
import glob
import os
import re
import sys


def kname(s):
    m = re.search(r"(\w+_kernel\w*|gol_structured_v3)", s)
    return m.group(1) if m else s[:48]


for root in sys.argv[1:]:
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
        for r in csv.DictReader(open(f)):
            per[kname(r["Kernel_Name"])][r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for k, cs in sorted(per.items()):
            out = {}
            for c, disp in cs.items():
                ids = sorted(disp)[1:] or sorted(disp)
                out[c] = sum(disp[i] for i in ids) / len(ids)
            print(os.path.basename(root), k, {c: f"{v:.4g}" for c, v in sorted(out.items())})
    for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            print(os.path.basename(root), kname(r["Name"]), "calls", r["Calls"], "avg_us", f"{float(r['AverageNs']) / 1e3:.1f}")
