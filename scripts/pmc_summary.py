"""Summarize rocprofv3 --pmc passes written by scripts/gpu_ab.sh: per
kernel and counter, the mean per dispatch (skipping each kernel's first,
warm-up dispatch)."""
import collections
import csv
import glob
import re
import sys

tag = sys.argv[1]
for d in sorted(glob.glob(f"gpurun_out/{tag}_pmc*_*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in csv.DictReader(open(d)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        per[k][r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    for k, cs in per.items():
        out = {}
        for c, disp in cs.items():
            ids = sorted(disp)[1:] or sorted(disp)
            out[c] = sum(disp[i] for i in ids) / len(ids)
        print(d.split("/")[1], k, {c: f"{v:.4g}" for c, v in out.items()})
