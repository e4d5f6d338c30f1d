"""Summarize rocprofv3 --pmc passes written by scripts/gpu_ab.sh:
per counter, the mean per dispatch (skipping the first, warm-up dispatch)."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
for d in sorted(glob.glob(f"gpurun_out/{tag}_pmc*_*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(d)):
        per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for c, disp in per.items():
        ids = sorted(disp)[1:] or sorted(disp)
        out[c] = sum(disp[i] for i in ids) / len(ids)
    print(d.split("/")[1], {k: f"{v:.4g}" for k, v in out.items()})
