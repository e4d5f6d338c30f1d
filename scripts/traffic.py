"""Per-step HBM traffic of the advection sweep from rocprofv3 PMC passes.

Usage: python scripts/traffic.py <regex> <FETCH_SIZE dir> <WRITE_SIZE dir> --bench-json J [--calib F]

Every kernel whose name matches <regex> is averaged over its dispatches and
the per-kernel averages are summed (the sweep is one dispatch of the
regular-tile kernel plus one of the general tile kernel per step).
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0 requests x 64 B).
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports exactly 1/2 of the
bytes of a wide coalesced streaming read, WRITE_SIZE is exact for streaming
stores; the read correction is therefore 2.0 (`--calib` overrides).  The
bench line of the profiled run (`--bench-json`) supplies the cell count so
that bench.py only uses the figure for the same mesh.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def per_kernel(d, pattern, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if re.search(pattern, r["Kernel_Name"]) and r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def short(name):
    m = re.search(r"(advection_\w+?kernel)", name)
    return m.group(1) if m else name[:60]


def main():
    pattern, fdir, wdir = sys.argv[1:4]
    calib = float(sys.argv[sys.argv.index("--calib") + 1]) if "--calib" in sys.argv else 2.0
    bench = json.load(open(sys.argv[sys.argv.index("--bench-json") + 1]))
    f = per_kernel(fdir, pattern, "FETCH_SIZE")
    w = per_kernel(wdir, pattern, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        kernels[short(k)] = dict(fetch_kib_raw=f.get(k, 0.0), write_kib=w.get(k, 0.0),
                                 hbm_bytes=(f.get(k, 0.0) * calib + w.get(k, 0.0)) * 1024)
    total = sum(v["hbm_bytes"] for v in kernels.values())
    out = dict(kernels=kernels, read_correction=calib,
               read_correction_source="MI355X_MICROARCH.md: FETCH_SIZE = 1/2 of wide coalesced reads on gfx950",
               hbm_bytes_per_step=total, cells=bench["config"]["cells_rank0"],
               alg_bytes_per_step=bench["roofline"]["alg_bytes_per_step"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
