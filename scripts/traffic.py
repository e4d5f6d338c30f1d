"""Per-step HBM traffic of a bench workload's kernels from rocprofv3 PMC passes.

Usage: python scripts/traffic.py <workload> <regex> <FETCH_SIZE dir> <WRITE_SIZE dir> --bench-json J [--calib F]

Every dispatch of a kernel whose name matches <regex> is summed and the sum
divided by the number of steps the profiled process ran, taken as the
dispatch count of the least-launched matching kernel (each step launches
every kernel of the path at least once: advection's two tile kernels, the
GoL box kernel, the two gol_amr phases, the three Poisson phases with their
two reductions).  FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0
requests x 64 B).  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports
exactly 1/2 of the bytes of a wide coalesced streaming read, WRITE_SIZE is
exact for streaming stores; the read correction is therefore 2.0 (`--calib`
overrides).  The bench line of the profiled run (`--bench-json`) supplies the
cell count and the algorithmic bytes per step so that bench.py only uses the
figure for the same mesh.
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
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<\w+>)?)", name)
    return m.group(1).split("::")[-1] if m else name[:60]


def main():
    workload, pattern, fdir, wdir = sys.argv[1:5]
    calib = float(sys.argv[sys.argv.index("--calib") + 1]) if "--calib" in sys.argv else 2.0
    bench = json.load(open(sys.argv[sys.argv.index("--bench-json") + 1]))
    f = per_kernel(fdir, pattern, "FETCH_SIZE")
    w = per_kernel(wdir, pattern, "WRITE_SIZE")
    if not f or not w:
        sys.exit(f"no dispatches matching {pattern!r}")
    steps = min(len(v) for v in f.values())
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fk, wk = f.get(k, []), w.get(k, [])
        kernels[k] = dict(dispatches=len(fk), fetch_kib_raw_avg=sum(fk) / max(len(fk), 1),
                          write_kib_avg=sum(wk) / max(len(wk), 1),
                          hbm_bytes_per_step=(sum(fk) * calib + sum(wk)) * 1024 / steps)
    total = sum(v["hbm_bytes_per_step"] for v in kernels.values())
    roof = bench["roofline"]
    out = dict(workload=workload, kernels=kernels, steps_profiled=steps, read_correction=calib,
               read_correction_source="MI355X_MICROARCH.md: FETCH_SIZE = 1/2 of wide coalesced reads on gfx950",
               hbm_bytes_per_step=total, cells=bench["config"]["cells_rank0"],
               alg_bytes_per_step=roof["alg_bytes_per_step"], traffic_over_alg=total / roof["alg_bytes_per_step"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
