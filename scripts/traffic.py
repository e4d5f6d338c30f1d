"""Per-dispatch HBM traffic of a kernel from rocprofv3 PMC passes.

Usage: python scripts/traffic.py <kernel-substring> <FETCH_SIZE dir> <WRITE_SIZE dir>
           [--calib F | --calib-dir D --calib-json J]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0 requests x 64 B).
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports exactly 1/2 of the
bytes of a wide coalesced streaming read; WRITE_SIZE is exact for streaming
stores.  The read correction factor for this kernel's access pattern is
`--calib` (default 2.0, the guide's streaming-read factor; other access
widths are uncalibrated there), or measured: `--calib-dir` holds a
FETCH_SIZE pass of the stream-only diagnostic form of the same kernel
(DCCRGX_ADV_DIAG=3: 8-B-per-lane loads of the seven fields, 56 B per cell,
nothing else) and `--calib-json` that run's bench line (cell count), so
factor = 56 * cells / FETCH_SIZE bytes.
"""
import csv
import glob
import json
import sys


def per_dispatch(d, kernel, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    vals = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    kernel, fdir, wdir = sys.argv[1:4]
    calib = 2.0
    calib_src = "guide (wide streaming reads)"
    if "--calib" in sys.argv:
        calib = float(sys.argv[sys.argv.index("--calib") + 1])
        calib_src = "command line"
    if "--calib-dir" in sys.argv:
        cdir = sys.argv[sys.argv.index("--calib-dir") + 1]
        cells = json.load(open(sys.argv[sys.argv.index("--calib-json") + 1]))["config"]["cells_rank0"]
        c = per_dispatch(cdir, kernel, "FETCH_SIZE")
        calib = 56.0 * cells / (sum(c) / len(c) * 1024)
        calib_src = f"measured: stream-only form, 56 B x {cells} cells"
    f = per_dispatch(fdir, kernel, "FETCH_SIZE")
    w = per_dispatch(wdir, kernel, "WRITE_SIZE")
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    out = dict(kernel=kernel, dispatches=[len(f), len(w)], fetch_kib_raw=fk, write_kib=wk, read_correction=calib,
               read_correction_source=calib_src, hbm_bytes_per_dispatch=(fk * calib + wk) * 1024)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
