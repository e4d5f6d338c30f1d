"""Per-dispatch HBM traffic of a kernel from rocprofv3 PMC passes.

Usage: python scripts/traffic.py <kernel-substring> <FETCH_SIZE dir> <WRITE_SIZE dir> [--calib F]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0 requests x 64 B).
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports exactly 1/2 of the
bytes of a wide coalesced streaming read; WRITE_SIZE is exact for streaming
stores.  The read correction factor for this kernel's access pattern is
`--calib` (default 2.0, the guide's streaming-read factor; other access
widths are uncalibrated there).
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
    if "--calib" in sys.argv:
        calib = float(sys.argv[sys.argv.index("--calib") + 1])
    f = per_dispatch(fdir, kernel, "FETCH_SIZE")
    w = per_dispatch(wdir, kernel, "WRITE_SIZE")
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    out = dict(kernel=kernel, dispatches=[len(f), len(w)], fetch_kib_raw=fk, write_kib=wk, read_correction=calib,
               hbm_bytes_per_dispatch=(fk * calib + wk) * 1024)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
