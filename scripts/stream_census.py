"""Census of a rocprofv3 csv trace directory (hip_api_trace, kernel_trace,
memory_copy_trace, one subdirectory per rank): HIP calls that act on the
null stream by their name (hipMemset / hipMemcpy / hipMemsetD* /
hipMemcpyHtoD ... - the synchronous, stream-less forms), and kernels / copies
grouped by the stream they were queued on (Stream_Id), per rank.

    python scripts/stream_census.py gpurun_out/trace_po1d_r06
"""
import collections
import csv
import glob
import os
import sys

NULL_STREAM_CALLS = ("hipMemset", "hipMemsetD8", "hipMemsetD16", "hipMemsetD32", "hipMemcpy", "hipMemcpyHtoD",
                     "hipMemcpyDtoH", "hipMemcpyDtoD", "hipMemcpy2D", "hipMemcpy3D", "hipMemcpyToSymbol",
                     "hipMemcpyFromSymbol", "hipLaunchKernel")  # hipLaunchKernel: stream in args, counted apart


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main(d):
    for rank_dir in sorted(glob.glob(os.path.join(d, "rank*"))):
        if not os.path.isdir(rank_dir):
            continue
        print(f"== {os.path.basename(rank_dir)}")
        for api in glob.glob(os.path.join(rank_dir, "**", "*hip_api_trace.csv"), recursive=True):
            r = rows(api)
            c = collections.Counter(x["Function"] for x in r)
            print(f"  HIP API calls: {len(r)}")
            nulls = {k: v for k, v in c.items() if k in NULL_STREAM_CALLS and k != "hipLaunchKernel"}
            print(f"  null-stream (synchronous) forms: {nulls if nulls else 'none'}")
            for k in ("hipStreamCreateWithFlags", "hipStreamCreate", "hipDeviceSynchronize", "hipStreamSynchronize",
                      "hipStreamWaitEvent", "hipEventRecord", "hipMemsetAsync", "hipMemcpyAsync"):
                if c.get(k):
                    print(f"  {k}: {c[k]}")
        for kind in ("kernel_trace", "memory_copy_trace"):
            for p in glob.glob(os.path.join(rank_dir, "**", f"*{kind}.csv"), recursive=True):
                r = rows(p)
                if not r:
                    continue
                key = "Stream_Id" if "Stream_Id" in r[0] else ("Queue_Id" if "Queue_Id" in r[0] else None)
                print(f"  {kind}: {len(r)} records; columns: {', '.join(list(r[0].keys())[:14])}")
                if key:
                    by = collections.Counter(x[key] for x in r)
                    print(f"    by {key}: {dict(sorted(by.items()))}")
                    if kind == "kernel_trace":
                        names = collections.defaultdict(collections.Counter)
                        for x in r:
                            names[x[key]][x.get("Kernel_Name", "?").split("(")[0][:60]] += 1
                        for sid, cn in sorted(names.items()):
                            print(f"    {key} {sid}: {dict(cn.most_common(8))}")
                    else:
                        dirs = collections.defaultdict(collections.Counter)
                        for x in r:
                            dirs[x[key]][x.get("Direction", x.get("Operation", "?"))] += 1
                        for sid, cn in sorted(dirs.items()):
                            print(f"    {key} {sid}: {dict(cn)}")


if __name__ == "__main__":
    main(sys.argv[1])
