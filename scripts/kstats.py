"""Per-kernel summary of a rocprofv3 kernel_stats.csv: short name, calls,
average us, ms per step.   python scripts/kstats.py stats.csv [steps] [top]"""
import csv
import re
import sys


def short(name):
    n = name.replace("dccrgx::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"rocprim::ROCPRIM_\w+::detail::", "rocprim::", n)
    m = re.match(r"rocprim::trampoline_kernel<rocprim::wrapped_(\w+?)_config", n)
    if m:
        return "rocprim " + m.group(1)
    return n.split("(")[0][:70]


def main(path, steps=1.0, top=40):
    rows = list(csv.DictReader(open(path)))
    for x in rows[:top]:
        print(f"{short(x['Name']):72s} calls {int(x['Calls']):6d} avg {float(x['AverageNs']) / 1e3:9.1f} us  "
              f"{float(x['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0, int(sys.argv[3]) if len(sys.argv) > 3 else 40)
