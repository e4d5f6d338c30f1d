#!/bin/bash
# FETCH_SIZE per advection kernel for several env configurations
# (CONFIGS, ';'-separated), one --pmc pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-fab}
IFS=';' read -ra CFGS <<< "${CONFIGS}"
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  env $cfg timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex advection -d gpurun_out/${TAG}_$i -o run \
      --output-format csv -- python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || exit $?
  echo "[$cfg]"
  python - "$TAG" "$i" <<'PY'
import collections, csv, glob, re, sys
tag, i = sys.argv[1], sys.argv[2]
per = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/{tag}_{i}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        per[m.group(1) if m else "?"].append(float(r["Counter_Value"]))
for k, v in per.items():
    v = v[1:] or v
    print(f"   {k}: FETCH_SIZE {sum(v)/len(v)*2*1024/1e6:.1f} MB (x2) over {len(v)} dispatches")
PY
done
