#!/bin/bash
# PMC passes (one counter group per run, --pmc never combined with tracing)
# on the advection kernels for a list of env configurations:
#   CONFIGS="A=1;B=2" KREGEX=advection_regular bash scripts/pmc_adv.sh tag
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pmc}
IFS=';' read -ra CFGS <<< "${CONFIGS:-X=0}"
GROUPS_=${GROUPS_:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum"}
IFS=';' read -ra GRPS <<< "$GROUPS_"
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  k=0
  for grp in "${GRPS[@]}"; do
    k=$((k+1))
    env $cfg timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-advection}" \
       -d gpurun_out/${TAG}_${i}_$k -o run --output-format csv -- \
       python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/${TAG}_${i}_$k.err || exit $?
  done
  python - "$cfg" gpurun_out ${TAG}_${i} <<'PY'
import csv, glob, sys
from collections import defaultdict
cfg, root, pre = sys.argv[1:4]
acc = defaultdict(list)
for f in glob.glob(f"{root}/{pre}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r['Kernel_Name'].split('(')[0].split('<')[0].split('::')[-1]
        acc[(kn, r['Counter_Name'])].append(float(r['Counter_Value']))
print('[%s]' % cfg)
for (kn, c), v in sorted(acc.items()):
    print('   %-32s %-14s %.4g (per dispatch, %d dispatches)' % (kn, c, sum(v) / len(v), len(v)))
PY
done
