#!/bin/bash
# per-kernel advection timings (rocprofv3 kernel trace) for a list of env
# configurations: CONFIGS="A=1;B=2" bash scripts/prof_adv.sh tag
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pa}
IFS=';' read -ra CFGS <<< "${CONFIGS:-X=0}"
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$i -o run --output-format csv -- \
      python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2>gpurun_out/${TAG}_$i.err || exit $?
  python - "$cfg" gpurun_out/${TAG}_$i/run_kernel_stats.csv <<'PY'
import csv, sys
out = []
for r in csv.DictReader(open(sys.argv[2])):
    if 'advection' in r['Name']:
        out.append('%s %.1fus' % (r['Name'].split('(')[0].split('::')[-1][:40], float(r['AverageNs']) / 1e3))
print('[%s]' % sys.argv[1], ' | '.join(out))
PY
done
