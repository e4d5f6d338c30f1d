#!/bin/bash
# Face table grid size (DCCRGX_FACE_GRID blocks: default 8192 = grid_for's cap,
# 1792 = 256 CUs x 7 resident blocks, 3584): kernel stats per size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06zm}
for g in ${GRIDS:-8192 1792 3584}; do
  DCCRGX_FACE_GRID=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$g -o run --output-format csv -- \
      python3 bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_$g.json 2>/dev/null || exit 1
  f=$(find gpurun_out/${TAG}_prof_$g -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'face_table' in r['Name']: print('grid=$g', r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')"
done
