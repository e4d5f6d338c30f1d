#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06n}
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/${TAG}_adapt_$i.json 2> gpurun_out/${TAG}_adapt_$i.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_$i.json').read().strip().splitlines()[-1]); print('adapt', round(d['ms_per_step'],3), d['adaptation']['created_total'], d['adaptation']['removed_total'])"
done
