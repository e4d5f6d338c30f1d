#!/bin/bash
# Requests kernel block size (DCCRGX_REQ_BS 1024 / 512 / 256; a block stages
# 8 slots per thread): the adaptive suites, paired lines, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06zj}
for bs in 256 512; do
  DCCRGX_REQ_BS=$bs timeout -k 10 300 python -u -m pytest tests/test_gpu_advection_adapt.py tests/test_gpu_ref_advection.py \
      -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_${TAG}_$bs.log 2>&1 || { tail -5 gpurun_out/pytest_${TAG}_$bs.log; exit 1; }
  tail -1 gpurun_out/pytest_${TAG}_$bs.log
done
for rep in 1 2; do
  for bs in 1024 512 256; do
    DCCRGX_REQ_BS=$bs timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/${TAG}_bs${bs}_${rep}.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bs${bs}_${rep}.json').read().strip().splitlines()[-1]); print('bs=$bs rep $rep', round(d['ms_per_step'],4))"
  done
done
for bs in 1024 512 256; do
  DCCRGX_REQ_BS=$bs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$bs -o run --output-format csv -- \
      python3 bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/${TAG}_prof_$bs -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'adv_requests' in r['Name']: print('bs=$bs', r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')"
done
