#!/bin/bash
# Poisson transpose factors: the Poisson suites, then paired bench lines (on / off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06zf}
timeout -k 10 600 python -u -m pytest tests/test_gpu_poisson.py tests/test_gpu_transport.py tests/test_gpu_facade.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    DCCRGX_PO_FT=$v timeout -k 10 300 python -u bench.py --workload poisson --steps 200 --warmup 5 --no-cpu-baseline \
        > gpurun_out/${TAG}_po_ft${v}_${rep}.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_po_ft${v}_${rep}.json').read().strip().splitlines()[-1]); print('ft=$v rep $rep', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done
