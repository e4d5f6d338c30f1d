#!/bin/bash
# Poisson iteration: its tests, then the config-4 bench line paired A/B of
# an environment knob (KNOB=1 / 0), two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-po}
KNOB=${2:-DCCRGX_PO_LDS}
timeout -k 10 600 python -u -m pytest tests/test_gpu_poisson.py tests/test_gpu_transport.py -k "oisson" -m gpu -v \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log
grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for round in 1 2; do
  for v in 1 0; do
    env $KNOB=$v timeout -k 10 300 python -u bench.py --workload poisson --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/ab_${TAG}_${v}_${round}.json 2> gpurun_out/ab_${TAG}_${v}_${round}.err || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/ab_${TAG}_${v}_${round}.json').read().strip().splitlines()[-1])
print('[ab] $KNOB=$v round $round: %.4f ms/step, kernels %.4f ms' % (d['ms_per_step'], d['roofline']['kernel_ms_per_step']))"
  done
done
