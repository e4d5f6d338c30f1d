#!/bin/bash
# Adaptive bench, paired A/B of an environment knob (KNOB=1 / 0), three rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-aba}
KNOB=${2:?knob}
for round in 1 2 3; do
  for v in 1 0; do
    env $KNOB=$v timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/ab_${TAG}_${v}_${round}.json 2> gpurun_out/ab_${TAG}_${v}_${round}.err || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/ab_${TAG}_${v}_${round}.json').read().strip().splitlines()[-1])
print('[ab] $KNOB=$v round $round: %.3f ms/step' % d['ms_per_step'])"
  done
done
