#!/bin/bash
# Config-5 shape and config 2: structured GoL z-chunk A/B (DCCRGX_G3_ZC), two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2; do
  for zc in 64 128 32; do
    for w in scalability gol; do
      DCCRGX_G3_ZC=$zc timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline \
          > gpurun_out/abzc_${w}_${zc}_${round}.json 2> gpurun_out/abzc_${w}_${zc}_${round}.err || exit $?
      python -c "
import json; d=json.loads(open('gpurun_out/abzc_${w}_${zc}_${round}.json').read().strip().splitlines()[-1])
print('[ab] $w zc=$zc round $round: %.4f ms/step' % d['ms_per_step'])"
    done
  done
done
