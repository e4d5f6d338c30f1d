#!/bin/bash
# GoL rows-per-wave A/B: parity of the variants, then paired bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06ze}
for v in "2 2" "2 3" "4 1" "4 2"; do
  set -- $v
  DCCRGX_GOL_YR=$1 DCCRGX_GOL_YDEPTH=$2 timeout -k 10 300 python -u -m pytest tests/test_gpu_gol.py tests/test_gpu_multirank.py \
      -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_${TAG}_yr$1_d$2.log 2>&1 || { tail -20 gpurun_out/pytest_${TAG}_yr$1_d$2.log; exit 1; }
  echo "yr=$1 d=$2 $(tail -1 gpurun_out/pytest_${TAG}_yr$1_d$2.log)"
done
for rep in 1 2; do
  for v in "1 2" "2 2" "2 3" "4 1" "4 2"; do
    set -- $v
    DCCRGX_GOL_YR=$1 DCCRGX_GOL_YDEPTH=$2 timeout -k 10 200 python -u bench.py --workload gol --steps 50 --warmup 5 \
        --no-cpu-baseline > gpurun_out/${TAG}_gol_yr$1_d$2_$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_gol_yr$1_d$2_$rep.json').read().strip().splitlines()[-1]); print('yr=$1 d=$2 rep $rep', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done
