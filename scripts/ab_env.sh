#!/bin/bash
# Paired A/B of one environment switch of the product library, interleaved
# per round on one box.
#   bash scripts/ab_env.sh TAG VAR "v0 v1 ..." [rounds] [workload] [pmc]
# prints ms/step, kernel ms/step and roofline frac per run; with pmc=1 also
# TCC hit/miss and FETCH_SIZE passes of the advection kernels per value
# (separate runs, --pmc never combined with tracing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
VAR=$2
VALS=$3
ROUNDS=${4:-3}
WL=${5:-advection}
PMC=${6:-0}
for round in $(seq "$ROUNDS"); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --workload $WL --steps 50 --warmup 3 \
        --no-cpu-baseline > gpurun_out/${TAG}_${v}_$round.json 2> gpurun_out/${TAG}_${v}_$round.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_${v}_$round.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$VAR=$v', '$WL', round(d['ms_per_step'],4), round(r['kernel_ms_per_step'],4), round(r['frac'],3), r.get('kernels_ms', ''))"
  done
done
[ "$PMC" = "0" ] && exit 0
for v in $VALS; do
  for c in "TCC_HIT_sum TCC_MISS_sum" FETCH_SIZE; do
    n=$(echo $c | cut -d' ' -f1)
    export $VAR=$v
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-advection}" \
        -d gpurun_out/${TAG}_pmc_${v}_$n -o run --output-format csv -- \
        python -u bench.py --workload $WL --steps 10 --warmup 1 --no-cpu-baseline > /dev/null \
        2> gpurun_out/${TAG}_pmc_${v}_$n.err || exit $?
    unset $VAR
  done
done
python scripts/pmc_summary.py ${TAG}
echo "[ab_env] done"
