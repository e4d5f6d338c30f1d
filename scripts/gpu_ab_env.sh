#!/bin/bash
# Paired A/B of an environment switch on the headline bench, alternating.
# Usage: scripts/gpu_ab_env.sh TAG VAR rounds [workload]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; VAR=$2; N=${3:-3}; W=${4:-advection}
for i in $(seq 1 $N); do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --workload $W --steps 40 --warmup 3 --no-cpu-baseline \
        > gpurun_out/ab_${TAG}_${v}_${i}.json 2> gpurun_out/ab_${TAG}_${v}_${i}.err || exit $?
    python - "$v" "$i" gpurun_out/ab_${TAG}_${v}_${i}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(f"[ab] {sys.argv[1]} round {sys.argv[2]}: ms/step {d['ms_per_step']:.4f} kernel {d['roofline']['kernel_ms_per_step']:.4f} frac {d['roofline']['frac']:.4f}")
PY
  done
done
