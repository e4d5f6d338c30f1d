#!/bin/bash
# Full GPU suite; adaptive bench with the LDS-staged table sweep on / off
# (paired, two rounds); headline and refined-GoL lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05j}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for round in 1 2; do
  for v in 1 0; do
    DCCRGX_ELL_LDS=$v timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 \
        --no-cpu-baseline > gpurun_out/ab_ell_${TAG}_${v}_${round}.json 2> gpurun_out/ab_ell_${TAG}_${v}_${round}.err || exit $?
    python - "$v" "$round" gpurun_out/ab_ell_${TAG}_${v}_${round}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print("[ab] ell_lds=%s round %s: %.3f ms/step, sweep %.3f ms" % (sys.argv[1], sys.argv[2], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"]))
PY
  done
done
for w in advection gol_amr; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/bench_${w}_${TAG}.json 2> gpurun_out/bench_${w}_${TAG}.err || exit $?
  tail -c 300 gpurun_out/bench_${w}_${TAG}.json; echo
done
