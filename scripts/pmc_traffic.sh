#!/bin/bash
# HBM traffic of the advection sweep (both kernels): FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes, then scripts/traffic.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'advection_(regular|tiles|fused)' -d gpurun_out/pmc_${TAG}_$c -o run \
      --output-format csv -- python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$c.json 2> gpurun_out/pmc_${TAG}_$c.err
  rc=$?
  echo "[pmc] $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python scripts/traffic.py 'advection_(regular|tiles|fused)' gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE \
    --bench-json gpurun_out/pmc_${TAG}_FETCH_SIZE.json > gpurun_out/traffic_${TAG}.json && cat gpurun_out/traffic_${TAG}.json
