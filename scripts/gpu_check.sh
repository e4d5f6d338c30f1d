#!/bin/bash
# One GPU session: parity tests, a short bench, a rocprofv3 kernel-trace of
# the bench.  Stops at the first crash / timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-100}
echo "[gpu_check] $(date) host=$(hostname) nproc=$(nproc)"
lscpu | grep -E 'Model name|^CPU\(s\)' > gpurun_out/host_cpu.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_${TAG}.log
echo "[gpu_check] pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps $STEPS --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?
cat gpurun_out/bench_${TAG}.json; tail -3 gpurun_out/bench_${TAG}.err
echo "[gpu_check] bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err
rc=$?
echo "[gpu_check] rocprof rc=$rc"
find gpurun_out/prof_${TAG} -name '*stats*' | head
[ $rc -eq 0 ] || exit $rc
# HBM traffic of the sweep (both advection kernels): FETCH_SIZE and
# WRITE_SIZE in separate --pmc runs
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'advection_(regular|tiles)' -d gpurun_out/pmc_${TAG}_$c -o run \
      --output-format csv -- python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${TAG}_$c.json 2> gpurun_out/pmc_${TAG}_$c.err
  rc=$?
  echo "[gpu_check] pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python scripts/traffic.py 'advection_(regular|tiles)' gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE \
    --bench-json gpurun_out/pmc_${TAG}_FETCH_SIZE.json > gpurun_out/traffic_${TAG}.json && cat gpurun_out/traffic_${TAG}.json
