#!/bin/bash
# GPU test pass: pytest -m gpu (all failures listed), then a short default
# bench.  Usage: scripts/gpu_tests.sh TAG [extra pytest args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02}
shift
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | tail -200 > gpurun_out/pytest_gpu_${TAG}.summary
tail -3 gpurun_out/pytest_gpu_${TAG}.log
echo "[gpu_tests] pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc2=$?
tail -c 3000 gpurun_out/bench_${TAG}.json; tail -3 gpurun_out/bench_${TAG}.err
echo "[gpu_tests] bench rc=$rc2"
exit $rc
