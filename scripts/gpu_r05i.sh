#!/bin/bash
# Full GPU suite, then the adaptive bench line and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05i}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_advection_adapt_${TAG}.json 2> gpurun_out/bench_advection_adapt_${TAG}.err || exit $?
tail -c 500 gpurun_out/bench_advection_adapt_${TAG}.json; echo
bash scripts/gpu_prof.sh $TAG advection_adapt
