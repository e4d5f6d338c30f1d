#!/bin/bash
# Round-6 GPU session: null-stream ordering probe, the GPU suite, the default
# bench line, bench.py --gpus 2 launching its own ranks (host transport on one
# GPU), the 3-process Poisson 1-D trace.  Stops at the first crash / hang.
# Usage: scripts/gpu_r06.sh TAG [skip-tests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06}
echo "[r06] $(date) host=$(hostname)"
timeout -k 10 180 scripts/microbench/null_stream_order 100 > gpurun_out/null_stream_order_${TAG}.txt 2>&1
rc=$?; cat gpurun_out/null_stream_order_${TAG}.txt; [ $rc -eq 0 ] || exit $rc
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_gpu_${TAG}.log
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | head -20
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 100 --warmup 5 > gpurun_out/bench_advection_${TAG}.json 2> gpurun_out/bench_advection_${TAG}.err
rc=$?; echo "[r06] bench rc=$rc"; cat gpurun_out/bench_advection_${TAG}.json; [ $rc -eq 0 ] || exit $rc
DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus 2 --workload advection --steps 20 --warmup 2 \
    --no-cpu-baseline > gpurun_out/bench_n2host_${TAG}.json 2> gpurun_out/bench_n2host_${TAG}.err
rc=$?; echo "[r06] n2 host rc=$rc"; cat gpurun_out/bench_n2host_${TAG}.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_n2host_${TAG}.err; exit $rc; }
scripts/trace_poisson1d.sh $TAG
