#!/bin/bash
# Round-5 GPU pass: the whole GPU suite (one process), then the named bench
# workloads.  Stops at the first crash / timeout.
# Usage: scripts/gpu_r05.sh TAG [workload ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in "$@"; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/bench_${w}_${TAG}.json 2> gpurun_out/bench_${w}_${TAG}.err
  r=$?
  echo "[r05] bench $w rc=$r"; tail -c 1200 gpurun_out/bench_${w}_${TAG}.json; echo
  [ $r -eq 0 ] || { tail -5 gpurun_out/bench_${w}_${TAG}.err; exit $r; }
done
exit $rc
