#!/bin/bash
# Full GPU suite, then bench lines, then kernel-trace profiles; stops on a
# crash / timeout (test failures do not stop it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in gol_amr advection_adapt advection; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/bench_${w}_${TAG}.json 2> gpurun_out/bench_${w}_${TAG}.err
  r=$?
  echo "[r05] bench $w rc=$r"; tail -c 700 gpurun_out/bench_${w}_${TAG}.json; echo
  [ $r -eq 0 ] || { tail -5 gpurun_out/bench_${w}_${TAG}.err; exit $r; }
done
bash scripts/gpu_prof.sh $TAG gol_amr advection_adapt
