#!/bin/bash
# rocprofv3 kernel-trace stats of bench workloads (one run each).
# Usage: scripts/gpu_prof.sh TAG workload [workload ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
for w in "$@"; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${w}_${TAG} -o run --output-format csv -- \
      python -u bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline \
      > gpurun_out/bench_prof_${w}_${TAG}.json 2> gpurun_out/prof_${w}_${TAG}.err
  r=$?
  echo "[prof] $w rc=$r"; tail -c 600 gpurun_out/bench_prof_${w}_${TAG}.json; echo
  [ $r -eq 0 ] || { tail -5 gpurun_out/prof_${w}_${TAG}.err; exit $r; }
done
