#!/bin/bash
# Evidence on one GPU: the GPU test suite, every bench line, rocprofv3
# kernel-trace stats of the bench lines.  Stops at the first crash / hang.
# Usage: scripts/gpu_round.sh TAG [skip-tests|tests] [pmc]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02}
echo "[round] $(date) host=$(hostname) nproc=$(nproc)"
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
run() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > gpurun_out/bench_${n}_${TAG}.json 2> gpurun_out/bench_${n}_${TAG}.err
  local r=$?
  echo "[round] bench $n rc=$r"; tail -c 1500 gpurun_out/bench_${n}_${TAG}.json; echo
  [ $r -eq 0 ] || { tail -5 gpurun_out/bench_${n}_${TAG}.err; exit $r; }
}
run advection 600
run gol 400 --workload gol
run gol_amr 400 --workload gol_amr
run poisson 500 --workload poisson --steps 200
run scalability 600 --workload scalability --steps 20
run advection_adapt 600 --workload advection_adapt --steps 20 --warmup 3
prof() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${n}_${TAG} -o run --output-format csv -- \
      python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_prof_${n}_${TAG}.json 2> gpurun_out/prof_${n}_${TAG}.err
  local r=$?
  echo "[round] rocprof $n rc=$r"
  [ $r -eq 0 ] || exit $r
}
prof advection 600 --steps 20 --warmup 2
prof gol 400 --workload gol --steps 20 --warmup 2
prof gol_amr 400 --workload gol_amr --steps 20 --warmup 2
prof poisson 500 --workload poisson --steps 50 --warmup 2
[ "$3" = "pmc" ] && { bash scripts/pmc_traffic.sh ${TAG} advection gol gol_amr poisson scalability || exit $?; }
echo "[round] done $(date)"
