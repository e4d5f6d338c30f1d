#!/bin/bash
# Round-end evidence on one GPU: full GPU test suite, default bench
# (advection, the BASELINE metric) and the other workload lines, rocprofv3
# kernel-trace stats of the advection and game-of-life benches, PMC traffic.
# Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
echo "[round] $(date) host=$(hostname)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_${TAG}.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
cat gpurun_out/bench_${TAG}.json
for w in gol gol_amr poisson; do
  timeout -k 10 600 python -u bench.py --workload $w $( [ $w = poisson ] && echo "--steps 200" ) \
      > gpurun_out/bench_${w}_${TAG}.json 2> gpurun_out/bench_${w}_${TAG}.err || exit $?
  echo "[round] bench $w done"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gol_${TAG} -o run --output-format csv -- \
    python -u bench.py --workload gol --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_gol_${TAG}.json 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_po_${TAG} -o run --output-format csv -- \
    python -u bench.py --workload poisson --steps 50 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_po_${TAG}.json 2>&1 || exit $?
bash scripts/pmc_traffic.sh ${TAG}
