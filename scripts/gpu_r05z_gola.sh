#!/bin/bash
# Refined-GoL evidence on the final tree: bench line (with its CPU baseline),
# kernel trace, FETCH / WRITE traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05z}
timeout -k 10 400 python -u bench.py --workload gol_amr > gpurun_out/bench_gol_amr_${TAG}.json \
    2> gpurun_out/bench_gol_amr_${TAG}.err || exit $?
tail -c 400 gpurun_out/bench_gol_amr_${TAG}.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gol_amr_${TAG} -o run --output-format csv -- \
    python -u bench.py --no-cpu-baseline --workload gol_amr --steps 20 --warmup 2 \
    > gpurun_out/bench_prof_gol_amr_${TAG}.json 2> gpurun_out/prof_gol_amr_${TAG}.err || exit $?
bash scripts/pmc_traffic.sh ${TAG} gol_amr || exit $?
