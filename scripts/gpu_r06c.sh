#!/bin/bash
# Neighbor records: parity tests, paired A/B (DCCRGX_NBREC=0/1) with TCC
# counters, kernel stats of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06c}
timeout -k 10 700 python -u -m pytest tests/test_gpu_advection.py tests/test_gpu_config_full.py \
    tests/test_gpu_ref_advection.py tests/test_gpu_transport.py tests/test_gpu_advection_adapt.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh ${TAG}_ab DCCRGX_NBREC "0 1" 3 advection 1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err
rc=$?; echo "[r06c] rocprof rc=$rc"; cat gpurun_out/prof_${TAG}/run_kernel_stats.csv | head -12
