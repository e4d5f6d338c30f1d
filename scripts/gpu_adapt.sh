#!/bin/bash
# Adaptive-step iteration: the face / advection / adaptation / KAT tests,
# the adaptive bench line, its kernel trace and the per-step breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-adapt}
timeout -k 10 700 python -u -m pytest tests/test_gpu_ref_kats.py tests/test_gpu_neighbors.py tests/test_gpu_advection.py \
    tests/test_gpu_advection_adapt.py tests/test_gpu_ref_advection.py tests/test_gpu_unrefine.py tests/test_gpu_mapping.py \
    -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log
grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_advection_adapt_${TAG}.json 2> gpurun_out/bench_advection_adapt_${TAG}.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/bench_advection_adapt_${TAG}.json').read().strip().splitlines()[-1])
print('[adapt] %.3f ms/step sweep %.3f created %d removed %d' % (d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['adaptation']['created_total'], d['adaptation']['removed_total']))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_adapt_${TAG} -o run --output-format csv -- \
    python -u bench.py --workload advection_adapt --steps 20 --warmup 2 --no-cpu-baseline \
    > gpurun_out/prof_adapt_${TAG}.json 2> gpurun_out/prof_adapt_${TAG}.err || exit $?
python scripts/step_breakdown.py gpurun_out/prof_adapt_${TAG}/run_kernel_trace.csv advection_ell 2 30
