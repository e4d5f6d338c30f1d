#!/bin/bash
# Fewer stream syncs in the adaptive step: the suites it touches, the N=1 / N=2
# lines, the N=1 sync counts per lap.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06y}
timeout -k 10 700 python -u -m pytest tests/test_gpu_advection_adapt.py tests/test_gpu_advection.py tests/test_gpu_transport.py \
    tests/test_gpu_multirank.py tests/test_gpu_unrefine.py tests/test_gpu_balance.py tests/test_gpu_ref_advection.py \
    tests/test_gpu_variable.py tests/test_gpu_facade.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
for n in 1 2; do
  DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus $n --workload advection_adapt --steps 20 \
      --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n$n.json 2> gpurun_out/${TAG}_adapt_n$n.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n$n.json').read().strip().splitlines()[-1]); print('n=$n', round(d['ms_per_step'],3), d['adaptation'])"
done
DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 10 --warmup 3 \
    --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n1.json 2> gpurun_out/${TAG}_adapt_pt_n1.err || exit $?
grep "phase r0" gpurun_out/${TAG}_adapt_pt_n1.err | grep -E "syncs|pool"
