#!/bin/bash
# Rebuild lists in one device pass: the N>1 suites, the N=2 / N=1 adaptive lines,
# the N=2 rebuild laps and their sync counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06zb}
timeout -k 10 800 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_multirank.py tests/test_gpu_advection_adapt.py \
    tests/test_gpu_unrefine.py tests/test_gpu_balance.py tests/test_gpu_config5.py tests/test_gpu_variable.py \
    tests/test_gpu_facade.py tests/test_gpu_user_hood.py tests/test_gpu_gol_amr.py tests/test_gpu_neighbors.py \
    -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
for n in 2 1; do
  DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus $n --workload advection_adapt --steps 20 \
      --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n$n.json 2> gpurun_out/${TAG}_adapt_n$n.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n$n.json').read().strip().splitlines()[-1]); print('n=$n', round(d['ms_per_step'],3), d['adaptation'])"
done
DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 400 python -u bench.py --gpus 2 \
    --workload advection_adapt --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n2.json \
    2> gpurun_out/${TAG}_adapt_pt_n2.err || exit $?
grep "phase r0" gpurun_out/${TAG}_adapt_pt_n2.err | grep -E "rb\.|sr\.7"
