#!/bin/bash
# Rebuild changes at N>1: the transport / multirank / adapt suites, then the
# N=2 adaptive line and its phase table (rebuild sub-phases, list sizes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_multirank.py tests/test_gpu_advection_adapt.py \
    tests/test_gpu_unrefine.py tests/test_gpu_balance.py tests/test_gpu_config5.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus 2 --workload advection_adapt --steps 20 \
    --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n2.json 2> gpurun_out/${TAG}_adapt_n2.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n2.json').read().strip().splitlines()[-1]); print('n=2', round(d['ms_per_step'],3), d['adaptation'])"
DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so DCCRGX_MESH_NOTES=1 timeout -k 10 400 python -u bench.py --gpus 2 \
    --workload advection_adapt --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n2.json \
    2> gpurun_out/${TAG}_adapt_pt_n2.err || exit $?
grep "mesh r0" gpurun_out/${TAG}_adapt_pt_n2.err | tail -2
grep "phase r0" gpurun_out/${TAG}_adapt_pt_n2.err | grep -E "rb\.|sr\.|chk\.|cs\.|adapt\.|comm\."
