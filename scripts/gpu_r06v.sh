#!/bin/bash
# Face-table renumbering: adaptive / advection / transport suites, N=1 and N=2
# adaptive lines and phase tables.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06v}
timeout -k 10 700 python -u -m pytest tests/test_gpu_advection_adapt.py tests/test_gpu_advection.py tests/test_gpu_transport.py \
    tests/test_gpu_multirank.py tests/test_gpu_unrefine.py tests/test_gpu_balance.py tests/test_gpu_ref_advection.py \
    tests/test_gpu_poisson.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
for n in 1 2; do
  DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus $n --workload advection_adapt --steps 20 \
      --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n$n.json 2> gpurun_out/${TAG}_adapt_n$n.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n$n.json').read().strip().splitlines()[-1]); print('n=$n', round(d['ms_per_step'],3), d['adaptation'])"
  DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 400 python -u bench.py --gpus $n \
      --workload advection_adapt --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n$n.json \
      2> gpurun_out/${TAG}_adapt_pt_n$n.err || exit $?
done
DCCRGX_FACE_REMAP=0 timeout -k 10 400 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/${TAG}_adapt_n1_noremap.json 2> gpurun_out/${TAG}_adapt_n1_noremap.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n1_noremap.json').read().strip().splitlines()[-1]); print('n=1 no remap', round(d['ms_per_step'],3))"
grep "phase r0" gpurun_out/${TAG}_adapt_pt_n1.err | grep -E "face|step\.|chk\.2a|adapt\.|rb\.6|sr\.7"
grep "phase r0" gpurun_out/${TAG}_adapt_pt_n2.err | grep -E "face|sr\.7|rb\.6"
