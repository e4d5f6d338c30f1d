#!/bin/bash
# N=2 adaptive: transport tests, near-filter A/B, phase table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06f}
STEPS=${STEPS:-20}
timeout -k 10 600 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_multirank.py tests/test_gpu_advection_adapt.py \
    tests/test_gpu_unrefine.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
for nf in 0 1; do
  DCCRGX_NEAR_FILTER=$nf DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus 2 --workload advection_adapt \
      --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n2_nf$nf.json 2> gpurun_out/${TAG}_adapt_n2_nf$nf.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n2_nf$nf.json').read().strip().splitlines()[-1]); print('nf=$nf', round(d['ms_per_step'],3), d['adaptation'])"
done
DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 400 python -u bench.py --gpus 2 \
    --workload advection_adapt --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n2.json \
    2> gpurun_out/${TAG}_adapt_pt_n2.err || exit $?
grep "\[phase" gpurun_out/${TAG}_adapt_pt_n2.err | sort -s -k1,1 | awk '$7 > 0.1 || $2 ~ /comm/'
