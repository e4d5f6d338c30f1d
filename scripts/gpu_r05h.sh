#!/bin/bash
# Round-5 evidence pass: face-table tests, then counters.
#  1. face-neighbor / advection / adaptive tests
#  2. refined GoL: FETCH / WRITE passes (traffic) + SQ / TCC groups
#  3. headline sweep TCC hit / miss, default kernels vs the 3-block regular
#     kernel (DCCRGX_REG3=1), plus their kernel traces
#  4. adaptive step phase table (phase-timing build libdccrgx_pt.so)
# Stops at the first crash / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ref_kats.py tests/test_gpu_neighbors.py tests/test_gpu_advection.py \
    tests/test_gpu_advection_adapt.py -m gpu -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/pmc_traffic.sh $TAG gol_amr || exit $?
KREGEX='lg_(table|game)_kernel' bash scripts/pmc_sq.sh ${TAG}_gola --workload gol_amr || exit $?
for v in 0 1; do
  DCCRGX_REG3=$v KREGEX='advection_(regular|tiles)' bash scripts/pmc_sq.sh ${TAG}_adv_reg3_$v || exit $?
  DCCRGX_REG3=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_adv_reg3_${v}_kt -o run \
      --output-format csv -- python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline \
      > gpurun_out/${TAG}_adv_reg3_${v}_kt.json 2> gpurun_out/${TAG}_adv_reg3_${v}_kt.err || exit $?
  echo "[kt] reg3=$v done"
done
DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 \
    --no-cpu-baseline > gpurun_out/${TAG}_adapt_phases.json 2> gpurun_out/${TAG}_adapt_phases.txt || exit $?
echo "[phases] done"
