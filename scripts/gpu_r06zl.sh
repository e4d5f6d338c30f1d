#!/bin/bash
# Face table: the three levels' range-map entries of an open direction loaded together
# (face_dir_rmap): the suites that build the table, paired adaptive lines
# (libdccrgx_old.so = the previous tree), and the sweep kernel's duration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06zl}
[ -n "$SKIP_TESTS" ] || timeout -k 10 700 python -u -m pytest tests/test_gpu_advection.py tests/test_gpu_advection_adapt.py tests/test_gpu_neighbors.py tests/test_gpu_ref_advection.py \
    tests/test_gpu_unrefine.py tests/test_gpu_multirank.py tests/test_gpu_balance.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
for rep in ${REPS:-1 2 3}; do
  for lib in libdccrgx_old.so libdccrgx.so; do
    DCCRGX_LIB=$lib timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/${TAG}_${lib}_${rep}.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_${lib}_${rep}.json').read().strip().splitlines()[-1]); print('$lib rep $rep', round(d['ms_per_step'],4))"
  done
done
for lib in libdccrgx_old.so libdccrgx.so; do
  DCCRGX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_${lib} -o run --output-format csv -- \
      python3 bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/${TAG}_prof_${lib} -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; grep -E "face_table|face_fine" "$f" | cut -d, -f1-4
done
