#!/bin/bash
# Face table, one pass over face_predict (DCCRGX_FACE_MISS=0 selected it while the
# two-pass form of r06zh existed): paired adaptive lines and the kernel stats.
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2 3; do
  for lib in libdccrgx_old.so libdccrgx.so; do
    DCCRGX_FACE_MISS=0 DCCRGX_LIB=$lib timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06zi_${lib}_${rep}.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/r06zi_${lib}_${rep}.json').read().strip().splitlines()[-1]); print('$lib rep $rep', round(d['ms_per_step'],4))"
  done
done
DCCRGX_FACE_MISS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06zi_prof -o run --output-format csv -- python3 bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2>&1 || exit 1
