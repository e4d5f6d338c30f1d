#!/bin/bash
# Adaptive advection at N=2 (host transport, one GPU): phase table with mesh
# notes, and the plain line with the thread- and wave-per-cell remote flags.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06e}
STEPS=${STEPS:-20}
for fw in 0 1; do
  DCCRGX_FLAGS_WAVE=$fw DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus 2 --workload advection_adapt \
      --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n2_fw$fw.json 2> gpurun_out/${TAG}_adapt_n2_fw$fw.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n2_fw$fw.json').read().strip().splitlines()[-1]); print('fw=$fw', round(d['ms_per_step'],3), d['adaptation'])"
done
DCCRGX_MESH_NOTES=1 DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 400 python -u bench.py --gpus 2 \
    --workload advection_adapt --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n2.json \
    2> gpurun_out/${TAG}_adapt_pt_n2.err || exit $?
grep "\[mesh" gpurun_out/${TAG}_adapt_pt_n2.err | tail -4
grep "\[phase" gpurun_out/${TAG}_adapt_pt_n2.err | sort -s -k1,1 | awk '$7 > 0.1 || $1 ~ /comm/'
