#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06g}
bash scripts/prof_ranks.sh ${TAG}_n2 2 --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline || exit $?
DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 400 python -u bench.py --gpus 2 \
    --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n2.json \
    2> gpurun_out/${TAG}_adapt_pt_n2.err || exit $?
grep "\[phase r0" gpurun_out/${TAG}_adapt_pt_n2.err | awk '$7 > 0.05 || $2 ~ /comm/'
