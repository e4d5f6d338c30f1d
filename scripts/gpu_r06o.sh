#!/bin/bash
# N=2 adaptive step, phase-timing build with the rebuild's list sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06o}
DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so DCCRGX_MESH_NOTES=1 timeout -k 10 400 python -u bench.py --gpus 2 \
    --workload advection_adapt --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n2.json \
    2> gpurun_out/${TAG}_adapt_pt_n2.err || exit $?
grep "mesh r0" gpurun_out/${TAG}_adapt_pt_n2.err | tail -4
