#!/bin/bash
# Stream syncs per lap of the one-process adaptive step (phase-timing build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06x}
DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 10 --warmup 3 \
    --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n1.json 2> gpurun_out/${TAG}_adapt_pt_n1.err || exit $?
grep "phase r0" gpurun_out/${TAG}_adapt_pt_n1.err | grep -E "syncs|pool"
