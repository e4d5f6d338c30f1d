#!/bin/bash
# HIP API + kernel trace of a short adaptive run (where the host time between
# kernels goes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ht}
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d gpurun_out/hiptrace_${TAG} -o run --output-format csv -- \
    python -u bench.py --workload advection_adapt --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/hiptrace_${TAG}.json 2> gpurun_out/hiptrace_${TAG}.err || exit $?
ls gpurun_out/hiptrace_${TAG}/*/ 2>/dev/null | head; ls gpurun_out/hiptrace_${TAG} | head
