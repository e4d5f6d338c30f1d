#!/bin/bash
# HIP API + kernel trace of the adaptive step on one GPU (gap analysis).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06m}
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d gpurun_out/hiptrace_${TAG} -o run \
    --output-format csv -- python -u bench.py --workload advection_adapt --steps 12 --warmup 2 --no-cpu-baseline \
    > gpurun_out/hiptrace_${TAG}.json 2> gpurun_out/hiptrace_${TAG}.err || exit $?
ls gpurun_out/hiptrace_${TAG}
