#!/bin/bash
# Adaptive step kernel trace on the final tree (for scripts/step_breakdown.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06zk}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
    python3 bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt.json 2> gpurun_out/${TAG}_adapt.err
