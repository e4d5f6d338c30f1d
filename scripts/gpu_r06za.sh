#!/bin/bash
# Kernel trace of the adaptive step (step breakdown) and its plain line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06za}
timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/${TAG}_adapt_n1.json 2> gpurun_out/${TAG}_adapt_n1.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n1.json').read().strip().splitlines()[-1]); print('n=1', round(d['ms_per_step'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv \
    -- python3 -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || exit $?
python3 scripts/step_breakdown.py gpurun_out/prof_${TAG}/run_kernel_trace.csv adv_reset 3 30
