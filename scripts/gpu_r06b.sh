#!/bin/bash
# send_single_cells guard tests + tile ext-list statistics of config 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl_loopback.py tests/test_gpu_transport.py -v --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DCCRGX_TILE_REASONS=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/tiles_${TAG}.json 2> gpurun_out/tiles_${TAG}.err
rc=$?; grep "\[tiles\]" gpurun_out/tiles_${TAG}.err; exit $rc
