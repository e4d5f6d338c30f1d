#!/bin/bash
# Stretched geometry file block: library and facade tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06zd}
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid_file.py tests/test_gpu_facade.py tests/test_gpu_transport.py \
    -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR|Error" gpurun_out/pytest_${TAG}.log | head
exit $rc
