#!/bin/bash
# Selected GPU test files, one pytest process, log under gpurun_out/.
# Usage: scripts/gpu_sel.sh TAG test_file [test_file ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
timeout -k 10 1000 python -u -m pytest "$@" -v --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_${TAG}.log | tail -30
exit $rc
