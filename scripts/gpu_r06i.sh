#!/bin/bash
# General-tile faces evaluated once: parity tests, paired A/B (DCCRGX_FACE_ONCE=0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06i}
timeout -k 10 700 python -u -m pytest tests/test_gpu_advection.py tests/test_gpu_config_full.py \
    tests/test_gpu_ref_advection.py tests/test_gpu_advection_adapt.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh ${TAG}_ab DCCRGX_FACE_ONCE "0 1" 3 advection 1 || exit $?
