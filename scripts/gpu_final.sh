#!/bin/bash
# Final evidence of a round on one GPU: the GPU suite, smoke, every bench line
# with its CPU baseline, rocprofv3 kernel stats, then the N=2 rehearsal of
# every workload through bench.py's own launcher.  Stops at the first crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06z}
bash scripts/gpu_round.sh $TAG || exit $?
STEPS=10 bash scripts/gpu_rehearse.sh ${TAG}_rehearse_n2 2 || exit $?
echo "[final] done"
