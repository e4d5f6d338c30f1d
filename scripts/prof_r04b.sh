#!/bin/bash
# Round-4 evidence set on one box: why tiles are general (reason histogram),
# SQ / TCC / FETCH / WRITE passes of the advection sweep and the refined
# game (prof_r04.sh), and a kernel + RCCL API trace of the one-GPU RCCL
# byte-mover test.  Usage: scripts/prof_r04b.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04m}
DCCRGX_TILE_REASONS=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/${TAG}_reasons.json 2> gpurun_out/${TAG}_reasons.err || exit $?
grep "\[tiles\]" gpurun_out/${TAG}_reasons.err | sort | uniq -c
bash scripts/prof_r04.sh ${TAG}_adv advection advection || exit $?
bash scripts/prof_r04.sh ${TAG}_gola gol_amr "geo_|gol_amr|collect|spread" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --rccl-trace --stats -d gpurun_out/${TAG}_rccl -o run --output-format csv -- \
    python -u -m pytest -x -q tests/test_gpu_rccl_loopback.py > gpurun_out/${TAG}_rccl.log 2>&1 || exit $?
tail -2 gpurun_out/${TAG}_rccl.log
echo "[prof_r04b] done"
