#!/bin/bash
# SQ / LDS / cache counters of the advection sweep kernels (one --pmc pass
# per counter group, kernel trace only).  Usage: scripts/pmc_sq.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-sq}
shift
k=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-advection_(regular|tiles)}" \
     -d gpurun_out/${TAG}_pmc$k -o run --output-format csv -- \
     python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2>gpurun_out/${TAG}_pmc$k.err || exit $?
  echo "[pmc $k] done"
done
