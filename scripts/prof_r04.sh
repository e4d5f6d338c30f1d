#!/bin/bash
# Round-4 profile set: kernel trace + stats of one bench workload, then its
# SQ / TCC counter passes (one rocprofv3 --pmc run per group, kernel trace
# only).  Usage: scripts/prof_r04.sh TAG WORKLOAD KERNEL_REGEX [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
W=$2
RE=$3
shift 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o run --output-format csv -- \
    python -u bench.py --workload $W --steps 20 --warmup 2 --no-cpu-baseline "$@" \
    > gpurun_out/${TAG}_kt.json 2> gpurun_out/${TAG}_kt.err || exit $?
echo "[prof] kernel trace done"
k=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "$RE" -d gpurun_out/${TAG}_pmc$k -o run \
      --output-format csv -- python -u bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline "$@" \
      > /dev/null 2> gpurun_out/${TAG}_pmc$k.err || exit $?
  echo "[prof] pmc $k done"
done
