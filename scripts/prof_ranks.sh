#!/bin/bash
# rocprofv3 kernel-trace stats of a bench.py run at N ranks on one GPU (host
# transport), every rank under its own rocprofv3 started from this shell
# (which never touches the GPU).  Usage: scripts/prof_ranks.sh TAG N bench-args...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
OUT=gpurun_out/profranks_${TAG}
rm -rf $OUT; mkdir -p $OUT
port=$((29700 + RANDOM % 200))
pids=()
for r in $(seq 0 $((N - 1))); do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$port DCCRG_BENCH_TRANSPORT=host \
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/rank$r -o run --output-format csv -- \
      python -u bench.py --gpus $N "$@" > $OUT/rank$r.json 2> $OUT/rank$r.err &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
echo "[prof_ranks] rc=$rc"
[ $rc -eq 0 ] || exit $rc
for r in $(seq 0 $((N - 1))); do
  echo "== rank $r"; head -25 $OUT/rank$r/run_kernel_stats.csv | cut -c1-200
done
