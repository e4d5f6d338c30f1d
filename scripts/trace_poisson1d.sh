#!/bin/bash
# HIP API + kernel + memory-copy trace of the 3-process Poisson 1-D case
# (scripts/trace_poisson1d.py), every rank under its own rocprofv3 (started
# from this shell, which never touches the GPU).  Then the census of calls
# per stream (scripts/stream_census.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06}
W=${W:-3}
OUT=gpurun_out/trace_po1d_${TAG}
rm -rf $OUT; mkdir -p $OUT
port=$((29600 + RANDOM % 200))
pids=()
for r in $(seq 0 $((W - 1))); do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=$W MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
    timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $OUT/rank$r -o run \
      --output-format csv -- python -u scripts/trace_poisson1d.py > $OUT/rank$r.out 2> $OUT/rank$r.err &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
cat $OUT/rank0.out
echo "[trace_poisson1d] rc=$rc"
[ $rc -eq 0 ] || exit $rc
python scripts/stream_census.py $OUT > $OUT/census.txt && cat $OUT/census.txt
