#!/bin/bash
# HBM traffic per step of each bench workload's kernels: FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes, then scripts/traffic.py writes
# gpurun_out/<workload>_traffic_<TAG>.json (copied to profiles/ by hand).
# Usage: scripts/pmc_traffic.sh TAG [workload ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02}
shift
WORKLOADS=${*:-advection gol gol_amr poisson}
for w in $WORKLOADS; do
  case $w in
    advection) re='advection_(regular|tiles)'; args="--steps 10 --warmup 1" ;;
    gol) re='gol_structured'; args="--workload gol --steps 10 --warmup 1" ;;
    scalability) re='gol_structured'; args="--workload scalability --steps 10 --warmup 1" ;;
    gol_amr) re='lg_(table|game)_kernel|gol_amr_spread|geo_collect'; args="--workload gol_amr --steps 10 --warmup 1" ;;
    poisson) re='po_(phase|reduce)'; args="--workload poisson --steps 10 --warmup 1" ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "$re" -d gpurun_out/pmc_${w}_${TAG}_$c -o run \
        --output-format csv -- python -u bench.py $args --no-cpu-baseline \
        > gpurun_out/pmc_${w}_${TAG}_$c.json 2> gpurun_out/pmc_${w}_${TAG}_$c.err
    rc=$?
    echo "[pmc] $w $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python scripts/traffic.py $w "$re" gpurun_out/pmc_${w}_${TAG}_FETCH_SIZE gpurun_out/pmc_${w}_${TAG}_WRITE_SIZE \
      --bench-json gpurun_out/pmc_${w}_${TAG}_FETCH_SIZE.json > gpurun_out/${w}_traffic_${TAG}.json \
      && cat gpurun_out/${w}_traffic_${TAG}.json
done
