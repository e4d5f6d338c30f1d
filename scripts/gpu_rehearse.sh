#!/bin/bash
# Rehearsal of bench.py's N > 1 path on one GPU: `bench.py --gpus N` launches
# its N ranks itself, all on cuda:0 over the library's host exchange (gloo),
# every workload.  Usage: scripts/gpu_rehearse.sh TAG [N]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-reh}
N=${2:-2}
for w in ${WORKLOADS:-advection gol gol_amr poisson scalability advection_adapt}; do
  DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus $N --steps ${STEPS:-5} --warmup 1 --workload $w \
      > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err
  rc=$?
  echo "[rehearse] $w rc=$rc"; tail -c 600 gpurun_out/${TAG}_$w.json; echo
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_$w.err; exit $rc; }
done
