#!/bin/bash
# Kernel stats of the adaptive step with and without the face-table renumbering.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06w}
for v in 1 0; do
  DCCRGX_FACE_REMAP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_remap$v -o run --output-format csv \
      -- python3 -u bench.py --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/${TAG}_remap$v.json 2> gpurun_out/${TAG}_remap$v.err || exit $?
  f=$(find gpurun_out/prof_${TAG}_remap$v -name "*kernel_stats.csv" | head -1)
  echo "remap=$v"; python3 scripts/kstats.py $f 23 12
done
