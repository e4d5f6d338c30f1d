#!/bin/bash
# N=1 and N=2 adaptive phase tables (net of the transport), plain lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06l}
for n in 1 2; do
  DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus $n --workload advection_adapt --steps 20 \
      --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n$n.json 2> gpurun_out/${TAG}_adapt_n$n.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n$n.json').read().strip().splitlines()[-1]); print('n=$n', round(d['ms_per_step'],3), d['adaptation'])"
  DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 400 python -u bench.py --gpus $n \
      --workload advection_adapt --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n$n.json \
      2> gpurun_out/${TAG}_adapt_pt_n$n.err || exit $?
done
