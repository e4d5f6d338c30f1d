#!/bin/bash
# Distributed adaptive step: correctness tests, N=1 / N=2 lines, N=2 phase
# table and per-rank kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06h}
STEPS=${STEPS:-20}
timeout -k 10 600 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_multirank.py tests/test_gpu_advection_adapt.py \
    tests/test_gpu_unrefine.py tests/test_gpu_balance.py tests/test_gpu_config5.py tests/test_gpu_advection.py tests/test_gpu_gol_amr.py tests/test_gpu_rccl_loopback.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head
[ $rc -eq 0 ] || exit $rc
for n in 1 2; do
  DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus $n --workload advection_adapt --steps $STEPS \
      --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_n$n.json 2> gpurun_out/${TAG}_adapt_n$n.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_adapt_n$n.json').read().strip().splitlines()[-1]); print('n=$n', round(d['ms_per_step'],3), d['adaptation'])"
  DCCRG_BENCH_TRANSPORT=host DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 400 python -u bench.py --gpus $n \
      --workload advection_adapt --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_adapt_pt_n$n.json \
      2> gpurun_out/${TAG}_adapt_pt_n$n.err || exit $?
done
bash scripts/prof_ranks.sh ${TAG}_n2 2 --workload advection_adapt --steps $STEPS --warmup 3 --no-cpu-baseline > /dev/null || exit $?
python scripts/kstats.py gpurun_out/profranks_${TAG}_n2/rank0/run_kernel_stats.csv 23 25
DCCRG_BENCH_TRANSPORT=host timeout -k 10 400 python -u bench.py --gpus 2 --workload gol_amr --steps 20 --warmup 2 \
    > gpurun_out/${TAG}_gola_n2.json 2> gpurun_out/${TAG}_gola_n2.err || { tail -20 gpurun_out/${TAG}_gola_n2.err; exit 1; }
tail -c 1500 gpurun_out/${TAG}_gola_n2.json
