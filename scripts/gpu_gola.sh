#!/bin/bash
# Refined-GoL iteration: its tests, then the bench line paired A/B of an
# environment knob (KNOB=0 / default), two rounds, and the kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-gola}
KNOB=${2:-DCCRGX_LG_COUNT}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gol_amr.py tests/test_gpu_ref_gol_amr.py tests/test_gpu_gol.py \
    tests/test_gpu_advection_adapt.py tests/test_gpu_ref_kats.py -m gpu -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log
grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for round in 1 2; do
  for v in 1 0; do
    env $KNOB=$v timeout -k 10 300 python -u bench.py --workload gol_amr --steps 50 --warmup 3 --no-cpu-baseline \
        > gpurun_out/ab_${TAG}_${v}_${round}.json 2> gpurun_out/ab_${TAG}_${v}_${round}.err || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/ab_${TAG}_${v}_${round}.json').read().strip().splitlines()[-1])
print('[ab] $KNOB=$v round $round: %.4f ms/step, kernels %.4f ms' % (d['ms_per_step'], d['roofline']['kernel_ms_per_step']))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gola_${TAG} -o run --output-format csv -- \
    python -u bench.py --workload gol_amr --steps 20 --warmup 2 --no-cpu-baseline \
    > gpurun_out/prof_gola_${TAG}.json 2> gpurun_out/prof_gola_${TAG}.err || exit $?
python scripts/step_breakdown.py gpurun_out/prof_gola_${TAG}/run_kernel_trace.csv lg_table 2 12
# the adaptive step's phase table from the phase-timing build, when present
if [ -f dccrg_amd/libdccrgx_pt.so ]; then
  DCCRGX_LIB=libdccrgx_pt.so timeout -k 10 300 python -u bench.py --workload advection_adapt --steps 20 --warmup 3 \
      --no-cpu-baseline > gpurun_out/${TAG}_adapt_phases.json 2> gpurun_out/${TAG}_adapt_phases.txt || exit $?
  grep phase gpurun_out/${TAG}_adapt_phases.txt | sort -k4 -n -r | head -25
fi
