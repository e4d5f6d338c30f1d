#!/bin/bash
# A/B of kernel variants (env-selected) + PMC passes (one counter group per
# run, --kernel-trace/--stats never combined with --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab}
ADV_VARIANTS=${ADV_VARIANTS:-"3"}
for v in $ADV_VARIANTS; do
  DCCRGX_ADV_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline \
     > gpurun_out/${TAG}_adv_v${v}.json 2>gpurun_out/${TAG}_adv_v${v}.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_adv_v${v}.json'));r=d['roofline'];print('adv variant $v', '%.3e'%d['value'], 'kernel ms %.4f'%r['kernel_ms_per_step'], 'frac %.3f'%r['frac'])"
done
GOL_VARIANTS=${GOL_VARIANTS:-""}
for v in $GOL_VARIANTS; do
  DCCRGX_GOL_VARIANT=$v timeout -k 10 300 python -u bench.py --workload gol --steps 50 --warmup 3 > gpurun_out/${TAG}_gol_v${v}.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_gol_v${v}.json'));r=d['roofline'];print('gol variant $v', '%.3e'%d['value'], 'kernel ms %.4f'%r['kernel_ms_per_step'], 'frac %.3f'%r['frac'])"
done
PMC_VARIANTS=${PMC_VARIANTS:-""}
i=0
for v in $PMC_VARIANTS; do
  for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    DCCRGX_ADV_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex advection_kernel \
       -d gpurun_out/${TAG}_pmc_v${v}_$i -o run --output-format csv -- \
       python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/${TAG}_pmc_v${v}_$i.err || exit $?
  done
done
echo done
