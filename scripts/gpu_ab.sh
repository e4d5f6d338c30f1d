#!/bin/bash
# A/B of kernel configurations (env assignments, ';'-separated in CONFIGS)
# + PMC passes on PMC_CONFIGS (one counter group per run; --pmc is never
# combined with tracing options).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab}
WORKLOAD=${WORKLOAD:-advection}
IFS=';' read -ra CFGS <<< "${CONFIGS:-DCCRGX_ADV_VARIANT=11}"
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python -u bench.py --workload $WORKLOAD --steps 50 --warmup 3 --no-cpu-baseline \
     > gpurun_out/${TAG}_c$i.json 2>gpurun_out/${TAG}_c$i.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c$i.json'));r=d['roofline'];print('[$cfg]', '%.3e'%d['value'], 'kernel ms %.4f'%r['kernel_ms_per_step'], 'frac %.3f'%r['frac'])"
done
IFS=';' read -ra PCFGS <<< "${PMC_CONFIGS:-}"
j=0
for cfg in "${PCFGS[@]}"; do
  j=$((j+1))
  k=0
  for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    k=$((k+1))
    env $cfg timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-advection}" \
       -d gpurun_out/${TAG}_pmc${j}_$k -o run --output-format csv -- \
       python -u bench.py --workload $WORKLOAD --steps 10 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/${TAG}_pmc${j}_$k.err || exit $?
  done
done
echo done
