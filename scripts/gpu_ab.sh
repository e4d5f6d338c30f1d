#!/bin/bash
# A/B of kernel variants (env-selected) + PMC traffic passes of the defaults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ab}
ADV_VARIANTS=${ADV_VARIANTS:-"1 2"}
for v in $ADV_VARIANTS; do
  DCCRGX_ADV_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline \
     > gpurun_out/${TAG}_adv_v${v}.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_adv_v${v}.json'));r=d['roofline'];print('adv variant $v', '%.3e'%d['value'], 'kernel ms %.4f'%r['kernel_ms_per_step'], 'frac %.3f'%r['frac'])"
done
GOL_VARIANTS=${GOL_VARIANTS:-"1 2"}
for v in $GOL_VARIANTS; do
  DCCRGX_GOL_VARIANT=$v timeout -k 10 300 python -u bench.py --workload gol --steps 50 --warmup 3 > gpurun_out/${TAG}_gol_v${v}.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_gol_v${v}.json'));r=d['roofline'];print('gol variant $v', '%.3e'%d['value'], 'kernel ms %.4f'%r['kernel_ms_per_step'], 'frac %.3f'%r['frac'])"
done
if [ -n "$PMC" ]; then
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/${TAG}_pmc_$c -o run --output-format csv -- \
     python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/${TAG}_pmc_$c.err || exit $?
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/${TAG}_pmcgol_$c -o run --output-format csv -- \
     python -u bench.py --workload gol --steps 10 --warmup 1 > /dev/null 2>gpurun_out/${TAG}_pmcgol_$c.err || exit $?
done
fi
echo done
