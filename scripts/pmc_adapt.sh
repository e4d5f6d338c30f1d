#!/bin/bash
# SQ / TCC / HBM counters of the adaptive step's kernels (separate --pmc
# passes), per-dispatch means in gpurun_out/pmc_adapt_<TAG>.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pa}
RE=${2:-'face_table|induced|adv_bands|adv_requests|advection_ell|adv_dt|adv_reset|range_insert|range_clear|kept_children|prefix_fill'}
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$RE" -d gpurun_out/pmca_${TAG}_$i -o run --output-format csv -- \
      python -u bench.py --workload advection_adapt --steps 5 --warmup 1 --no-cpu-baseline \
      > gpurun_out/pmca_${TAG}_$i.json 2> gpurun_out/pmca_${TAG}_$i.err
  rc=$?
  echo "[pmc] pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python - "$TAG" > gpurun_out/pmc_adapt_${TAG}.txt <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob('gpurun_out/pmca_%s_*/run_counter_collection.csv' % tag)):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)', 'anon').split('(')[0].split('<')[0].split('::')[-1]
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k in sorted(acc):
    print(k, {c: '%.4g' % (sum(v) / len(v)) for c, v in sorted(acc[k].items())})
PY
cat gpurun_out/pmc_adapt_${TAG}.txt
