#!/bin/bash
# Paired A/B of in-tree library builds (dccrg_amd/libdccrgx_<v>.so, built
# here with dccrg_amd/build.py out=/defines=), interleaved per round on one
# box; the product build dccrg_amd/libdccrgx.so is never touched.
#   bash scripts/ab_libs.sh TAG "a b" [rounds] [workload] [pmc]
# prints ms/step, kernel ms/step and roofline frac per run; with pmc=1 also
# a rocprofv3 kernel-trace stats pass and FETCH_SIZE / WRITE_SIZE passes per
# variant (separate runs, --pmc never combined with tracing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
VARS=${2:-"a b"}
ROUNDS=${3:-2}
WL=${4:-advection}
PMC=${5:-0}
for round in $(seq "$ROUNDS"); do
  for v in $VARS; do
    DCCRGX_LIB=libdccrgx_$v.so timeout -k 10 300 python -u bench.py --workload $WL --steps 50 --warmup 3 \
        --no-cpu-baseline > gpurun_out/${TAG}_${v}_$round.json 2> gpurun_out/${TAG}_${v}_$round.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_${v}_$round.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', '$WL', round(d['ms_per_step'],4), round(r['kernel_ms_per_step'],4), round(r['frac'],3), r.get('kernels_ms', ''))"
  done
done
# pmc: 0 none, 1 kernel stats + PMC passes, 2 kernel stats only
[ "$PMC" = "0" ] && exit 0
for v in $VARS; do
  DCCRGX_LIB=libdccrgx_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$v -o run \
      --output-format csv -- python -u bench.py --workload $WL --steps 20 --warmup 2 --no-cpu-baseline \
      > /dev/null 2> gpurun_out/${TAG}_prof_$v.err || exit $?
  python - "$TAG" "$v" <<'EOF'
import csv, glob, sys
tag, v = sys.argv[1], sys.argv[2]
for f in glob.glob(f"gpurun_out/{tag}_prof_{v}/**/*kernel_stats.csv", recursive=True):
    for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"])):
        if "advection" not in r["Name"] and "gol" not in r["Name"] and "po_" not in r["Name"]:
            continue
        print(v, f'{r["Name"][:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"]) / 1e3:8.1f}')
EOF
  [ "$PMC" = "2" ] && continue
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $c | cut -d' ' -f1)
    DCCRGX_LIB=libdccrgx_$v.so timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-advection}" \
        -d gpurun_out/${TAG}_pmc_${v}_$n -o run --output-format csv -- \
        python -u bench.py --workload $WL --steps 10 --warmup 1 --no-cpu-baseline > /dev/null \
        2> gpurun_out/${TAG}_pmc_${v}_$n.err || exit $?
  done
done
python scripts/pmc_summary.py ${TAG}
echo "[ab_libs] done"
