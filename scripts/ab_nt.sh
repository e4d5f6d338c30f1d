# Paired A/B of two builds of the library on one box:
#   bash scripts/ab_nt.sh "<workloads>" [rounds]
# expects dccrg_amd/libdccrgx_base.so and dccrg_amd/libdccrgx_nt.so (the two
# variants, built here beforehand); prints ms/step, kernel ms/step, roofline frac.
cd "${GRAFT_REPO_ROOT:-.}"
# the library built from the committed sources is restored whatever happens
cp dccrg_amd/libdccrgx.so /tmp/libdccrgx_orig.so || exit 1
trap 'cp /tmp/libdccrgx_orig.so dccrg_amd/libdccrgx.so' EXIT
WL=${1:-"gol scalability"}
ROUNDS=${2:-2}
for round in $(seq "$ROUNDS"); do
for v in base nt; do
  cp dccrg_amd/libdccrgx_$v.so dccrg_amd/libdccrgx.so
  for w in $WL; do
    timeout -k 10 300 python -u bench.py --workload $w --steps 40 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', '$w', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_per_step'],4), round(d['roofline']['frac'],3))" || exit 1
  done
done
done
