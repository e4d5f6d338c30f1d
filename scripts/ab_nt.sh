cd "${GRAFT_REPO_ROOT:-.}"
for round in 1 2; do
for v in base nt; do
  cp dccrg_amd/libdccrgx_$v.so dccrg_amd/libdccrgx.so
  for w in gol scalability; do
    timeout -k 10 300 python -u bench.py --workload $w --steps 40 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', '$w', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_per_step'],4), round(d['roofline']['frac'],3))"
  done
done
done
