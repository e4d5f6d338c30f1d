#!/bin/bash
# One focused GPU pass while iterating on a kernel: the selected GPU tests,
# then for each named workload a bench line and a rocprofv3 kernel-trace
# stats run.  Stops at the first crash / timeout.
# Usage: scripts/gpu_quick.sh TAG "pytest -k expression" workload [workload ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
SEL=$2
shift 2
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "$SEL" \
      > gpurun_out/pytest_${TAG}.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_${TAG}.log
  grep -E "FAILED|ERROR" gpurun_out/pytest_${TAG}.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
for w in "$@"; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/bench_${w}_${TAG}.json 2> gpurun_out/bench_${w}_${TAG}.err
  rc=$?
  echo "[quick] bench $w rc=$rc"; tail -c 1200 gpurun_out/bench_${w}_${TAG}.json; echo
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${w}_${TAG}.err; exit $rc; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${w}_${TAG} -o run --output-format csv -- \
      python -u bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 2 \
      > gpurun_out/bench_prof_${w}_${TAG}.json 2> gpurun_out/prof_${w}_${TAG}.err
  rc=$?
  echo "[quick] rocprof $w rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python - "$w" "$TAG" <<'EOF'
import csv, glob, sys
w, tag = sys.argv[1], sys.argv[2]
for f in glob.glob(f"gpurun_out/prof_{w}_{tag}/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]
    for r in rows:
        print(f'{r["Name"][:90]:90s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"]) / 1e3:9.1f}')
EOF
done
echo "[quick] done"
