#!/bin/bash
# Round-3 iteration: selected parity tests, C3 / C2 / C4 bench lines (no CPU
# leg) and a rocprofv3 kernel-stats pass of C4.  Each GPU step has its own
# time limit; the first failure ends the script.
#   KEXPR   pytest -k selection over tests/test_gpu_parity.py ("" = skip)
#   CONFIGS bench configs (default "C3 C2 C4");  PROFC  config to profile ("" = none)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${KEXPR:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests/test_gpu_parity.py -k "$KEXPR" -x -q -m gpu \
      --timeout 300 --timeout-method thread > gpurun_out/pytest_r3.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_r3.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CONFIGS:-C3 C2 C4}; do
  timeout -k 10 400 python -u bench.py --config $c --steps ${STEPS:-5} --warmup 2 --no-cpu --no-host \
      ${BENCH_ARGS:-} --json-out gpurun_out/bench_$c.json > gpurun_out/bench_$c.log 2>&1 \
      || { tail -20 gpurun_out/bench_$c.log; exit 1; }
  python - "$c" <<'PY'
import json, sys
c = sys.argv[1]
b = json.load(open(f"gpurun_out/bench_{c}.json"))
print(c, "ms/step %.2f value %.3e kernel %.3f" % (b["ms_per_step"], b["value"], b["roofline"]["kernel_ms"]))
print("  stages", b["stages_ms"])
PY
done
if [ -n "${PROFC:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$PROFC \
      -o k -- python bench.py --config $PROFC --steps 2 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-} \
      > gpurun_out/prof_$PROFC.log 2>&1 || { tail -5 gpurun_out/prof_$PROFC.log; exit 1; }
  f=$(find gpurun_out/prof_$PROFC -name "*kernel_stats.csv" | head -1)
  python tools/kstats.py "$f" 25
fi
echo "r3 ok"
