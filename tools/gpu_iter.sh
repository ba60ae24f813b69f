#!/bin/bash
# One development iteration on the GPU box: (optional) parity tests, the C2
# bench without the CPU leg, and a rocprofv3 kernel-stats pass of the same
# bench.  Every GPU step has its own time limit; the first failure ends it.
#   TESTS="tests/test_gpu_parity.py" KEXPR="kd"   pytest selection ("" = skip)
#   BENCH_ARGS="--config C2"                  extra bench.py arguments
#   PROF=0                                    skip the rocprofv3 pass
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -x -q -m gpu --timeout 300 \
      --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_iter.log
  [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_iter.log | head -20; exit $rc; }
fi
timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu --no-host ${BENCH_ARGS:-} \
    --json-out gpurun_out/bench_iter.json > gpurun_out/bench_iter.log 2>&1 \
    || { tail -20 gpurun_out/bench_iter.log; exit 1; }
python - <<'EOF'
import json
b = json.load(open("gpurun_out/bench_iter.json"))
print("ms/step %.2f  value %.3e  count %.3f ms" % (b["ms_per_step"], b["value"], b["roofline"]["kernel_ms"]))
print("stages", b["stages_ms"])
print("kd", b.get("kd_ms"))
EOF
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iter \
      -o it -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host ${BENCH_ARGS:-} \
      > gpurun_out/prof_iter.log 2>&1 || { tail -5 gpurun_out/prof_iter.log; exit 1; }
  f=$(ls gpurun_out/prof_iter/*/it_kernel_stats.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find gpurun_out/prof_iter -name "*kernel_stats.csv" | head -1)
  python tools/kstats.py "$f" 45
fi
echo "iter ok"
