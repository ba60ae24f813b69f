#!/bin/bash
# Selected GPU tests (PYTEST_K), then bench.py once per sweep variant in SWEEP_GROUPS
# (A/B of PD_OPT_SWEEP_VARIANT).  Each step has its own time limit; stop at the
# first failure and never retry a GPU step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
    timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -x -q -m gpu -k "$PYTEST_K" \
        --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
    rc=$?; tail -5 gpurun_out/pytest_ab.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for g in ${SWEEP_GROUPS:-0 8 16}; do
    timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu \
        --sweep-variant $g ${BENCH_ARGS:-} --json-out gpurun_out/bench_g$g.json \
        > gpurun_out/bench_g$g.log 2>&1
    rc=$?; echo "group $g rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_g$g.log; exit $rc; }
    python -c "import json; z=json.load(open('gpurun_out/bench_g$g.json')); print($g, round(z['ms_per_step'],2), z['stages_ms'])"
done
# optional second config (e.g. C1) over SWEEP_GROUPS2
if [ -n "$CONFIG2" ]; then
    for g in ${SWEEP_GROUPS2:-0}; do
        timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu \
            --config $CONFIG2 --sweep-variant $g --json-out gpurun_out/bench_${CONFIG2}_g$g.json \
            > gpurun_out/bench_${CONFIG2}_g$g.log 2>&1
        rc=$?; echo "$CONFIG2 group $g rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${CONFIG2}_g$g.log; exit $rc; }
        python -c "import json; z=json.load(open('gpurun_out/bench_${CONFIG2}_g$g.json')); print('$CONFIG2', $g, round(z['ms_per_step'],2), z['stages_ms'])"
    done
fi
