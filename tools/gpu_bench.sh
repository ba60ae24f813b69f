#!/bin/bash
# bench.py at the default config + a rocprofv3 kernel-trace summary of the
# same command.  Each GPU step has its own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-5}
timeout -k 10 ${BENCH_TIMEOUT:-900} python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} \
    --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "$NO_PROF" ]; then exit 0; fi
timeout -k 10 ${PROF_TIMEOUT:-900} rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/prof -o bench -- python bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} \
    > gpurun_out/prof.log 2>&1
rc=$?; tail -3 gpurun_out/prof.log; echo "prof rc=$rc"; exit $rc
