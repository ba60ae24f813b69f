#!/bin/bash
# C3 (dense path): PMC passes over one warm train, then bench.py --config C3
# under a kernel-trace summary.  Each GPU step has its own time limit; stop at
# the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
PROF_CFG=C3 PROF_N=1000000 PASS_TIMEOUT=240 bash tools/pmc_run.sh || exit $?
cp gpurun_out/pmc_summary.json gpurun_out/pmc_summary_c3.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 \
    -o c3 -- python bench.py --config C3 --steps 3 --warmup 1 --no-cpu \
    --json-out gpurun_out/bench_c3_prof.json > gpurun_out/prof_c3.log 2>&1
rc=$?; tail -2 gpurun_out/prof_c3.log; echo "prof rc=$rc"; exit $rc
