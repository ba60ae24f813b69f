#!/bin/bash
# HBM bytes of the sort / gather kernels with and without PD_OPT_SORT_PAYLOAD
# (C2, 100M): FETCH_SIZE and WRITE_SIZE passes per mode, then summaries
# gpurun_out/pmc_pay{0,1}_summary.json.  The first failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
export PROF_REPS=1
for m in 0 1; do
  for pass in FETCH_SIZE WRITE_SIZE; do
    PROF_SORT_PAYLOAD=$m timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv \
      -d gpurun_out/pmc_pay${m}_$pass -o p -- python tools/prof_one.py \
      > gpurun_out/pmc_pay${m}_$pass.log 2>&1 || { echo "pass $m $pass failed"; exit 1; }
  done
  python tools/pmc_summary.py gpurun_out/pmc_pay${m}_* > gpurun_out/pmc_pay${m}_summary.json || exit 1
done
echo "payload pmc ok"
