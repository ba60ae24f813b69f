#!/bin/bash
# PMC passes (each its own rocprofv3 run, no tracing domains mixed in) over
# tools/prof_one.py, then a per-kernel summary.  Stops at the first failure.
#   PROF_CFG=C2|C3|C4  PROF_N=<points>  TAG=<suffix of the output names>
# Output: gpurun_out/pmc${TAG}_<pass>/, gpurun_out/pmc${TAG}_summary.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
export PROF_REPS=${PROF_REPS:-2}
T=${TAG:-}
i=0
run_pass() {
  i=$((i+1))
  timeout -k 10 ${PASS_TIMEOUT:-300} rocprofv3 --pmc "$@" --output-format csv \
     -d gpurun_out/pmc${T}_$i -o p -- python tools/prof_one.py > gpurun_out/pmc${T}_$i.log 2>&1
  rc=$?; echo "pass $i ($*) rc=$rc"; return $rc
}
run_pass SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit $?
run_pass TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum || exit $?
run_pass FETCH_SIZE || exit $?
run_pass WRITE_SIZE TA_BUSY_avr || exit $?
python tools/pmc_summary.py gpurun_out/pmc${T}_[0-9]* > gpurun_out/pmc${T}_summary.json && echo summary ok
