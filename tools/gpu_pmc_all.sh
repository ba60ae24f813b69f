#!/bin/bash
# PMC summaries of the current build for C2 (100M), C4 (1B) and C3 (1M, d=64):
# gpurun_out/pmc_c2_summary.json, pmc_c4_summary.json, pmc_c3_summary.json.
# CONFIGS="C2 C4 C3" selects.  The first failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for c in ${CONFIGS:-C2 C4 C3}; do
  case $c in
    C2) n=100000000 ;; C4) n=1000000000 ;; C3) n=1000000 ;; C1) n=10000000 ;;
  esac
  lc=$(echo $c | tr 'A-Z' 'a-z')
  PROF_CFG=$c PROF_N=$n TAG=_$lc bash tools/pmc_run.sh || exit $?
done
echo "pmc all ok"
