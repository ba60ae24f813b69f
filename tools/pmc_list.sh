#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1; echo "list rc=$?"
grep -o -E "^[[:space:]]*[A-Z][A-Z0-9_]+(\[[0-9:]+\])?" gpurun_out/pmc_list.txt | sort -u | wc -l
