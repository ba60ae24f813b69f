#!/bin/bash
# A/B of two library builds on the C2 bench (no CPU leg), alternating:
# ab/$LIB_A vs the in-tree build, REPS times each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-2}); do
  for v in A B; do
    if [ $v = A ]; then export PYPARDIS_LIB=$PWD/ab/$LIB_A; else unset PYPARDIS_LIB; fi
    timeout -k 10 300 python -u bench.py --config ${CFG:-C2} --steps 10 --warmup 2 --no-cpu --no-host \
        --json-out gpurun_out/ab_$v$i.json > gpurun_out/ab_$v$i.log 2>&1 || { tail -5 gpurun_out/ab_$v$i.log; exit 1; }
    python -c "
import json; b=json.load(open('gpurun_out/ab_$v$i.json')); s=b['stages_ms']
print('$v$i', round(b['ms_per_step'],2), 'count', s['count'], 'border', s['border'], 'link', s['link'])"
  done
done
