#!/bin/bash
# A/B/... of library builds on the C2 bench (no CPU / host legs), alternating:
# LIBS = space-separated names under ab/ ("-" = the in-tree build), REPS rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-2}); do
  for v in ${LIBS:--}; do
    if [ "$v" = "-" ]; then unset PYPARDIS_LIB; else export PYPARDIS_LIB=$PWD/ab/$v; fi
    tag=${v%.so}; tag=${tag//-/tree}
    timeout -k 10 300 python -u bench.py --config ${CFG:-C2} --steps 10 --warmup 2 --no-cpu --no-host \
        --json-out gpurun_out/abl_${tag}_$i.json > gpurun_out/abl_${tag}_$i.log 2>&1 \
        || { tail -5 gpurun_out/abl_${tag}_$i.log; exit 1; }
    python -c "
import json; b=json.load(open('gpurun_out/abl_${tag}_$i.json')); s=b['stages_ms']
print('$tag', $i, round(b['ms_per_step'],2), {k: v for k, v in s.items() if v and k not in ('total', 'grid_grow')})"
  done
done
echo "ab ok"
