#!/bin/bash
# A/B/C... of library builds on one config (no CPU leg), alternating:
# the in-tree build ("tree") and ab/libpardis_<v>.so for each v in $LIBS,
# REPS rounds.  Prints ms/step and the stages named in $STAGES.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/abm
for i in $(seq 1 ${REPS:-2}); do
  for v in tree ${LIBS}; do
    if [ $v = tree ]; then unset PYPARDIS_LIB; else export PYPARDIS_LIB=$PWD/ab/libpardis_$v.so; fi
    timeout -k 10 300 python -u bench.py --config ${CFG:-C2} --steps ${STEPS:-10} --warmup 2 --no-cpu --no-host \
        --json-out gpurun_out/abm/${v}_$i.json > gpurun_out/abm/${v}_$i.log 2>&1 \
        || { tail -5 gpurun_out/abm/${v}_$i.log; exit 1; }
    python -c "
import json; b=json.load(open('gpurun_out/abm/${v}_$i.json')); s=b['stages_ms']
print('$v', $i, round(b['ms_per_step'],2), {k: s[k] for k in '${STAGES:-halo count link border}'.split()})"
  done
done
