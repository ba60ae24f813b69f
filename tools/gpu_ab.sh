#!/bin/bash
# A/B bench lines (no CPU / host legs): each AB_i="<label>|<bench args>" runs
# once; prints ms/step and the stage times.  The first failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1)); label="${spec%%|*}"; args="${spec#*|}"
  timeout -k 10 ${AB_TIMEOUT:-300} python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu \
      --no-host $args --json-out gpurun_out/ab_$i.json > gpurun_out/ab_$i.log 2>&1 \
      || { tail -20 gpurun_out/ab_$i.log; exit 1; }
  python - "$label" gpurun_out/ab_$i.json <<'PY'
import json, sys
b = json.load(open(sys.argv[2]))
print(sys.argv[1], "ms/step %.2f" % b["ms_per_step"], {k: v for k, v in b["stages_ms"].items()
      if k not in ("grid_grow",)}, flush=True)
PY
done
echo "ab ok"
