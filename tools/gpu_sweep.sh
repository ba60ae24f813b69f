#!/bin/bash
# Sweep one bench knob: SWEEP="--centre-window 16|--centre-window 32" (|-separated
# argument sets); prints ms/step and the stage times per setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IFS='|' read -ra SETS <<< "$SWEEP"
for a in "${SETS[@]}"; do
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu --no-host ${BENCH_ARGS:-} $a \
      --json-out gpurun_out/sweep.json > gpurun_out/sweep.log 2>&1 || { tail -5 gpurun_out/sweep.log; exit 1; }
  python -c "
import json; b=json.load(open('gpurun_out/sweep.json'))
print('$a', 'ms/step %.2f' % b['ms_per_step'], {k: v for k, v in b['stages_ms'].items() if k in ('count','link','merge','roots','border','total')}, {k: v for k, v in (b.get('sweep_stats') or {}).items() if k.startswith('s_')})"
done
