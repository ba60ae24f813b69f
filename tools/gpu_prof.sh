#!/bin/bash
# Round-4 profiling call (each step time-limited, stop at the first failure):
#   PMC=1        the four PMC passes over one C2 train -> gpurun_out/pmc_${TAG}_summary.json
#   SHARDPROF=1  rocprofv3 kernel stats of tools/shard_overhead.py (SP_ARGS)
#   BENCH=1      bench.py C2 (no CPU / host legs) -> gpurun_out/bench_prof.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
if [ "${PMC:-0}" = "1" ]; then
  TAG=${TAG:-_r4} PROF_CFG=${PROF_CFG:-C2} bash tools/pmc_run.sh || exit $?
  # PMC_SAVE=rNN_vMM: the summary becomes profiles/rNN_vMM_pmc[_cK]_summary.json, so
  # a bench later in this call reads it (copy it back into the repo afterwards)
  [ -n "${PMC_SAVE:-}" ] && cp gpurun_out/pmc${TAG:-_r4}_summary.json \
      profiles/${PMC_SAVE}_pmc${PMC_CTAG:-}_summary.json
fi
if [ "${SHARDPROF:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sprof -o sp \
      -- python tools/shard_overhead.py ${SP_ARGS:---config C4 --points 125000000 --steps 1} \
      > gpurun_out/sprof.log 2>&1 || { tail -5 gpurun_out/sprof.log; exit 1; }
  tail -1 gpurun_out/sprof.log | cut -c1-400
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-host \
      --json-out gpurun_out/bench_prof.json > gpurun_out/bench_prof.log 2>&1 \
      || { tail -5 gpurun_out/bench_prof.log; exit 1; }
  python -c "
import json; b=json.load(open('gpurun_out/bench_prof.json'))
print(round(b['ms_per_step'],2), b['stages_ms']); print(b.get('train_roofline'))"
fi
echo "prof ok"
