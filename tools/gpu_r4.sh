#!/bin/bash
# Round-4 development call.  Steps (each with its own time limit, stop at the
# first failure):
#   TESTS   pytest node ids / files to run first ("" = none); KEXPR: their -k expression
#   AB      space-separated sweep variants for C2 bench A/B (e.g. "29 61")
#   PMCV    a sweep variant for one PMC pass set (SQ + TA + TCP + fetch) on C2
#   FLOOR=1 the sharded floor (tools/gpu_floor.sh without its tests)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  KARGS=(); [ -n "${KEXPR:-}" ] && KARGS=(-k "$KEXPR")
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout ${PER_TEST:-300} --timeout-method thread \
      -m gpu "${KARGS[@]}" $TESTS > gpurun_out/r4_pytest.log 2>&1
  rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r4_pytest.log | tail -25
  [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in ${AB:-}; do
    timeout -k 10 300 python -u bench.py --config ${CFG:-C2} --steps 10 --warmup 2 --no-cpu --no-host \
        --sweep-variant $v --json-out gpurun_out/r4_ab_${v}_$rep.json > gpurun_out/r4_ab_${v}_$rep.log 2>&1 \
        || { tail -5 gpurun_out/r4_ab_${v}_$rep.log; exit 1; }
    python -c "
import json; b=json.load(open('gpurun_out/r4_ab_${v}_$rep.json')); s=b['stages_ms']; w=b.get('sweep_stats') or {}
print('v$v rep$rep', round(b['ms_per_step'],2), 'count', s['count'], 'border', s['border'], 'link', s['link'],
      'staged', w.get('s_count_staged'), '/', w.get('s_count_batches'), 'cand', w.get('s_count_cand'))"
  done
done
# ABX: '|'-separated bench argument sets, alternated twice (e.g. "--border-lists 0|--border-lists 1")
if [ -n "${ABX:-}" ]; then
  IFS='|' read -ra SETS <<< "$ABX"
  for rep in 1 2; do
    i=0
    for a in "${SETS[@]}"; do
      i=$((i+1))
      timeout -k 10 300 python -u bench.py --config ${CFG:-C2} --steps 10 --warmup 2 --no-cpu --no-host \
          $a --json-out gpurun_out/r4_abx_${i}_$rep.json > gpurun_out/r4_abx_${i}_$rep.log 2>&1 \
          || { tail -5 gpurun_out/r4_abx_${i}_$rep.log; exit 1; }
      python -c "
import json; b=json.load(open('gpurun_out/r4_abx_${i}_$rep.json')); s=b['stages_ms']
print('[$a] rep$rep', round(b['ms_per_step'],2), {k: v for k, v in s.items() if k not in ('total', 'grid_grow')},
      b.get('dense') or '')"
    done
  done
fi
if [ -n "${PMCV:-}" ]; then
  export PROF_VARIANT=$PMCV PROF_REPS=1
  T=_v$PMCV
  i=0
  for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
              "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
              "FETCH_SIZE" "WRITE_SIZE TA_BUSY_avr"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/pmc${T}_$i -o p \
        -- python tools/prof_one.py > gpurun_out/pmc${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc${T}_$i.log; exit 1; }
  done
  python tools/pmc_summary.py gpurun_out/pmc${T}_[0-9]* > gpurun_out/pmc${T}_summary.json && python - <<PY
import json
s = json.load(open("gpurun_out/pmc${T}_summary.json"))
for k in ("count4_kernel", "count5_kernel"):
    if k in s:
        print(k, {c: round(v / 1e6, 2) for c, v in s[k].items()}, "(1e6)")
PY
fi
if [ "${FLOOR:-0}" = "1" ]; then
  for a in "c2_12m --config C2 --points 12500000 --steps 5" "c4_125m --config C4 --points 125000000 --steps 3"; do
    set -- $a; name=$1; shift
    timeout -k 10 300 python -u tools/shard_overhead.py "$@" > gpurun_out/floor_$name.log 2>&1 \
      || { tail -20 gpurun_out/floor_$name.log; exit 1; }
    tail -1 gpurun_out/floor_$name.log
  done
fi
echo "r4 ok"
