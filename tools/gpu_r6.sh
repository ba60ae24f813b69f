#!/bin/bash
# Round-6 development call.  Steps (each under its own time limit; the call
# stops at the first failure):
#   CHK_TESTS  pytest -k expression run against the bounds-checked build
#              (ab/libpardis_chk.so, -DPD_CHECK_BOUNDS=1) first
#   TESTS      pytest node ids / files ("" = none); KEXPR: their -k expression
#   BENCH      space-separated configs benched once each, no CPU leg
#   ABX        '|'-separated bench argument sets, alternated twice on CFG (default C2)
#   PROF=1     rocprofv3 --kernel-trace --stats of a short CFG bench
#   SMOKE=1    __graft_entry__.smoke()
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/r6
mkdir -p $O
if [ -n "${CHK_TESTS:-}" ]; then
  PYPARDIS_LIB=$PWD/ab/libpardis_chk.so timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v \
      --timeout ${PER_TEST:-300} --timeout-method thread -m gpu -k "$CHK_TESTS" tests/test_gpu_parity.py \
      > $O/pytest_chk.log 2>&1
  rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest_chk.log | tail -20
  [ $rc -eq 0 ] || { tail -60 $O/pytest_chk.log; exit $rc; }
fi
if [ -n "${TESTS:-}" ]; then
  KARGS=(); [ -n "${KEXPR:-}" ] && KARGS=(-k "$KEXPR")
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v --durations=15 \
      --timeout ${PER_TEST:-300} --timeout-method thread -m gpu "${KARGS[@]}" $TESTS \
      > $O/pytest.log 2>&1
  rc=$?; grep -E "FAIL|Error|passed|failed|^[0-9.]+s call" $O/pytest.log | tail -40
  [ $rc -eq 0 ] || { tail -60 $O/pytest.log; exit $rc; }
fi
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
b = json.load(open(sys.argv[1])); s = b.get('stages_ms') or {}
print(sys.argv[2], round(b['ms_per_step'], 2), 'ms', {k: v for k, v in s.items()
      if k not in ('total', 'grid_grow')}, (b.get('roofline') or {}).get('frac'))
PY
}
for c in ${BENCH:-}; do
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py --config $c --steps ${STEPS:-10} --warmup 2 \
      --no-cpu --no-host ${BENCH_ARGS:-} --json-out $O/bench_$c.json > $O/bench_$c.log 2>&1 \
      || { tail -20 $O/bench_$c.log; exit 1; }
  summ $O/bench_$c.json "$c"
done
if [ -n "${ABX:-}" ]; then
  IFS='|' read -ra SETS <<< "$ABX"
  for rep in 1 2; do
    i=0
    for a in "${SETS[@]}"; do
      i=$((i+1))
      timeout -k 10 400 python -u bench.py --config ${CFG:-C2} --steps 10 --warmup 2 --no-cpu --no-host \
          $a --json-out $O/abx_${i}_$rep.json > $O/abx_${i}_$rep.log 2>&1 \
          || { tail -20 $O/abx_${i}_$rep.log; exit 1; }
      summ $O/abx_${i}_$rep.json "[$a] rep$rep"
    done
  done
fi
#   LIBS       space-separated ab/ library names (or "base"), benched alternately twice on
#              LCFG (default C3) — LIB_TESTS: a -k expression run with each non-base library
if [ -n "${LIBS:-}" ]; then
  for l in $LIBS; do
    [ "$l" = base ] && continue
    if [ -n "${LIB_TESTS:-}" ]; then
      PYPARDIS_LIB=$PWD/ab/$l timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v \
          --timeout ${PER_TEST:-300} --timeout-method thread -m gpu -k "$LIB_TESTS" tests/ \
          > $O/pytest_$l.log 2>&1
      rc=$?; grep -E "FAIL|Error|passed|failed" $O/pytest_$l.log | tail -10
      [ $rc -eq 0 ] || { tail -60 $O/pytest_$l.log; exit $rc; }
    fi
  done
  for rep in 1 2; do
    for l in $LIBS; do
      if [ "$l" = base ]; then unset PYPARDIS_LIB; else export PYPARDIS_LIB=$PWD/ab/$l; fi
      timeout -k 10 400 python -u bench.py --config ${LCFG:-C3} --steps ${STEPS:-5} --warmup 2 --no-cpu --no-host \
          --json-out $O/lib_${l}_$rep.json > $O/lib_${l}_$rep.log 2>&1 \
          || { tail -20 $O/lib_${l}_$rep.log; exit 1; }
      summ $O/lib_${l}_$rep.json "[$l] rep$rep"
    done
  done
  unset PYPARDIS_LIB
fi
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python bench.py --config ${CFG:-C2} --steps 5 --warmup 1 --no-cpu --no-host ${PROF_ARGS:-} \
      > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" $O/kernel_stats.csv && head -30 $O/kernel_stats.csv | cut -c1-160
fi
#   PROBE      a probe binary under tools/ (with its arguments), output to $O/<name>.txt
if [ -n "${PROBE:-}" ]; then
  pn=$(basename ${PROBE%% *})
  timeout -k 10 300 tools/$PROBE > $O/$pn.txt 2>&1 || { tail -20 $O/$pn.txt; exit 1; }
  cat $O/$pn.txt
fi
if [ "${SMOKE:-0}" = "1" ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
      || { cat $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
echo r6 ok
