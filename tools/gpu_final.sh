#!/bin/bash
# Round evidence, in two GPU calls (each step time-limited; the first failure
# ends the call):
#   PHASE=pmc   PMC summaries of C2, C4, C3 -> gpurun_out/final/pmc_<cfg>_summary.json
#               (copy them to profiles/<TAG>_pmc[_cK]_summary.json before PHASE=bench,
#               so the bench's measured roofline fields come from this build)
#   PHASE=bench full pytest -m gpu, smoke, C2 bench (CPU + host legs) + rocprofv3
#               kernel stats, C4 bench + stats, C3 bench, C1 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
if [ "${PHASE:-bench}" = "pmc" ]; then
  CONFIGS="${CONFIGS:-C2 C4 C3}" bash tools/gpu_pmc_all.sh || exit $?
  for c in c2 c4 c3; do cp gpurun_out/pmc_${c}_summary.json $O/ 2>/dev/null; done
  echo "pmc phase ok"
  exit 0
fi
#   PARTS (default "tests c2 c4 c3 c1") selects the bench phase's parts;
#   c1 first takes C1's PMC into profiles/${TAG:-rNN}_pmc_c1_summary.json
has() { case " ${PARTS:-tests c2 c4 c3 c1} " in *" $1 "*) return 0 ;; esac; return 1; }
if has tests; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
if has c2; then
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --json-out $O/bench.json \
    > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
echo "C2 bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 \
    -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host > $O/prof.log 2>&1 \
    || { tail -5 $O/prof.log; exit 1; }
fi
if has c4; then
timeout -k 10 600 python -u bench.py --config C4 --steps 3 --warmup 1 --no-host \
    --json-out $O/bench_c4.json > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 1; }
echo "C4 bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 \
    -- python bench.py --config C4 --steps 2 --warmup 1 --no-cpu --no-host > $O/prof_c4.log 2>&1 \
    || { tail -5 $O/prof_c4.log; exit 1; }
fi
if has c3; then
timeout -k 10 400 python -u bench.py --config C3 --steps 3 --warmup 1 \
    --json-out $O/bench_c3.json > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 \
    -- python bench.py --config C3 --steps 3 --warmup 1 --no-cpu --no-host > $O/prof_c3.log 2>&1 \
    || { tail -5 $O/prof_c3.log; exit 1; }
fi
if has c1; then
CONFIGS=C1 bash tools/gpu_pmc_all.sh > $O/pmc_c1.log 2>&1 || { tail -5 $O/pmc_c1.log; exit 1; }
cp gpurun_out/pmc_c1_summary.json $O/ && cp gpurun_out/pmc_c1_summary.json profiles/${TAG:-r99_v99}_pmc_c1_summary.json
timeout -k 10 300 python -u bench.py --config C1 --steps 5 --warmup 2 --no-host \
    --json-out $O/bench_c1.json > $O/bench_c1.log 2>&1 || { tail -5 $O/bench_c1.log; exit 1; }
fi
echo "final bench phase ok"
