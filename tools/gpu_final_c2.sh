#!/bin/bash
# Round-end C2 evidence after a late change: full pytest -m gpu, smoke, the
# C2 bench line (CPU + host legs) and rocprofv3 kernel stats of the same
# command, the C1 and C4 bench lines.  Each step time-limited; the first
# failure ends the call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --json-out $O/bench.json \
    > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
echo "C2 bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 \
    -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host > $O/prof.log 2>&1 \
    || { tail -5 $O/prof.log; exit 1; }
timeout -k 10 300 python -u bench.py --config C1 --steps 5 --warmup 2 --no-host \
    --json-out $O/bench_c1.json > $O/bench_c1.log 2>&1 || { tail -5 $O/bench_c1.log; exit 1; }
timeout -k 10 600 python -u bench.py --config C4 --steps 3 --warmup 1 --no-host \
    --json-out $O/bench_c4.json > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 1; }
echo "final2 ok"
