#!/bin/bash
# Round evidence in one GPU session: parity suite + smoke, C2 bench (with the
# CPU baseline) + rocprofv3 kernel stats, C4 bench (1B points) + kernel stats.
# Every GPU step has its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --json-out gpurun_out/bench.json \
    > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1 \
    || { tail -5 gpurun_out/prof.log; exit 1; }
timeout -k 10 400 python -u bench.py --config C4 --steps 3 --warmup 1 \
    --json-out gpurun_out/bench_c4.json > gpurun_out/bench_c4.log 2>&1 \
    || { tail -5 gpurun_out/bench_c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 \
    -- python bench.py --config C4 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_c4.log 2>&1 \
    || { tail -5 gpurun_out/prof_c4.log; exit 1; }
echo "round ok"
