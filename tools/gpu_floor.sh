#!/bin/bash
# Round-4: the per-rank floor at 8-GPU size on one GPU — the sharded train as a
# 1-rank RCCL group against the single-device train, at C2/8 = 12.5M points
# and C4/8 = 125M points (tools/shard_overhead.py), plus optional extras:
#   FULL=1   the same at C2 100M
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u tools/shard_overhead.py "$@" > gpurun_out/floor_$name.log 2>&1 \
    || { tail -20 gpurun_out/floor_$name.log; exit 1; }
  tail -1 gpurun_out/floor_$name.log
}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_bench_launch.py "tests/test_gpu_parity.py::test_rccl_comm_single_rank" \
    > gpurun_out/floor_pytest.log 2>&1 || { tail -30 gpurun_out/floor_pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/floor_pytest.log | tail -2
run c2_12m --config C2 --points 12500000 --steps 5
run c4_125m --config C4 --points 125000000 --steps 3
if [ "${FULL:-0}" = "1" ]; then
  run c2_100m --config C2 --points 100000000 --steps 3
fi
echo "floor ok"
