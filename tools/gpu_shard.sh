#!/bin/bash
# Round-3 multi-GPU readiness on one GPU: the sharded fixed costs as a 1-rank
# RCCL group (tools/shard_overhead.py), the full-size rehearsals
# (tests/test_gpu_rehearsal.py), then optional extras:
#   C3FULL=1   tests/test_gpu_fullsize.py::test_c3_full_1m_vs_oracle
#   C4KD=1     tools/c4_kd_report.py -> gpurun_out/c4_kd.json
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/shard_overhead.py --points 100000000 --steps 3 \
    > gpurun_out/shard_overhead.log 2>&1 || { tail -20 gpurun_out/shard_overhead.log; exit 1; }
tail -1 gpurun_out/shard_overhead.log
if [ "${REHEARSE:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_rehearsal.py -x -v -s -m gpu --timeout 800 \
      --timeout-method thread > gpurun_out/pytest_rehearsal.log 2>&1
  rc=$?; grep -E "PASS|FAIL|Error|seconds|passed|failed" gpurun_out/pytest_rehearsal.log | tail -15
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${C3FULL:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k c3_full -x -v -s -m gpu \
      --timeout 500 --timeout-method thread > gpurun_out/pytest_c3full.log 2>&1
  rc=$?; grep -E "C3 1M|passed|failed|Error" gpurun_out/pytest_c3full.log | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${C4KD:-0}" = "1" ]; then
  timeout -k 10 600 python -u tools/c4_kd_report.py --out gpurun_out/c4_kd.json \
      > gpurun_out/c4_kd.log 2>&1 || { tail -20 gpurun_out/c4_kd.log; exit 1; }
  grep '"P"' gpurun_out/c4_kd.log
fi
echo "shard ok"
