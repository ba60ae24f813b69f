#!/bin/bash
# Rehearse the sharded bench path on a one-GPU box: N gloo ranks sharing
# cuda:0 (correctness of the N>1 code path; the numbers are not a measurement).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
N=${N:-2}
timeout -k 10 ${SHARD_TIMEOUT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port ${PORT:-29517} bench.py --gpus $N --steps ${STEPS:-3} \
    --warmup 1 --rehearse --no-cpu ${BENCH_ARGS:-} > gpurun_out/shard_bench.log 2>&1
rc=$?; tail -5 gpurun_out/shard_bench.log; echo "shard bench rc=$rc"; exit $rc
