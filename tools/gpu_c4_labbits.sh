#!/bin/bash
# C4 label-pass A/B over the bucket width (PD_LAB_BITS), after the label tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "c4_full or c2_full or label_buckets or goldens or sklearn" \
    -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_lab.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_lab.log; [ $rc -eq 0 ] || exit $rc
for b in ${BITS:-20 19 18}; do
  PD_LAB_BITS=$b timeout -k 10 400 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-host \
      --json-out gpurun_out/bench_C4_b$b.json > gpurun_out/bench_C4_b$b.log 2>&1 || { tail -5 gpurun_out/bench_C4_b$b.log; exit 1; }
  python -c "
import json; b=json.load(open('gpurun_out/bench_C4_b$b.json')); print('bits $b', round(b['ms_per_step'],2), 'border', b['stages_ms']['border'])"
done
CONFIGS=C2 bash tools/gpu_r3.sh
