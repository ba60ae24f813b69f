cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "dense" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || exit $rc
for sc in 1 0; do
  timeout -k 10 300 python -u bench.py --config C3 --steps 5 --warmup 2 --no-cpu --no-host --dense-screen $sc --json-out gpurun_out/bench_c3_s$sc.json > gpurun_out/bench_c3_s$sc.log 2>&1 || { tail -20 gpurun_out/bench_c3_s$sc.log; exit 1; }
  python -c "
import json; b=json.load(open('gpurun_out/bench_c3_s$sc.json')); print('screen $sc', b['ms_per_step'], b['roofline'], b.get('stages_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python bench.py --config C3 --steps 3 --warmup 1 --no-cpu --no-host > gpurun_out/prof_c3.log 2>&1 || exit 1
f=$(find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1); python tools/kstats.py "$f" 12
