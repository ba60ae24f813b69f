cd "${GRAFT_REPO_ROOT:-/root/repo}"
KEXPR="dir_ or growth or globe or golden or variants" CONFIGS="C2" bash tools/gpu_r3.sh || exit $?
for m in 16 64 256; do
  PD_LAB_TILE_MULT=$m timeout -k 10 400 python -u bench.py --config C4 --steps 3 --warmup 1 --no-cpu --no-host --json-out gpurun_out/bench_C4_m$m.json > gpurun_out/bench_C4_m$m.log 2>&1 || { tail -5 gpurun_out/bench_C4_m$m.log; exit 1; }
  python -c "
import json; b=json.load(open('gpurun_out/bench_C4_m$m.json')); print('mult $m', round(b['ms_per_step'],2), b['stages_ms'])"
done
