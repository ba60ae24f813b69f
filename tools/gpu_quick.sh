#!/bin/bash
# Round-3 development call: selected GPU tests, the C2 bench, rocprofv3 kernel
# stats, and one PMC pass of instruction counters (SQ_*) over tools/prof_one.py.
#   TESTS / KEXPR   pytest files / -k expression ("" = skip tests)
#   PMC=0           skip the PMC pass
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS="${TESTS:-}" KEXPR="${KEXPR:-}" PROF="${PROF:-1}" BENCH_ARGS="${BENCH_ARGS:-}" \
  bash tools/gpu_iter.sh || exit $?
if [ "${PMC:-1}" = "1" ]; then
  T=_quick
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv \
      -d gpurun_out/pmc${T}_1 -o p -- python tools/prof_one.py > gpurun_out/pmc${T}_1.log 2>&1 \
      || { tail -5 gpurun_out/pmc${T}_1.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc${T}_1 > gpurun_out/pmc${T}_summary.json && \
  python - <<'PY'
import json
s = json.load(open("gpurun_out/pmc_quick_summary.json"))
for k in ("count4_kernel", "count2_kernel", "border4_kernel", "border2_kernel", "window_uf_kernel", "gather_kernel"):
    if k in s:
        v = s[k]
        print(k, {c: round(v[c] / 1e6, 2) for c in v if c.startswith("SQ_")}, "(1e6)")
PY
fi
echo quick ok
