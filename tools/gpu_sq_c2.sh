#!/bin/bash
# C2 bench line (no CPU leg) + one SQ counter pass over a warm C2 train:
# VALU instructions and waves per kernel (gpurun_out/sq_c2_summary.json).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
CONFIGS="${CONFIGS:-C2}" bash tools/gpu_r3.sh || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d gpurun_out/sq_c2 -o p -- python tools/prof_one.py > gpurun_out/sq_c2.log 2>&1 || { tail -5 gpurun_out/sq_c2.log; exit 1; }
python tools/pmc_summary.py gpurun_out/sq_c2 > gpurun_out/sq_c2_summary.json || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/sq_c2_summary.json"))
for k in sorted(d, key=lambda k: -d[k].get("SQ_INSTS_VALU", 0))[:8]:
    v = d[k]
    print("%-28s VALU %.3e waves %.0f VALU/wave %.0f" % (k[:28], v.get("SQ_INSTS_VALU", 0), v.get("SQ_WAVES", 0),
          v.get("SQ_INSTS_VALU", 0) / max(1, v.get("SQ_WAVES", 1))))
PY
