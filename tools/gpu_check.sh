#!/bin/bash
# One GPU session: parity tests, then smoke.  Stops at the first crash/timeout
# (exit 124/134/137/139) and never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
cat gpurun_out/smoke.log | tail -5
echo "smoke rc=$src"
[ $rc -eq 0 ] && [ $src -eq 0 ]
