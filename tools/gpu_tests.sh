#!/bin/bash
# GPU-box test pass: the -m gpu suite (one process, per-test timeout) then smoke; stop at a crash.
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
echo "[pytest_gpu] rc=$rc" | tee -a gpurun_out/steps.txt
tail -5 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1
rc2=$?
echo "[smoke] rc=$rc2" | tee -a gpurun_out/steps.txt
tail -3 gpurun_out/smoke.txt
exit $(( rc | rc2 ))
