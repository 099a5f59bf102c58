#!/bin/bash
# round-3 GPU pass: the whole -m gpu suite, smoke, the default bench line, a C4 kernel trace
mkdir -p gpurun_out
R=$(pwd); export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_gpu.txt 2>&1
rc=$?; echo "[pytest_gpu] rc=$rc"; tail -3 gpurun_out/r3_pytest_gpu.txt
[ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.txt 2>&1 || { echo smoke failed; exit 3; }
tail -1 gpurun_out/r3_smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/r3_bench_default.json 2> gpurun_out/r3_bench_default.err || { echo bench failed; exit 4; }
echo "[bench] ok"
WL=c4 TAG=r3 timeout -k 10 400 bash tools/trace_wl.sh || exit 5
python tools/trace_gaps.py gpurun_out/trace_c4_r3 > gpurun_out/trace_c4_r3.gaps.txt; cat gpurun_out/trace_c4_r3.gaps.txt
