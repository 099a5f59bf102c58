#!/bin/bash
# The split dither generator (K3t / K3s / K3f): the render / dither GPU suites, then c5fir and c2fir
# TPDF + flat against the one-kernel K3a (ICW_DITHER=coop), then the whole -m gpu suite
mkdir -p gpurun_out; TAG=${TAG:-r6f}
timeout -k 10 500 python -u -m pytest tests/test_gpu_dither_flat.py tests/test_gpu_cwave_graph.py tests/test_gpu_render_spec.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
VAR=ICW_DITHER VALS="- coop" WLS="c5fir c5" REPS=2 STEPS=3 TAG=${TAG}ab bash tools/env_ab.sh || exit 3
ICW_BENCH_RENDER=tpdf_flat VAR=ICW_DITHER VALS="- coop" WLS="c2fir" REPS=1 STEPS=2 TAG=${TAG}abf bash tools/env_ab.sh || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_suite.txt 2>&1
rc=$?; echo "[suite] rc=$rc"; tail -3 gpurun_out/${TAG}_suite.txt; exit $rc
