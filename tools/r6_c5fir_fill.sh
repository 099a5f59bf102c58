#!/bin/bash
# c5fir's fill: where a FIR / CWAVE call with a serial render runs its dither generator (ICW_DITH_OWN:
# 2 = converter, generator and render on CU-masked streams with queues of their own, the default;
# 1 = the generator on a plain stream of its own; 0 = after the converter on its stream): the parity
# suites that run serial renders after a converter, a kernel trace of 2, then the A/B
mkdir -p gpurun_out; TAG=${TAG:-r6n}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_full_size.py tests/test_gpu_cwave_graph.py \
    tests/test_gpu_render_spec.py tests/test_gpu_dither_flat.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
WL=c5fir TAG=${TAG}own2 bash tools/trace_wl.sh || exit 2
VAR=ICW_DITH_OWN VALS="2 0 1" WLS="c5fir c5" REPS=2 STEPS=3 TAG=${TAG}ab bash tools/env_ab.sh || exit 3
