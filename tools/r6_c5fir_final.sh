#!/bin/bash
# the kept c5fir block plan (first block 2 048, ramp 1.5): FIR / serial-render parity suites, a kernel
# trace (tools/fill_timeline.py reads it), three c5fir runs
mkdir -p gpurun_out; TAG=${TAG:-r6s}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_full_size.py tests/test_gpu_fir_sig.py \
    tests/test_gpu_render_spec.py tests/test_gpu_dither_flat.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
WL=c5fir TAG=${TAG} bash tools/trace_wl.sh || exit 2
VAR=ICW_NONE VALS="-" WLS="c5fir" REPS=3 STEPS=3 TAG=${TAG}b bash tools/env_ab.sh || exit 3
