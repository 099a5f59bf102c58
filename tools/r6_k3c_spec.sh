#!/bin/bash
# K3c speculative clamp-free blocks: the forced-redo suite and the render suites, then c5fir / c5 against
# the build without speculation (libicw_nospec.so, -DICW_K3C_SPEC=0), then an SQ pass of c5fir
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r6g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_k3c_redo.py tests/test_gpu_render_spec.py tests/test_gpu_parity.py tests/test_gpu_dither_flat.py tests/test_gpu_cwave_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
LIBS="libicw.so libicw_nospec.so libicw_head.so" WLS="c5fir" REPS=2 STEPS=3 TAG=${TAG}ab bash tools/ab_bench.sh || exit 3
( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_trace" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_trace.txt 2>&1 || { echo "trace failed"; exit 3; }
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM \
    --output-format csv -d "$R/gpurun_out/${TAG}_sq" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_sq.txt 2>&1 || { echo "sq failed"; exit 3; }
echo "profiles ok"
