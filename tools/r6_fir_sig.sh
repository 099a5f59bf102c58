#!/bin/bash
# KF2's signature form (icw_fir_sig): the FIR parity suites, then the A/B of the default build
# (5 / 6 workgroups per CU, 4-tap blocks) against libicw_sig4.so (4 per CU, 8-tap blocks) and against
# icw_fir_graph for every tile (ICW_FIR_SIG=0) on c2fir / c4fir / c3fir, then kernel-trace stats
# and SQ passes of c2fir
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r6h}
timeout -k 10 700 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_sig_fast.py tests/test_gpu_production_random.py \
    tests/test_gpu_full_size.py tests/test_gpu_dither_flat.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
for r in 1 2; do
  LIBS="libicw.so ${VLIBS:-libicw_sig4.so}" WLS="${WLS:-c2fir c4fir c3fir}" REPS=1 STEPS=3 TAG=${TAG}ab$r bash tools/ab_bench.sh || exit 3
  VAR=ICW_FIR_SIG VALS="0" WLS="${WLS:-c2fir c4fir c3fir}" REPS=1 STEPS=3 TAG=${TAG}off$r bash tools/env_ab.sh || exit 3
done
( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_trace" -o run \
    -- python3 "$R/bench.py" --workload c2fir --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_trace.txt 2>&1 || { echo "trace failed"; exit 3; }
LIBS="libicw.so ${VLIBS:-libicw_sig4.so}" W=c2fir TAG=${TAG}sq bash tools/sq_pass.sh || exit 3
echo "profiles ok"
