#!/bin/bash
# round 3 pass V: KF2 stereo chain path with the second pass's rotation factors loaded before the
# first pass (A) against HEAD (libicw_prev.so): FIR parity incl. full size, then the FIR legs twice
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_graph_random.py "tests/test_gpu_full_size.py::test_full_size_step[c2fir]" "tests/test_gpu_full_size.py::test_full_size_step[c4fir]" -x -q --timeout 200 --timeout-method thread > gpurun_out/r3v_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3v_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for lib in libicw.so libicw_prev.so; do
    for w in c2fir c4fir; do
      ICW_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3v_${lib%.so}_${w}_$r.json 2>>gpurun_out/r3v_err.log || exit 3
    done
  done
done
echo ok
