#!/bin/bash
# round 3 pass U: KF2 tile loop (tiles per workgroup, next tile's new frames by LDS DMA beside the graph
# phase) -- FIR parity incl. full size, then the FIR legs: ICW_FIR_TPW 1 / 2 / default(4) / 8 against
# HEAD (libicw_prev.so), twice each
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_unaligned.py "tests/test_gpu_full_size.py::test_full_size_step[c2fir]" "tests/test_gpu_full_size.py::test_full_size_step[c4fir]" "tests/test_gpu_full_size.py::test_full_size_step[c3fir]" -x -q --timeout 200 --timeout-method thread > gpurun_out/r3u_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3u_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for v in prev 1 d 8 16; do
    lib=libicw.so; env=""
    [ $v = prev ] && lib=libicw_prev.so
    case $v in 1|2|8|16) env="ICW_FIR_TPW=$v";; esac
    for w in ${WLS:-c2fir c3fir c4fir}; do
      env $env ICW_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3u_${v}_${w}_$r.json 2>>gpurun_out/r3u_err.log || exit 3
    done
  done
done
echo ok
