#!/bin/bash
# round 3 pass X: one-block calls record no join event (A) against HEAD (B): the stream1 / C-host /
# live-edit tests, then the C1 drop-in leg three times each (the C host links in_cwave_amd/libicw.so,
# so the box's copy of the tree swaps the file between runs)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream1.py tests/test_c_host.py tests/test_gpu_live.py tests/test_gpu_host_io.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3x_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3x_tests.txt
[ $rc -eq 0 ] || exit 2
cp in_cwave_amd/libicw.so in_cwave_amd/libicw_new.so
for r in 1 2 3; do
  for v in new prev; do
    cp in_cwave_amd/libicw_$v.so in_cwave_amd/libicw.so
    timeout -k 10 200 python -u bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3x_${v}_c1_$r.json 2>>gpurun_out/r3x_err.log || exit 3
  done
done
cp in_cwave_amd/libicw_new.so in_cwave_amd/libicw.so
echo ok
