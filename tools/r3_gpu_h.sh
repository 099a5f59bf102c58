#!/bin/bash
# round 3 pass H: the geometric tail for the lane kernel again, now that K0 + K2 take ~0.75-0.79 of
# K1 per frame (C3 / C4): ICW_TAPER 0 (default), 0.85, 0.8, 0.75; and the FIR staging's uniform
# fade / history skips on the FIR legs
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3h_fir.txt 2>&1
rc=$?; echo "[fir tests] rc=$rc"; tail -2 gpurun_out/r3h_fir.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for tp in 0 0.85 0.8 0.75; do
    for w in c3 c4; do
      ICW_TAPER=$tp timeout -k 10 200 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3h_tp${tp}_${w}_$r.json 2>>gpurun_out/r3h_err.log || exit 3
    done
  done
done
echo "[taper ab] ok"
for w in c2fir c3fir c4fir; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
    > gpurun_out/r3h_$w.json 2>>gpurun_out/r3h_err.log || exit 4
done
echo ok
