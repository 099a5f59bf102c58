#!/bin/bash
# round 3 pass Q: KF2 chain programs read through the constant address space (A/B against
# the previous commit built as libicw_prev.so): FIR parity, the FIR legs, the cost-split probe
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_unaligned.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3q_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3q_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for lib in libicw.so libicw_prev.so; do
    for w in c2fir c3fir c4fir; do
      ICW_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3q_${lib%.so}_${w}_$r.json 2>>gpurun_out/r3q_err.log || exit 3
    done
  done
done
echo "[legs] ok"
ICW_LIB=libicw.so timeout -k 10 300 python -u tools/fir_probe.py > gpurun_out/r3q_fir_probe.jsonl 2>>gpurun_out/r3q_err.log || exit 4
cat gpurun_out/r3q_fir_probe.jsonl
echo ok
