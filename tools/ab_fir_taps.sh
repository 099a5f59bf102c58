#!/bin/bash
# FIR taps from SGPRs: GPU parity of the FIR converter, then old / new library A/B on the FIR legs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fir_tests.log 2>&1 || exit 1
for r in 1 2; do
  for lib in libicw_ab_old.so libicw.so; do
    for w in c2fir c3fir c4fir; do
      ICW_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/abfir_${w}_${lib}_$r.json 2>>gpurun_out/abfir_err.log || exit 2
    done
  done
done
echo ok
