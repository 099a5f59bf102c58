#!/bin/bash
# round 3 pass J: K5 completion polled in host memory (ICW_SPIN A/B on C1), and the KF2 cost split
# by order and graph (tools/fir_probe.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3j_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3j_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for sp in 1 0; do
    ICW_SPIN=$sp timeout -k 10 300 python -u bench.py --workload c1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3j_c1_sp${sp}_$r.json 2>>gpurun_out/r3j_err.log || exit 3
    python3 -c "import json;d=json.loads(open('gpurun_out/r3j_c1_sp${sp}_$r.json').read().strip().splitlines()[-1]);print('spin $sp', round(d['value'],3), d['block_latency_us'])"
  done
done
timeout -k 10 300 python -u tools/fir_probe.py > gpurun_out/r3j_fir_probe.jsonl 2>>gpurun_out/r3j_err.log || exit 4
cat gpurun_out/r3j_fir_probe.jsonl
echo ok
