#!/bin/bash
# round 3 pass K: K5's output phase beside the recurrence (ICW_S1_OVL A/B): parity, C1 timing,
# phase stamps; and the KF2 cost split (tools/fir_probe.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3k_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3k_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for ov in 1 0; do
    ICW_S1_OVL=$ov timeout -k 10 300 python -u bench.py --workload c1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3k_c1_ov${ov}_$r.json 2>>gpurun_out/r3k_err.log || exit 3
    python3 -c "import json;d=json.loads(open('gpurun_out/r3k_c1_ov${ov}_$r.json').read().strip().splitlines()[-1]);print('ovl $ov', round(d['value'],3), d['block_latency_us'])"
  done
done
python tools/c1_wav.py /tmp/c1.wav 10 || exit 5
for ov in 1 0; do
  ICW_S1_OVL=$ov ICW_TIMING=1 ICW_S1_STAMPS=1 timeout -k 10 120 ./examples/icw_transcode /tmp/c1.wav /tmp/c1_out.wav 576 shift 16 \
      > gpurun_out/r3k_c1_576_ov$ov.json 2> gpurun_out/r3k_c1_576_ov$ov.stamps || exit 6
  echo "ovl $ov"; python tools/s1_phases.py gpurun_out/r3k_c1_576_ov$ov.stamps
done
timeout -k 10 300 python -u tools/fir_probe.py > gpurun_out/r3k_fir_probe.jsonl 2>>gpurun_out/r3k_err.log || exit 4
cat gpurun_out/r3k_fir_probe.jsonl
echo ok
