#!/bin/bash
# round 3 pass F: K5 phase stamps of the one-stream drop-in (576 / 1152 / 2304 / 4096-frame calls)
mkdir -p gpurun_out
python tools/c1_wav.py /tmp/c1.wav 10 || exit 1
for b in 576 1152 2304 4096; do
  ICW_TIMING=1 ICW_S1_STAMPS=1 timeout -k 10 120 ./examples/icw_transcode /tmp/c1.wav /tmp/c1_out.wav $b shift 16 \
    > gpurun_out/r3f_c1_$b.json 2> gpurun_out/r3f_c1_$b.stamps || exit 2
  python tools/s1_phases.py gpurun_out/r3f_c1_$b.stamps
  tail -1 gpurun_out/r3f_c1_$b.json
done
