#!/bin/bash
# quick per-workload bench: prints value ms K1 K2
mkdir -p gpurun_out
for spec in "$@"; do
  w=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  env $envs timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wl_${w}_${envs//[= ]/_}.txt 2>&1 || exit 2
  echo "$spec $(grep '^{' gpurun_out/wl_${w}_${envs//[= ]/_}.txt | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value'],1), round(d['ms_per_step'],2), 'K1', round(r['avg_launch_ms'],3), 'K2', round(r['output_kernel_avg_launch_ms'],3))")" | tee -a gpurun_out/wl_summary.txt
done
