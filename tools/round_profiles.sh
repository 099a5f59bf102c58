#!/bin/bash
# Summaries of a tools/profile_round.sh run (gpurun_out/prof_<w>, pmc_<w>_*) into profiles/<R>_<w>_*:
#   R=r04 WLS="c2fir c4fir" bash tools/round_profiles.sh
set -e
R=${R:-r04}
for W in ${WLS:-c2 c3 c4 c5}; do
  st=$(find gpurun_out/prof_$W -name '*kernel_stats.csv' | head -1)
  cp "$st" profiles/${R}_${W}_kernel_stats.csv
  fpl=$(python3 -c "
import json,sys
for l in open('gpurun_out/prof_$W.txt'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline') or {}
        print(int(r.get('frames_per_launch') or 0)); break
")
  python3 tools/pmc_summary.py gpurun_out/pmc_${W}_FETCH_SIZE gpurun_out/pmc_${W}_WRITE_SIZE profiles/${R}_${W}_pmc.json \
      --frames-per-launch $fpl --note "$R $W: bench.py --workload $W --steps 2 --warmup 1, FETCH_SIZE / WRITE_SIZE passes" > /dev/null
  python3 tools/sq_summary.py gpurun_out/pmc_${W}_SQ_WAVES gpurun_out/prof_$W profiles/${R}_${W}_sq.json \
      --note "$R $W: SQ pass (bench.py --steps 2 --warmup 1) + kernel-trace stats of bench.py --steps 3" > /dev/null
  echo "$W: frames/launch $fpl"
done
