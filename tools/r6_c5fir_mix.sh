#!/bin/bash
# c5fir: where the render's chain waves meet the converter and the dither generator.  Combinations of
# ICW_DITH_OWN (2: CU-masked streams with queues of their own, 0: generator after the converter),
# ICW_K3C_LDS (LDS bytes K3c reserves beyond its own, so fewer other workgroups share its CUs) and
# ICW_FIR_RAMP; two alternating repetitions, every run under its own time limit
mkdir -p gpurun_out; TAG=${TAG:-r6o}
for r in 1 2; do
  for combo in "0 0 -" "2 0 -" "2 65536 -" "2 114688 -" "0 114688 -" "2 114688 1.6" "2 65536 1.6"; do
    set -- $combo
    export ICW_DITH_OWN=$1 ICW_K3C_LDS=$2
    if [ "$3" = "-" ]; then unset ICW_FIR_RAMP; else export ICW_FIR_RAMP=$3; fi
    f=gpurun_out/${TAG}_${1}_${2}_${3}_$r.json
    timeout -k 10 200 python -u bench.py --workload c5fir --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
        > $f 2>>gpurun_out/${TAG}_err.log || { echo "[bench $combo $r] failed"; exit 3; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2:], round(d['value'],1), round(d['ms_per_step'],3))" $f $combo $r
  done
done
echo ok
