#!/bin/bash
# c5fir's block ramp with the dither generator after the converter (the default streams): first block
# (ICW_FIRST_BLOCK) x ramp (ICW_FIR_RAMP) as COMBOS="first:ramp ..." (- = the default), three alternating
# repetitions, every run its own time limit
mkdir -p gpurun_out; TAG=${TAG:-r6p}
for r in 1 2 3; do
  for combo in ${COMBOS:--:- -:1.4 -:1.6 -:1.8 8192:- 8192:1.6 2048:1.6}; do
    set -- ${combo/:/ }
    if [ "$1" = "-" ]; then unset ICW_FIRST_BLOCK; else export ICW_FIRST_BLOCK=$1; fi
    if [ "$2" = "-" ]; then unset ICW_FIR_RAMP; else export ICW_FIR_RAMP=$2; fi
    f=gpurun_out/${TAG}_${1}_${2}_$r.json
    timeout -k 10 200 python -u bench.py --workload c5fir --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
        > $f 2>>gpurun_out/${TAG}_err.log || { echo "[bench $combo $r] failed"; exit 3; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2:], round(d['value'],1), round(d['ms_per_step'],3))" $f $combo $r
  done
done
echo ok
