#!/bin/bash
# A/B of one environment knob on one GPU box:  VAR=ICW_REST_CUS VALS="0 96 128" WLS="c3 c4" REPS=2 TAG=x bash tools/env_ab.sh
# (value "-" leaves the variable unset).  Every bench run has its own time limit; stops at the first failure.
mkdir -p gpurun_out
TAG=${TAG:-env}
for r in $(seq 1 ${REPS:-2}); do
  for W in ${WLS:-c3}; do
    for v in ${VALS:-"-"}; do
      if [ "$v" = "-" ]; then unset $VAR; else export $VAR=$v; fi
      timeout -k 10 ${BENCH_LIMIT:-200} python -u bench.py --workload $W --steps ${STEPS:-3} --warmup 1 \
          --no-cpu-baseline --e2e-steps 0 > gpurun_out/${TAG}_${W}_${v}_$r.json 2>>gpurun_out/${TAG}_err.log \
          || { echo "[bench $W $VAR=$v $r] failed"; exit 3; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['value'],1), round(d['ms_per_step'],3))" \
          gpurun_out/${TAG}_${W}_${v}_$r.json $W "$VAR=$v" $r
    done
  done
done
echo ok
