#!/bin/bash
# Refresh the round's evidence on one GPU box: kernel stats + PMC passes of C2 / C5, then the
# driver's default bench line.  Each step has its own time limit; the first failure stops it.
set -o pipefail
WLS="c2 c5" bash tools/profile_round.sh > gpurun_out/profile_round.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 3
echo refresh-ok
