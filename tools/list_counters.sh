#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -s KILL 60 rocprofv3 --list-avail > $OLDPWD/gpurun_out/r5_counters_avail.txt 2>&1; echo rc=$?
