#!/bin/bash
# r03 (t): kernel trace of the multi-rank legs at one rank (config-3 chain, sharded
# config 5) for the config-3 split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --multi-legs --no-gw --no-batch-ot --no-cpu-baseline --no-hbm-probe --no-config5 --no-f64 > $O/bench.log 2>&1; rc=$?
grep -o '"config3_epoch_chain": {[^}]*}' $O/bench.log; exit $rc
