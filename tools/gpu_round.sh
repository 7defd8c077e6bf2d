#!/bin/bash
# GPU-box round script: parity tests, headline bench (with CPU baseline), rocprofv3 kernel stats of
# the same bench command.  Outputs under gpurun_out/$TAG/.
set -e
TAG=${TAG:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/tests.txt 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof_bench.json 2> $OUT/prof.err
