#!/bin/bash
# GPU-box round script: parity tests, headline bench (with CPU baseline), rocprofv3 kernel stats of
# the same bench command, and two PMC passes (FETCH_SIZE, WRITE_SIZE) of the PnP section for the
# HBM traffic per launch.  Outputs under gpurun_out/$TAG/.  Every step has its own time limit and
# the script stops at the first failure.
set -e
TAG=${TAG:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof_bench.json 2> $OUT/prof.err
PMCARGS="--no-cpu --only-headline --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_write.log 2>&1
if [ -n "$GPUS2" ]; then
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --only-headline --no-cpu --steps 5 --warmup 1 > $OUT/bench_gpus2_gloo.json 2> $OUT/bench_gpus2_gloo.err
  timeout -k 10 300 python bench.py --gpus 2 --strong --dist-backend gloo --only-headline --no-cpu --steps 5 --warmup 1 > $OUT/bench_gpus2_strong_gloo.json 2> $OUT/bench_gpus2_strong_gloo.err
fi
echo done > $OUT/done
