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
if [ -n "$SQ" ]; then
  # SQ counters of the headline launches (eig-stage waves per SIMD, issue / wait shares): two passes
  # of 8 SQ counters each (the per-pass limit), tools/pmc_summary.py summarises them
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sqA -o a --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_sqA.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM -d $OUT/pmc_sqB -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_sqB.log 2>&1
fi
if [ -n "$GPUS2" ]; then
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --only-headline --no-cpu --steps 5 --warmup 1 > $OUT/bench_gpus2_gloo.json 2> $OUT/bench_gpus2_gloo.err
  timeout -k 10 300 python bench.py --gpus 2 --strong --dist-backend gloo --only-headline --no-cpu --steps 5 --warmup 1 > $OUT/bench_gpus2_strong_gloo.json 2> $OUT/bench_gpus2_strong_gloo.err
fi
echo done > $OUT/done
