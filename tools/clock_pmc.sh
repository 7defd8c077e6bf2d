#!/bin/bash
# Effective shader clock per kernel of the headline launch set: GRBM_GUI_ACTIVE / 8 XCDs / kernel
# time (MI355X_MICROARCH.md, DVFS), one PMC pass; then the SQ pass A of gpu_round.sh.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-clk}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PMCARGS="--no-cpu --only-headline --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $OUT/pmc_clk -o c --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_clk.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sqA -o a --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_sqA.log 2>&1
echo done > $OUT/done
