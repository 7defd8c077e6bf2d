set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS="--no-cpu --no-sim3 --no-mlpnp --no-events --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $R/gpurun_out/pmcA -o a --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcA.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmcB -o b --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcB.log 2>&1
echo ok
