#!/bin/bash
# GPU-box script for the MLPnP kernel work: parity tests, config-4 timings at 128 and 32 candidates,
# and a rocprofv3 kernel trace of the 32-candidate section.  Outputs under gpurun_out/$TAG/.
set -e
TAG=${TAG:-ml}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
ONLY="--no-cpu --no-sim3 --no-events --no-latency --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --no-rccl-check"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_mlpnp.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
fi
timeout -k 10 300 python bench.py $ONLY > $OUT/bench128.json 2> $OUT/bench128.err
timeout -k 10 300 python bench.py $ONLY --mlpnp-candidates 32 > $OUT/bench32.json 2> $OUT/bench32.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ml --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ONLY --mlpnp-candidates 32 --steps 8 > $OUT/prof.txt 2>&1
echo done > $OUT/done
