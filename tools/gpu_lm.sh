#!/bin/bash
# GPU-box script for the LM kernels (PoseOptimization, OptimizeSim3): their parity tests (plus the
# gated events, the fault path and the device math self-tests), the phase-clock probes of the
# variant libraries named in POVARS / SOVARS (tools/bin/librsc_<name>.so, built with
# make -C tools variant NAME=<name> SRC=poseopt|sim3opt DEFS="-DRSC_POSE_PHASES=1 ..." /
# "-DRSC_SO_PHASES=1 ..."), and the bench's LM sections.  Outputs under gpurun_out/$TAG/.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-lm}; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_poseopt.py tests/test_gpu_sim3opt.py tests/test_gpu_gated.py tests/test_gpu_events.py tests/test_gpu_fault.py tests/test_gpu_math.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || rc=$?
echo "pytest rc=$rc" >> $OUT/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in $SOVARS; do echo "== $v" >> $OUT/sim3opt_probe.txt; RSC_LIBRSC=tools/bin/librsc_$v.so timeout -k 10 200 python tools/sim3opt_probe.py >> $OUT/sim3opt_probe.txt 2>&1; done
for v in $POVARS; do echo "== $v" >> $OUT/poseopt_probe.txt; RSC_LIBRSC=tools/bin/librsc_$v.so timeout -k 10 200 python tools/poseopt_probe.py >> $OUT/poseopt_probe.txt 2>&1; done
timeout -k 10 300 python bench.py --no-cpu --no-sim3 --no-mlpnp --no-events --no-latency --no-bow --no-sim3match --no-kfdb --no-config1 --no-rccl-check > $OUT/bench_lm.json 2> $OUT/bench_lm.err
echo done > $OUT/done
