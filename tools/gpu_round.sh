#!/bin/bash
# GPU-box round script: parity tests, headline bench (with CPU baseline), rocprofv3 kernel stats of
# the same bench command, and (PMC=1) two PMC passes (FETCH_SIZE, WRITE_SIZE) of the PnP section for
# the HBM traffic per launch; VARIANTS=1 / PLANAR=1 the round-4 A/B measurements (build first:
# make -C tools qr_bench nonan_lib ldsrows_lib stamps_lib, cp tools/build/qr_bench tools/bin/).  Outputs under gpurun_out/$TAG/.  Every step has its own time limit and
# the script stops at the first failure.
set -e
TAG=${TAG:-run}
# a diagnostic step that fails (a Python error) is recorded and the script goes on; a time limit, an
# abort or a crash ends it (nothing more runs on the GPU after those)
step() {
  local rc=0
  "$@" || rc=$?
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc: $*" >> $OUT/fatal.txt; exit $rc; fi
  [ $rc -eq 0 ] || echo "step rc=$rc: $*" >> $OUT/step_errors.txt
  return 0
}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
nproc > $OUT/host.txt; python3 -c 'import os; print(len(os.sched_getaffinity(0)), os.environ.get("OMP_NUM_THREADS"))' >> $OUT/host.txt
if [ -z "$NO_TESTS" ]; then
  # the whole suite (no -x): test failures (rc 1) are recorded and the later steps still run; any
  # other status (a crash, a time limit) ends the script here
  rc=0
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1 || rc=$?
  echo "pytest rc=$rc" >> $OUT/tests.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.txt 2>&1
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
fi
cd /tmp && export TMPDIR=/tmp
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu > $OUT/prof_bench.json 2> $OUT/prof.err
fi
PMCARGS="--no-cpu --only-headline --steps 5 --warmup 1"
if [ -n "$PMC" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_write.log 2>&1
fi
if [ -n "$SQ" ]; then
  # SQ counters of the headline launches: two passes of 8 SQ counters each (the per-pass limit),
  # tools/pmc_summary.py summarises them
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/pmc_sqA -o a --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_sqA.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM -d $OUT/pmc_sqB -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/pmc_sqB.log 2>&1
fi
if [ -n "$VARIANTS" ]; then
  # off-default A/B variants: their parity tests, the single-event A/B of the rows-form
  # eigen stage, the chase-only sink variants, and the VGPR-row chase library on the headline
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python bench.py --no-cpu --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --eig-rows-ab > $OUT/bench_eig_rows_ab.json 2> $OUT/bench_eig_rows_ab.err
  timeout -k 10 120 tools/bin/qr_bench > $OUT/qr_bench.txt 2>&1
  for v in a b a b; do
    if [ $v = a ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=tools/bin/librsc_ldsrows.so; fi
    RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/ldsrows_ab_$v.jsonl 2>> $OUT/ldsrows_ab.err
  done
  # the small-launch forms on the whole config-2 batch (rows-form eigen stage; uniform betas is
  # pointless there: 57,600 waves)
  for v in a r a r; do
    if [ $v = a ]; then E=0; else E=1000000; fi
    RSC_EIG_ROWS=$E timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/rows_headline_ab_$v.jsonl 2>> $OUT/rows_headline_ab.err
  done
fi
if [ -n "$PLANAR" ]; then
  # planar-content config-2 eigen stage with and without the NaN-block exit
  cd $GRAFT_REPO_ROOT
  timeout -k 10 200 python tools/planar_ab.py $OUT/planar_ab_exit.json exit > $OUT/planar_exit.log 2>&1
  RSC_LIBRSC=tools/bin/librsc_nonanexit.so timeout -k 10 200 python tools/planar_ab.py $OUT/planar_ab_noexit.json noexit > $OUT/planar_noexit.log 2>&1
fi
if [ -n "$LDSAB" ]; then
  # the eigen chase's own Q rows in VGPRs (product) vs in LDS (RSC_EIG_LDSROWS build), headline only
  cd $GRAFT_REPO_ROOT
  for v in a b a b; do
    if [ $v = a ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=tools/bin/librsc_ldsrows.so; fi
    RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/ldsrows_ab_$v.jsonl 2>> $OUT/ldsrows_ab.err
  done
fi
if [ -n "$LAT" ]; then
  # single-event latency with the eigen-form A/B (pairs vs rows)
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python bench.py --no-cpu --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --eig-rows-ab > $OUT/bench_eig_rows_ab.json 2> $OUT/bench_eig_rows_ab.err
fi
if [ -n "$SPINAB" ]; then
  # host wait for a round: hipStreamSynchronize (0) vs spin on a pinned completion flag (1)
  cd $GRAFT_REPO_ROOT
  for v in 0 1 0 1; do
    RSC_SPIN_WAIT=$v timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/spin_ab_$v.jsonl 2>> $OUT/spin_ab.err
    RSC_SPIN_WAIT=$v TIMING=0 timeout -k 10 120 python tools/host_overhead.py >> $OUT/host_overhead_spin$v.txt 2>&1
    RSC_SPIN_WAIT=$v timeout -k 10 300 python bench.py --no-cpu --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --no-mlpnp --no-events --no-sim3 >> $OUT/spin_ab_lat_$v.jsonl 2>> $OUT/spin_ab.err
  done
fi
if [ -n "$PROBE" ]; then
  # per-phase device clocks of the Refine kernel (stamped build: make -C tools stamps_lib)
  cd $GRAFT_REPO_ROOT
  RSC_LIBRSC=tools/bin/librsc_stamps.so timeout -k 10 200 python tools/refine_probe.py event > $OUT/refine_probe_event.txt 2>&1
fi
if [ -n "$GPUS2" ]; then
  cd $GRAFT_REPO_ROOT
  timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu --no-latency --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --steps 8 --warmup 2 > $OUT/bench_gpus2_gloo.json 2> $OUT/bench_gpus2_gloo.err
  timeout -k 10 300 python bench.py --gpus 4 --dist-backend gloo --no-cpu --no-latency --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --steps 8 --warmup 2 > $OUT/bench_gpus4_gloo.json 2> $OUT/bench_gpus4_gloo.err
fi
if [ -n "$REFAB" ]; then
  # Refine phase stamps of the single relocalization event for stamped builds of the libraries named
  # in REFAB (tools/bin/librsc_<name>.so: make -C tools variant NAME=<name> DEFS=...), interleaved
  cd $GRAFT_REPO_ROOT
  for rep in 1 2; do
    for v in $REFAB; do
      echo "== $v rep $rep" >> $OUT/refine_probe_$v.txt
      step env RSC_LIBRSC=tools/bin/librsc_$v.so timeout -k 10 120 python tools/refine_probe.py event >> $OUT/refine_probe_$v.txt 2>&1
    done
  done
fi
if [ -n "$LIBAB" ]; then
  # headline + single-event latency per library (product = "product"), interleaved twice
  cd $GRAFT_REPO_ROOT
  for rep in 1 2; do
    for v in $LIBAB; do
      if [ $v = product ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=tools/bin/librsc_$v.so; fi
      step env RSC_LIBRSC=$L timeout -k 10 300 python bench.py --no-cpu --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --no-mlpnp --no-events --no-sim3 >> $OUT/libab_$v.jsonl 2>> $OUT/libab.err
    done
  done
fi
if [ -n "$ML" ]; then
  # config-4 MLPnP kernel: phase stamps (stamped build), kernel trace, two SQ
  # passes and the HBM traffic passes of the bench's 128 x 4096 launch (tools/mlpnp_probe.py)
  cd $GRAFT_REPO_ROOT
  step env RSC_LIBRSC=tools/bin/librsc_mlstamps.so timeout -k 10 200 python tools/mlpnp_probe.py 128 stamps > $OUT/mlpnp_probe.txt 2>&1
  cd /tmp
  P="python3 $GRAFT_REPO_ROOT/tools/mlpnp_probe.py 128 run 4"
  step env timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ml_prof -o ml --output-format csv -- $P > $OUT/ml_prof.log 2>&1
  step env timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $OUT/ml_sqA -o a --output-format csv -- $P > $OUT/ml_sqA.log 2>&1
  step env timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM -d $OUT/ml_sqB -o b --output-format csv -- $P > $OUT/ml_sqB.log 2>&1
  step env timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/ml_fetch -o f --output-format csv -- $P > $OUT/ml_fetch.log 2>&1
  step env timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/ml_write -o w --output-format csv -- $P > $OUT/ml_write.log 2>&1
fi
if [ -n "$VARTEST" ]; then
  # the Refine / event parity tests against an A/B library (tools/bin/librsc_<name>.so)
  cd $GRAFT_REPO_ROOT
  for v in $VARTEST; do
    step env RSC_LIBRSC=tools/bin/librsc_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_events.py tests/test_gpu_degenerate.py tests/test_gpu_gated.py "tests/test_gpu_configs.py::test_config2_parity_batch_with_refine" "tests/test_gpu_configs.py::test_config5_full_event_stream" -m gpu -q --timeout 180 --timeout-method thread > $OUT/vartest_$v.txt 2>&1 || echo "rc=$?" >> $OUT/vartest_$v.txt
  done
fi
if [ -n "$POAB" ]; then
  # PoseOptimization pass timing per library (tools/poseopt_probe.py; RSC_POSE_PHASES builds)
  cd $GRAFT_REPO_ROOT
  for v in $POAB; do
    echo "== $v" >> $OUT/poseopt_probe.txt
    step env RSC_LIBRSC=tools/bin/librsc_$v.so timeout -k 10 200 python tools/poseopt_probe.py >> $OUT/poseopt_probe.txt 2>&1
  done
fi
if [ -n "$TRAFAB" ]; then
  # HBM traffic attribution of the headline launch set: FETCH_SIZE / WRITE_SIZE passes per library
  # (product = "product", else tools/bin/librsc_<name>.so)
  cd /tmp
  for v in $TRAFAB; do
    if [ $v = product ]; then L=$GRAFT_REPO_ROOT/orb-slam2-optimized_amd/lib/librsc.so; else L=$GRAFT_REPO_ROOT/tools/bin/librsc_$v.so; fi
    step env RSC_LIBRSC=$L timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/traf_fetch_$v -o f --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/traf_fetch_$v.log 2>&1
    step env RSC_LIBRSC=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/traf_write_$v -o w --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $PMCARGS > $OUT/traf_write_$v.log 2>&1
  done
fi
if [ -n "$SOLVEPROBE" ]; then
  cd $GRAFT_REPO_ROOT
  step env RSC_LIBRSC=tools/bin/librsc_solvestamps.so timeout -k 10 120 python tools/solve_probe.py event > $OUT/solve_probe_event.txt 2>&1
fi
if [ -n "$ENVAB" ]; then
  # headline + single-event latency per environment setting (e.g. "RSC_BETAS_HB=64 RSC_BETAS_HB=16"), interleaved twice
  cd $GRAFT_REPO_ROOT
  for rep in 1 2; do
    for v in $ENVAB; do
      step env $v timeout -k 10 300 python bench.py --no-cpu --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb --no-config1 --no-mlpnp --no-events --no-sim3 >> $OUT/envab_$v.jsonl 2>> $OUT/envab.err
    done
  done
fi
if [ -n "$ENVTEST" ]; then
  # the Refine / event parity tests under an environment setting of the product library
  cd $GRAFT_REPO_ROOT
  for v in $ENVTEST; do
    step env $v timeout -k 10 400 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_events.py tests/test_gpu_degenerate.py tests/test_gpu_gated.py "tests/test_gpu_configs.py::test_config2_parity_batch_with_refine" "tests/test_gpu_configs.py::test_config5_full_event_stream" -m gpu -q --timeout 180 --timeout-method thread > $OUT/envtest_$v.txt 2>&1
  done
fi
echo done > $OUT/done
