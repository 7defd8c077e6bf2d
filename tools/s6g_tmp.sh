set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-s6g}; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_poseopt.py tests/test_gpu_sim3opt.py tests/test_gpu_gated.py tests/test_gpu_events.py tests/test_gpu_mlpnp.py tests/test_gpu_math.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || rc=$?
echo "pytest rc=$rc" >> $OUT/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
RSC_LIBRSC=tools/bin/librsc_po0.so timeout -k 10 200 python tools/poseopt_probe.py > $OUT/poseopt_probe.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu --no-sim3 --no-events --no-latency --no-bow --no-sim3match --no-kfdb --no-config1 --no-rccl-check > $OUT/bench_lm.json 2> $OUT/bench_lm.err
