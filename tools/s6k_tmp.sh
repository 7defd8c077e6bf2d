set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-s6k}; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_poseopt.py tests/test_gpu_sim3opt.py tests/test_gpu_gated.py tests/test_gpu_events.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || rc=$?
echo "pytest rc=$rc" >> $OUT/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in po0 pon3 pow7 po0 pon3; do echo "== $v" >> $OUT/poseopt_probe.txt; RSC_LIBRSC=tools/bin/librsc_$v.so timeout -k 10 200 python tools/poseopt_probe.py >> $OUT/poseopt_probe.txt 2>&1; done
timeout -k 10 300 python bench.py --no-cpu --no-sim3 --no-mlpnp --no-events --no-latency --no-bow --no-sim3match --no-kfdb --no-config1 --no-rccl-check > $OUT/bench_lm.json 2> $OUT/bench_lm.err
RSC_LIBRSC=tools/bin/librsc_pon3p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_poseopt.py tests/test_gpu_gated.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests_narrow.txt 2>&1 || true
