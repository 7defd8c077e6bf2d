set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-s6i}; mkdir -p $OUT; cd $GRAFT_REPO_ROOT
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_poseopt.py tests/test_gpu_gated.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || rc=$?
echo "pytest rc=$rc" >> $OUT/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
RSC_LIBRSC=tools/bin/librsc_ponarrowp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_poseopt.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests_narrow.txt 2>&1 || true
for v in po0 poidle1 poidle2 ponarrow po0 poidle1; do echo "== $v" >> $OUT/poseopt_probe.txt; RSC_LIBRSC=tools/bin/librsc_$v.so timeout -k 10 200 python tools/poseopt_probe.py >> $OUT/poseopt_probe.txt 2>&1; done
timeout -k 10 300 python bench.py --no-cpu --no-sim3 --no-mlpnp --no-events --no-latency --no-bow --no-sim3match --no-kfdb --no-config1 --no-rccl-check --no-sim3opt > $OUT/bench_lm.json 2> $OUT/bench_lm.err
