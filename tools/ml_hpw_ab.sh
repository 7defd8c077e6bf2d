set -e
O=gpurun_out/r3b; mkdir -p $O
for w in 64 32 16 8; do
  RSC_ML_HPW=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_mlpnp.py tests/test_gpu_configs.py -k "mlpnp or config4" -x -q --timeout 200 --timeout-method thread > $O/tests_$w.txt 2>&1
  RSC_ML_HPW=$w timeout -k 10 200 python bench.py --no-cpu --no-sim3 --no-events --no-latency --no-poseopt --no-bow --no-sim3match --no-sim3opt --no-kfdb > $O/bench_$w.json 2> $O/bench_$w.err
done
