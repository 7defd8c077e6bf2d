#!/bin/bash
# A/B of the betas stage's hypotheses per wave: product (64) vs tools/bin/librsc_betas32.so (32),
# headline bench interleaved, plus the config parity tests on the variant.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-betasab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
RSC_LIBRSC=tools/bin/librsc_betas32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_degenerate.py -q --timeout 180 --timeout-method thread > $OUT/betas32_tests.txt 2>&1
for v in a b a b; do
  if [ $v = a ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=tools/bin/librsc_betas32.so; fi
  RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/betas_ab_$v.jsonl 2>> $OUT/betas_ab.err
done
echo done > $OUT/done
