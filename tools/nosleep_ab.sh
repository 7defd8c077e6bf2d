#!/bin/bash
# Split-form eigen stage polling without s_sleep (tools/bin/librsc_nosleep.so) vs s_sleep 1 (the product):
# headline interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-nosleep}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
RSC_LIBRSC=tools/bin/librsc_nosleep.so timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_configs.py tests/test_gpu_pnp.py tests/test_gpu_degenerate.py -x -q --timeout 120 --timeout-method thread > $OUT/nosleep_tests.txt 2>&1
for v in a b a b a b; do
  if [ $v = a ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=tools/bin/librsc_nosleep.so; fi
  RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/ab_$v.jsonl 2>> $OUT/ab.err
done
echo done > $OUT/done
