#!/bin/bash
# Split-form eigen stage (RSC_EIG_SPLIT=1): parity tests on the large-launch configurations, then
# the headline interleaved against the pair form.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-splitab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
RSC_EIG_SPLIT=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $OUT/split_tests.txt 2>&1
RSC_EIG_SPLIT=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_degenerate.py tests/test_gpu_pnp.py -q --timeout 120 --timeout-method thread >> $OUT/split_tests.txt 2>&1
for v in 0 1 0 1; do
  RSC_EIG_SPLIT=$v timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/split_ab_$v.jsonl 2>> $OUT/split_ab.err
done
echo done > $OUT/done
