#!/bin/bash
# counts written by the scan straight into pinned host memory (1, default) vs into HBM + a D2H copy (0)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-dcab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for v in 1 0 1 0; do
  RSC_DIRECT_COUNTS=$v timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/dc_$v.jsonl 2>> $OUT/dc.err
done
echo done > $OUT/done
