#!/bin/bash
# Interleaved headline A/B of two library builds on one box: LIBA vs LIBB (paths), 3 rounds each
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-libab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for v in a b a b a b; do
  if [ $v = a ]; then L=$LIBA; else L=$LIBB; fi
  RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/ab_$v.jsonl 2>> $OUT/ab.err
done
echo done > $OUT/done
