#!/bin/bash
# split-form eigen stage: chase-wave priority (product) vs none (tools/bin/librsc_noprio.so) vs the
# pair form, headline interleaved
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-prioab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for v in p n 0 p n 0; do
  case $v in
    p) L=orb-slam2-optimized_amd/lib/librsc.so; S=1;;
    n) L=tools/bin/librsc_noprio.so; S=1;;
    0) L=orb-slam2-optimized_amd/lib/librsc.so; S=0;;
  esac
  RSC_EIG_SPLIT=$S RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/prio_ab_$v.jsonl 2>> $OUT/prio_ab.err
done
echo done > $OUT/done
