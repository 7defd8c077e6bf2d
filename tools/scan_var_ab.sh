#!/bin/bash
# scan variants on one box, headline interleaved: A = packed f32 + double projection (tools/bin/librsc_scanA.so),
# B = float filter, per-point conditional loads (librsc_scanB.so), C = the product library
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-scanvar}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for v in A B C A B C A B C; do
  if [ $v = C ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=tools/bin/librsc_scan$v.so; fi
  RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/scan_var_$v.jsonl 2>> $OUT/scan_var.err
done
echo done > $OUT/done
