#!/bin/bash
# tridiag_qr's non-finite-block test every 8th QR step (the product) vs every step
# (tools/bin/librsc_nancheck1.so, or LIBB): the whole GPU suite on the product, then the headline
# interleaved, then one full bench line (single-event latency) per library.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-nancheck}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1
for v in a b a b a b; do
  if [ $v = a ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=${LIBB:-tools/bin/librsc_nancheck1.so}; fi
  RSC_LIBRSC=$L timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/ab_$v.jsonl 2>> $OUT/ab.err
done
for v in a b; do
  if [ $v = a ]; then L=orb-slam2-optimized_amd/lib/librsc.so; else L=${LIBB:-tools/bin/librsc_nancheck1.so}; fi
  RSC_LIBRSC=$L timeout -k 10 300 python bench.py --no-cpu > $OUT/full_$v.json 2>> $OUT/ab.err
done
echo done > $OUT/done
