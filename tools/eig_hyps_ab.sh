#!/bin/bash
# Diagnostic A/B on one box: headline bench with the product librsc.so against a variant build in
# tools/build/librsc_h19.so (RSC_EIG_HYPS=19: 1,011 eigen-stage waves instead of 960 on config 2),
# interleaved, plus the PnP parity tests through the variant.  Outputs under gpurun_out/$TAG/.
set -e
TAG=${TAG:-eigab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
RSC_LIBRSC=$GRAFT_REPO_ROOT/tools/build/librsc_h19.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests_h19.txt 2>&1
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu --only-headline > $O/base_$i.json 2>/dev/null
  RSC_LIBRSC=$GRAFT_REPO_ROOT/tools/build/librsc_h19.so timeout -k 10 120 python bench.py --no-cpu --only-headline > $O/h19_$i.json 2>/dev/null
done
echo done > $O/done
