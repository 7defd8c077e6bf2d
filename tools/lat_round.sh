#!/bin/bash
# GPU-box script for the single-event latency work: GPU tests (unless NO_TESTS), the latency event
# with the fused select+refine on and off, the refine phase probe, and a rocprofv3 kernel trace of the
# latency event alone.  Outputs under gpurun_out/$TAG/.
set -e
TAG=${TAG:-lat}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/tests.txt 2>&1
fi
timeout -k 10 120 python tools/latency_trace.py reloc 100 > $OUT/lat_fused.txt 2>&1
RSC_FUSED_REFINE=0 timeout -k 10 120 python tools/latency_trace.py reloc 100 > $OUT/lat_unfused.txt 2>&1
timeout -k 10 120 python tools/latency_trace.py reloc 100 >> $OUT/lat_fused.txt 2>&1
timeout -k 10 120 python tools/latency_trace.py loop 100 > $OUT/lat_loop.txt 2>&1
timeout -k 10 120 python tools/refine_latency_probe.py tools/bin/librsc_stamps.so > $OUT/refine_probe.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_lat -o lat --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/latency_trace.py reloc 50 > $OUT/prof_lat.txt 2>&1
echo done > $OUT/done
