#!/bin/bash
# Diagnostic: GPU parity tests, then the headline bench once per solve mode (no CPU baseline).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t_modes.txt 2>&1
for m in ${MODES:-split quad mono}; do
  RSC_SOLVE_MODE=$m timeout -k 10 200 python bench.py --no-cpu --no-sim3 > gpurun_out/b_$m.json 2>&1
done
