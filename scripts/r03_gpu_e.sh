#!/bin/bash
mkdir -p gpurun_out
for c in clone rec direct auto; do
  DIAG_CASE=$c timeout -k 5 60 python -u scripts/diag_view.py > gpurun_out/r03e_$c.log 2>&1
  echo "$c rc=$?"; grep case gpurun_out/r03e_$c.log | cut -c1-300
done
exit 0
