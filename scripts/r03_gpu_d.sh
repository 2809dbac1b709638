#!/bin/bash
# round 3, pass d: config C shard 3 stall hunt -- (1) its own 4M-row tensor, all 1M queries in
# one call; (2) a view of the 32M-row tensor with the queries in passes of 65536
# (KNN_WS_QUERIES); (3) shard 3 alone as a view, 1M queries, profile stages per pass.
mkdir -p gpurun_out
DIAG_NQ=1000000 DIAG_SHARDS=3 timeout -k 5 75 python -u scripts/diag_c_shards.py > gpurun_out/r03d_1.log 2>&1
echo "(1) own tensor, 1M queries: rc=$?"; grep -v '\.\.\.' gpurun_out/r03d_1.log | tail -3 | cut -c1-400
KNN_WS_QUERIES=65536 DIAG_ORDER=3 timeout -k 5 100 python -u scripts/repro_c.py > gpurun_out/r03d_2.log 2>&1
echo "(2) view, passes of 65536: rc=$?"; grep -v '\.\.\.' gpurun_out/r03d_2.log | tail -3 | cut -c1-400
DIAG_ORDER=4 timeout -k 5 75 python -u scripts/repro_c.py > gpurun_out/r03d_3.log 2>&1
echo "(3) view, shard 4, 1M queries: rc=$?"; grep -v '\.\.\.' gpurun_out/r03d_3.log | tail -3 | cut -c1-400
exit 0
