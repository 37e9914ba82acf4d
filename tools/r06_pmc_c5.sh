#!/bin/bash
# Round 6: PMC HBM traffic per kernel at the configs[4] geometry with the sparse K4, for
# 100M- and 200M-packet device batches (one FETCH_SIZE and one WRITE_SIZE pass each), then
# tools/pmc_traffic.py -> gpurun_out/<tag>/traffic_b<batch>.json
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r06_pmc_c5}
mkdir -p $O
for P in 100000000 200000000; do
  B="python3 bench.py --steps 3 --warmup 1 --no-cpu --windows 0 --width 16777216 --depth 8 --packets $P"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$P -o cm -- $B > $O/fetch_$P.log 2>&1 || { echo "FAIL fetch $P"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$P -o cm -- $B > $O/write_$P.log 2>&1 || { echo "FAIL write $P"; exit 1; }
  python3 tools/pmc_traffic.py $O/fetch_$P/*counter_collection.csv $O/write_$P/*counter_collection.csv $O/traffic_b$P.json > $O/traffic_b$P.txt 2>&1
  echo "== $P"; grep -E "k_extract|k_scatter_st|k_apply|k_hot_hist|k_hot_collect" $O/traffic_b$P.txt
done
