#!/bin/bash
# Round 6: attribute K1's bytes with counters.  The product library and the timing
# ablation (libgns_sketch_k1abl.so, -DGNS_K1_ABL_DICT: the dictionary probe reads one of
# 4096 L2-resident records; wrong counters, timing only) each run the headline bench
# (3 steps) under a kernel trace, then one FETCH_SIZE and one WRITE_SIZE pass.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r06_k1abl}
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --windows 0"
# The ablation's fingerprints name arbitrary slots, so its run ends with the heavy-hitter
# list's GNS_E_HIP ("names no dictionary slot") after the timed steps: rc 1 is expected
# there (status 124/137 = a time limit still stops the script).
ok() { local rc=$1 v=$2; [ $rc -eq 0 ] || { [ $v = abl ] && [ $rc -eq 1 ]; }; }
for v in ${VARIANTS:-prod abl}; do
    mkdir -p $O/$v
    if [ $v = abl ]; then export GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_k1abl.so; else unset GNS_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v/trace -o cm -- $B > $O/$v/trace.log 2>&1; ok $? $v || { echo "FAIL trace $v"; exit 1; }
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$v/fetch -o cm -- $B > $O/$v/fetch.log 2>&1; ok $? $v || { echo "FAIL fetch $v"; exit 1; }
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$v/write -o cm -- $B > $O/$v/write.log 2>&1; ok $? $v || { echo "FAIL write $v"; exit 1; }
    python3 tools/pmc_traffic.py $O/$v/fetch/*counter_collection.csv $O/$v/write/*counter_collection.csv $O/$v/traffic.json > $O/$v/traffic.txt 2>&1
    python3 tools/prof_steady.py --last 3 $O/$v/trace/*kernel_trace.csv k_extract k_scatter_st k_apply > $O/$v/steady.txt 2>&1
    echo "== $v"; cat $O/$v/steady.txt; cat $O/$v/traffic.txt | head -20
done
