#!/bin/bash
# Round 6: k_apply_sparse phase cycles (libgns_sketch_spprof.so, -DGNS_SP_PROF) at configs[4]
# geometry: engine_counters = cycles of thread 0 per phase (map probes, gather + rewrite,
# classify, decide, compact + replay, flush, loop top), then chunks.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_spprof}
mkdir -p $O
for v in ${2:-spprof}; do
  GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_$v.so timeout -k 10 300 python3 bench.py --width 16777216 --depth 8 --no-cpu --windows 0 --steps 3 --warmup 1 > $O/c5_$v.json 2> $O/c5_$v.err
  echo "$v rc=$?"
  python3 -c "
import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); c=list(d['engine_counters'].values()); t=sum(c[:7]); print('$v', d['value'], d['stage_ms_per_step']); print([round(x/t,3) for x in c[:7]], c)"
done
