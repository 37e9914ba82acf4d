#!/bin/bash
# K4 phase cycles (GNS_K4_PROF build, wave 0's s_memtime per phase summed over chunks) at the
# headline and configs[4] geometries.  Build first: make -C go2netspectra_amd/csrc variant NAME=k4p
# VARIANT_FLAGS=-DGNS_K4_PROF.  engine_counters then read: inserted=classify, dropped=decide,
# unsupported=compact, dict_full=replay clear + loop top, ovf_full=summed per-wave replay cycles,
# replayed=tile load + store, chunks=the slowest wave's replay cycles, chunks_replay=replay groups.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
export GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_k4p.so
timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --warmup 1 --windows 0 > $O/k4p_c2.json 2> $O/k4p_c2.err &&
timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --warmup 1 --windows 0 --width 16777216 --depth 8 > $O/k4p_c5.json 2> $O/k4p_c5.err &&
for w in c2 c5; do python3 -c "
import json
d=json.loads(open('$O/k4p_$w.json').read().strip().splitlines()[-1])
c=d['engine_counters']
ph=[('classify','inserted'),('decide','dropped'),('compact','unsupported'),('replay barrier + top','dict_full'),('tile load + store','replayed'),('replay groups','chunks_replay')]
tot=sum(c[k] for _,k in ph)
print('$w', d['stage_ms_per_step'].get('apply'), ' '.join(f'{n}={100*c[k]/tot:.1f}%' for n,k in ph),
      'replay balance (slowest wave cycles x 16 / all) =', round(c['chunks']*16/max(c['ovf_full'],1), 2))
"; done
