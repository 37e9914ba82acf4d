#!/bin/bash
# SuperSpread bench A/B over an env knob: tools/ab_ss.sh VAR val1 val2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 200 python bench.py --sketch superspread --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_ss_$v.json 2> gpurun_out/ab_ss_$v.err
  rc=$?
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_ss_$v.json').read()); print('$var=$v', d['value'], d['stage_ms_per_step'])" | tee -a gpurun_out/ab.log
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; exit $rc; fi
done
