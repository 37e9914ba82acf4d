cd $GRAFT_REPO_ROOT
for f in 16384 262144 1048576 4194304; do
  timeout -k 10 200 python bench.py --no-cpu --flows $f > gpurun_out/flows_$f.json 2>gpurun_out/flows_$f.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/flows_$f.json')); print($f, d['value'], d['stage_ms_per_step'])"
done
