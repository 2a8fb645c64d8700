#!/bin/bash
# Round 6: C2 with the HEAD side stream only (AAA_SIDE 0 / 1, same box), then the driver's default line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r06c2s; mkdir -p $O; cd $R; export TMPDIR=/tmp
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-dropin --no-episode > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$n',d['value'],d['ms_per_step'],{n[:14]:round(v.get('ms',v.get('avg_us',0)/1e3),4) for n,v in k.items()})"
}
for v in 0 1 0 1 0 1; do run c2_s$v AAA_SIDE=$v; mv $O/c2_s$v.json $O/c2_s${v}_$RANDOM.json; done
timeout -k 10 600 python bench.py > $O/default.json 2> $O/default.err || { echo "default rc=$?"; tail -5 $O/default.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/default.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('episode',{}).get('episode_frames_per_s'), d.get('cpu_baseline',{}).get('value'))"
echo done
