R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > $O/ab_on_$i.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --no-kernel-timing > $O/ab_off_$i.json 2>/dev/null || exit 1
done
for f in $O/ab_*.json; do echo $f; python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"; done
