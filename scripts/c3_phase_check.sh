cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3t
for i in 1 2; do timeout -k 10 300 python bench.py --workload c3 --steps 50 --warmup 5 --no-cpu > gpurun_out/c3t/c3_$i.log 2>&1 || exit $?; done
python - <<'P'
import json
for i in (1,2):
    for l in open(f'gpurun_out/c3t/c3_{i}.log'):
        if l.startswith('{'):
            d=json.loads(l); g=d['phases']['gradients']; r=d['phases']['round']
            print(i, round(d['value'],1), 'grad', round(g['launch_ms']*1e3,1), 'step-round', round(g['step_minus_round_ms']*1e3,1), 'frac', round(g['frac'],3), 'rocprof', g['rocprof_launch_ms'], 'round', round(r['launch_ms']*1e3,1), g['kernel'][-90:])
P
