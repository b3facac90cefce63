#!/bin/bash
# c3 round-phase grid/tile sweep: balanced persistent grid on/off, 128- vs 64-column tiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c3grid
mkdir -p $OUT
i=0
for cfg in "DLAMD_BALANCE_GRID=0" "DLAMD_BALANCE_GRID=1" "DLAMD_MAX_TILE_CHUNKS=16 DLAMD_BALANCE_GRID=0" "DLAMD_MAX_TILE_CHUNKS=16 DLAMD_BALANCE_GRID=1" "DLAMD_BALANCE_GRID=0" "DLAMD_BALANCE_GRID=1"; do
    i=$((i+1))
    echo "=== $i $cfg"
    env $cfg timeout -k 10 200 python bench.py --workload c3 --steps 300 --warmup 20 --no-cpu > $OUT/$i.log 2>&1 || exit $?
    tail -n 1 $OUT/$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), 'grad', round(d['phases']['gradients']['launch_ms']*1e3,1), 'round', round(d['phases']['round']['launch_ms']*1e3,1), d['config']['params_padded'])"
done
