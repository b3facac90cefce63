#!/bin/bash
# Round 6: the buffer-op streaming fix -- parity tests of every tile-kernel path, then same-box
# A/B against the round-4 build on c2, c4 and c3.  Any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r13/fix
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_mix_gpu.py tests/test_mix_ragged_gpu.py tests/test_pack_gpu.py tests/test_sharding_gpu.py tests/test_mixer_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
L="new=new r4=scripts/_build/libdlamd_r4.so"
bash scripts/ab_matrix.sh r13/fix/c2 3 "$L" --steps 50 --warmup 5 --no-cpu --no-fdla-probe || exit $?
bash scripts/ab_matrix.sh r13/fix/c4 2 "$L" --workload c4 --steps 20 --warmup 3 --no-cpu || exit $?
bash scripts/ab_matrix.sh r13/fix/c3 2 "$L" --workload c3 --steps 50 --warmup 5 --no-cpu || exit $?
echo done
