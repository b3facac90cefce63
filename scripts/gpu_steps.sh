#!/bin/bash
# Run GPU steps from the command line, one per argument ("name|timeout|command"), each under its
# own time limit.  A test failure (rc 1) lets the next step run; any other non-zero status (a
# fault, abort, time limit) ends the script so nothing else touches the GPU after trouble.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
    echo "=== $name ($t s): $cmd"
    timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
echo "=== done"
