#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that passes or merely fails its tests (exit 0/1)
# lets the next one run, anything else (a fault, an abort, a time limit) ends the call.
# usage: tools/gsteps.sh LIMIT1 'cmd1' LIMIT2 'cmd2' ...
export TMPDIR=/tmp
mkdir -p gpurun_out
rc_all=0
while [ $# -ge 2 ]; do
    lim=$1; cmd=$2; shift 2
    timeout -k 10 "$lim" bash -c "$cmd"
    rc=$?
    echo "step rc=$rc: $cmd"
    if [ $rc -ne 0 ]; then rc_all=$rc; fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit $rc_all
