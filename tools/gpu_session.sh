#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box.  Each step has its own time limit; the
# session stops at the first step that faults, aborts, segfaults or times out (exit status
# other than 0 or 1), so nothing else touches the GPU after trouble.  Exit status 1 (e.g.
# pytest failures) is recorded and the session continues.
#   usage: tools/gpu_session.sh "<secs>|<name>|<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
overall=0
for spec in "$@"; do
    secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
    echo "=== [$name] (limit ${secs}s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
    st=$?
    echo "=== [$name] exit $st after $(( $(date +%s) - start ))s"
    tail -n 15 "gpurun_out/${name}.log"
    if [ "$st" -ne 0 ] && [ "$st" -ne 1 ]; then
        echo "=== stopping: step $name exited $st"
        exit "$st"
    fi
    [ "$st" -ne 0 ] && overall=1
done
exit $overall
