#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench configuration.  Usage: gpu_prof.sh NAME bench-args...
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
NAME=$1; shift
mkdir -p "$R/gpurun_out/prof_$NAME"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$NAME" -o "$NAME" -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/prof_$NAME/stdout.log" 2>&1
rc=$?
tail -3 "$R/gpurun_out/prof_$NAME/stdout.log"
find "$R/gpurun_out/prof_$NAME" -name "*stats*" | head
exit $rc
