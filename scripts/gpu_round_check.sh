#!/bin/bash
# Round GPU check under driver-like conditions: fresh HOME (no MIOpen / kernel caches),
# the default bench (both halves) first, then the GPU test suite and smoke. Each step is time-limited
# and chained so the first failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-check}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
H=$(mktemp -d /tmp/fresh.XXXXXX)
export HOME=$H XDG_CACHE_HOME=$H/.cache
unset MIOPEN_USER_DB_PATH
# the shipped library must be the one built from these sources (no GPU touched by this check)
python -c "from cloudtik_amd.ops.build import stale_sources as s; r = s(); assert r == [], r" || exit 1
# the bench runs FIRST, as the first GPU process of a fresh box (the driver's condition)
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.log" 2> "$O/bench.err" \
 && tail -1 "$O/bench.log" | cut -c1-3000 \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.txt" 2>&1 \
 && tail -2 "$O/gpu_tests.txt" \
 && timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
 && tail -1 "$O/smoke.log"
rc=$?
[ $rc -eq 0 ] || { tail -40 "$O/gpu_tests.txt" 2>/dev/null | grep -E "FAIL|Error|passed|failed" | head; tail -20 "$O/bench.err" 2>/dev/null; }
exit $rc
