#!/bin/bash
# Reproduce the driver's fresh-box conditions for the ResNet-50 half of bench.py:
# fresh HOME / XDG_CACHE_HOME (no MIOpen kernel cache, no user db), MIOPEN_USER_DB_PATH unset.
#   A: shipped find-db installed by cloudtik_amd.ops (default)
#   B: no find-db (CLOUDTIK_AMD_MIOPEN_DB=0): MIOpen immediate-mode fallback
#   C: kernel trace of B (which conv kernels run)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/diag"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
unset MIOPEN_USER_DB_PATH MIOPEN_CUSTOM_CACHE_DIR
{
  echo "whoami=$(whoami) HOME=$HOME XDG_CACHE_HOME=${XDG_CACHE_HOME:-} TMPDIR=$TMPDIR"
  env | grep -E '^(MIOPEN|HIP|ROCR|HSA|PYTORCH|TORCH|NCCL|XDG)' | sort
  ls -ld "$HOME" "$HOME/.cache" 2>&1
  [ -w "$HOME" ] && echo "HOME writable" || echo "HOME NOT writable"
  ls -la "$HOME/.cache" 2>&1 | head
  ls -la "$HOME/.cache/miopen" 2>&1 | head
  ls -la "$HOME/.config/miopen" 2>&1 | head
} > "$O/env.txt" 2>&1
fresh() { local d; d=$(mktemp -d /tmp/fresh.XXXXXX); echo "$d"; }
H1=$(fresh)
HOME=$H1 XDG_CACHE_HOME=$H1/.cache timeout -k 10 300 python3 -u "$R/bench.py" --model resnet50 --steps 10 --warmup 3 \
  > "$O/A_db.log" 2>&1
rc=$?; echo "A rc=$rc"; tail -c 600 "$O/A_db.log"; [ $rc -eq 0 ] || exit $rc
find "$H1" -maxdepth 4 | head -30 > "$O/A_home_tree.txt"
H2=$(fresh)
HOME=$H2 XDG_CACHE_HOME=$H2/.cache CLOUDTIK_AMD_MIOPEN_DB=0 timeout -k 10 300 python3 -u "$R/bench.py" --model resnet50 \
  --steps 10 --warmup 3 > "$O/B_nodb.log" 2>&1
rc=$?; echo "B rc=$rc"; tail -c 600 "$O/B_nodb.log"; [ $rc -eq 0 ] || exit $rc
H3=$(fresh)
export HOME=$H3 XDG_CACHE_HOME=$H3/.cache CLOUDTIK_AMD_MIOPEN_DB=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_nodb" -o nodb -- \
  python3 "$R/bench.py" --model resnet50 --steps 3 --warmup 1 > "$O/C_prof.log" 2>&1
rc=$?; echo "C rc=$rc"; tail -c 300 "$O/C_prof.log"
exit $rc
