#!/bin/bash
# rocprofv3 kernel stats of bench/conv_igemm_one.py for a list of shapes "ci,co,H,k,s"
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for sh in "$@"; do
  IFS=, read ci co H k s <<< "$sh"
  d="$R/gpurun_out/conv_one/$ci-$co-$H-$k-$s"
  mkdir -p "$d"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o p -- \
    python3 "$R/bench/conv_igemm_one.py" $ci $co $H $k $s > "$d/log.txt" 2>&1 || { echo "FAIL $sh"; tail -5 "$d/log.txt"; exit 1; }
  echo "== $sh"; f=$(find "$d" -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -8
done
