#!/bin/bash
# conv weight-gradient split-K target sweep: the probe's wgrad column at several CLOUDTIK_AMD_WGRAD_BLOCKS
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/wgblocks"; mkdir -p "$O"; cd "$R"
for nb in ${BLOCKS:-256 512 1024}; do
  CLOUDTIK_AMD_WGRAD_BLOCKS=$nb WCFGS="${WCFGS:--1,3,11}" timeout -k 10 300 python -u bench/conv_igemm_probe.py --cfgs=-1 > "$O/probe_$nb.md" 2> "$O/probe_$nb.err" || exit $?
  echo "blocks $nb"; grep "cfg fwd" "$O/probe_$nb.err" | sed 's/.*| wgrad/wgrad/'
done
