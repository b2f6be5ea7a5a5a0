#!/bin/bash
# Attention GPU tests + kernel probe (BERT-large phase-1 and S 512 shapes) + the LDS counter pass.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/attn_quick"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_model_parity.py -k "attention or attn or bert" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do
for v in ${AB_VALUES:-1}; do
for shape in "--S 128 --B 256 --p 0.1" "--S 128 --B 256 --p 0.0" "--S 512 --B 32 --p 0.1"; do
  env ${AB_VAR:-AB_NONE}=$v timeout -k 10 120 python3 bench/attn_kernel_probe.py $shape 2>&1 | grep -v amdgpu.ids | sed "s/^/${AB_VAR:-}=$v /" || exit 1
done
done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex attn_ --output-format csv -d "$OUT/p" -o p -- python3 "$R/bench/attn_kernel_probe.py" > "$OUT/p.log" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/p.log"; exit 1; }
f=$(find "$OUT/p" -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in d.items()))
PY
rm -rf "$OUT/p"
