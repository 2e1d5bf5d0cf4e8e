#!/bin/bash
# HBM traffic per codegen variant: one FETCH_SIZE and one WRITE_SIZE rocprofv3 pass per variant
# (separate passes, MI355X_MICROARCH.md), plus the interleaved timing sweep of all variants.
# Usage: CONFIG=hdiff VARIANTS="jchunk=16;jchunk=32" bash scripts/variant_pmc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-hdiff}
OUT=gpurun_out/vpmc_${CONFIG}
mkdir -p $OUT
echo "== timing sweep"
timeout -k 10 300 python scripts/sweep.py --config $CONFIG --variants "$VARIANTS" > $OUT/sweep.log 2>&1 || exit $?
grep '^{' $OUT/sweep.log
i=0
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/v${i}_$c -o pmc -- \
      python3 scripts/sweep.py --config $CONFIG --variants "$v" --rounds 1 --reps 2 > $OUT/v${i}_$c.log 2>&1 || exit $?
  done
  echo "variant $i: $v"
  python3 - "$OUT" "$i" <<'EOF'
import csv, glob, sys
out, i = sys.argv[1], sys.argv[2]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{out}/v{i}_{c}/**/*counter_collection.csv", recursive=True)
    vals = []
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == c and ("_plane" in r["Kernel_Name"] or "_column" in r["Kernel_Name"]):
            vals.append(float(r["Counter_Value"]))
    res[c] = sum(vals) / len(vals) / 1024 if vals else float("nan")
print(f"  FETCH {res['FETCH_SIZE']:.1f} MiB (x2 = {2 * res['FETCH_SIZE']:.1f})  WRITE {res['WRITE_SIZE']:.1f} MiB  "
      f"total {2 * res['FETCH_SIZE'] + res['WRITE_SIZE']:.1f} MiB")
EOF
  i=$((i + 1))
done
