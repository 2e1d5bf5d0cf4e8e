#!/bin/bash
# Round 5: cache policy of the LDS-tail fields (tail_nt). tridiag and vadv timed interleaved per
# variant, then FETCH_SIZE / WRITE_SIZE of tridiag per variant (separate passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05q}
mkdir -p $O
timeout -k 10 300 python3 scripts/sweep.py --config tridiag --rounds 9 --variants "tail_nt=0;tail_nt=1;tail_nt=2;tail_nt=3" \
  > $O/sweep_tridiag.log 2>&1 || { tail -20 $O/sweep_tridiag.log; exit 1; }
grep -v Warn $O/sweep_tridiag.log
timeout -k 10 300 python3 scripts/sweep.py --config vadv --rounds 9 --variants "tail_nt=0;tail_nt=2" \
  > $O/sweep_vadv.log 2>&1 || { tail -20 $O/sweep_vadv.log; exit 1; }
grep -v Warn $O/sweep_vadv.log
for v in 0 1 3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_tridiag_nt${v}_$c -o pmc -- \
      python3 bench.py --config tridiag --steps 3 --warmup 1 --no-cpu-baseline --no-extra --placement-candidates 0 --opt tail_nt=$v \
      > $O/pmc_tridiag_nt${v}_$c.log 2>&1 || { tail -20 $O/pmc_tridiag_nt${v}_$c.log; exit 1; }
  done
done
O=$O python3 - <<'EOF'
import csv, glob, os
O = os.environ.get("O", "gpurun_out/r05q")
for v in (0, 1, 3):
    r = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = [float(x["Counter_Value"]) for f in glob.glob(f"{O}/pmc_tridiag_nt{v}_{c}/**/*counter_collection.csv", recursive=True)
                for x in csv.DictReader(open(f)) if "_column" in x["Kernel_Name"] and x["Counter_Name"] == c]
        r[c] = sum(vals) / len(vals) if vals else float("nan")
    print(f"tail_nt={v}: FETCH {r['FETCH_SIZE'] / 1024:.1f} MiB  WRITE {r['WRITE_SIZE'] / 1024:.1f} MiB  "
          f"hbm {(2 * r['FETCH_SIZE'] + r['WRITE_SIZE']) * 1024 / 1e9:.3f} GB")
EOF
