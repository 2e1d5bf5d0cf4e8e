#!/bin/bash
# Round 5: fast vs slow placements of tridiag's fields in one process, counter by counter
# (scripts/column_placement_probe.py; every pass prints its own per-set times, since each process
# gets its own placements).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05x}
mkdir -p $O
S=${SETS:-8}; R=${REPS:-6}; C=${CFG:-tridiag}
timeout -k 10 180 python3 scripts/column_placement_probe.py --config $C --sets $S --reps $R > $O/plain.json 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/plain.json')); print('plain', [s['ms'] for s in d['sets']])"
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum"
P2="TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
P4="SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
P5="GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
P6="TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_PENDING_STALL_CYCLES_sum"
P7="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_LEVEL_sum"
for p in ${PASSES:-1 2 3 4}; do
  eval "ctrs=\$P$p"
  timeout -s KILL 180 rocprofv3 --pmc $ctrs --output-format csv -d $O/p$p -o pmc -- \
    python3 scripts/column_placement_probe.py --config $C --sets $S --reps $R > $O/p$p.json 2> $O/p$p.err || { tail -20 $O/p$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/p$p.json')); print('p$p', [s['ms'] for s in d['sets']])"
  python3 scripts/column_placement_probe.py --summarize $O/p$p --sets $S --reps $R > $O/p${p}_summary.json || exit 1
  cat $O/p${p}_summary.json
done
