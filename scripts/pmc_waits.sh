#!/bin/bash
# Where the wave cycles go: per config one rocprofv3 pass each of
#   A  SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES
#   B  TCC_HIT_sum TCC_MISS_sum
#   C  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
# (separate passes; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md
# "rocprofv3 PMC slots"), then scripts/summarize_waits.py prints the split per config.
# Usage: CONFIGS="vadv copy" TAG=r05a [PASSES="A B C D E F"] [BENCH_OPTS="--opt ..." VARIANT=name] bash scripts/pmc_waits.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
OUT=gpurun_out/waits_${TAG}
mkdir -p $OUT
PASS_A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
PASS_B="TCC_HIT_sum TCC_MISS_sum"
PASS_C="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
# D: is an issue stall the memory pipe pushing back? (TA FIFOs full, VMEM instructions in flight)
PASS_D="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES"
# E/F: is an issue stall an instruction-fetch stall? (instruction cache hits/misses, fetches in flight)
PASS_E="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES"
PASS_F="SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"
for cfg in ${CONFIGS:-vadv copy}; do
  tag=$cfg${VARIANT:+_$VARIANT}
  for p in ${PASSES:-A B C}; do
    eval "ctrs=\$PASS_$p"
    echo "== $cfg pass $p: $ctrs"
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/${tag}_$p -o pmc -- \
      python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-extra --placement-candidates 0 ${BENCH_OPTS:-} \
      > $OUT/${tag}_$p.log 2>&1 || { tail -20 $OUT/${tag}_$p.log; exit 1; }
  done
done
python3 scripts/summarize_waits.py $OUT $(for c in ${CONFIGS:-vadv copy}; do echo $c${VARIANT:+_$VARIANT}; done) | tee $OUT/summary${VARIANT:+_$VARIANT}.json
