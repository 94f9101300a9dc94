#!/bin/bash
# PMC passes over a short bench run (counters collected in separate passes, --kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_WAIT_INST_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F32" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "=== pass $i: $set"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 3 gpurun_out/pmc/p$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    if grep -q "not supported\|invalid\|Invalid" gpurun_out/pmc/p$i.log; then continue; fi
    exit $rc
  fi
done
