#!/bin/bash
# PMC of the wave-per-key absent kernels on C4_deep_state (kernel trace + instruction mix + wait states), one
# counter group per rocprofv3 pass.  Output: gpurun_out/pmc_absd/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export SG_EXP_STEPS=${SG_EXP_STEPS:-3}
OUT=${PMC_OUT:-gpurun_out/pmc_absd}
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
    -- python3 tools/exp_gen.py C4_deep_state > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "k_absd_" --pmc $grp -d $OUT/g$i -o run \
      --output-format csv -- python3 tools/exp_gen.py C4_deep_state > $OUT/g$i.log 2>&1 \
      || { echo "pass $i failed: $grp"; tail -5 $OUT/g$i.log; exit 1; }
  echo "pass $i ok"
done
