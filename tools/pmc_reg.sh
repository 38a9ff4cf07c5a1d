#!/bin/bash
# PMC counters and kernel traces of the register-window kernels (k_abs_* on C4, k_cnt_* on C3_min1), one
# counter group per rocprofv3 pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in passes of their own).
# Output: gpurun_out/pmc_reg/<cfg>_g*/run_counter_collection.csv, gpurun_out/pmc_reg/<cfg>_trace/run_kernel_stats.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export SG_EXP_STEPS=3
mkdir -p gpurun_out/pmc_reg
for cfg in ${PMC_CFGS:-C4 C3_min1}; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_reg/${cfg}_trace -o run --output-format csv \
      -- python3 tools/exp_gen.py $cfg > gpurun_out/pmc_reg/${cfg}_trace.log 2>&1 || { echo "trace $cfg failed"; tail -5 gpurun_out/pmc_reg/${cfg}_trace.log; exit 1; }
  echo "trace $cfg ok"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --kernel-include-regex "k_abs_|k_cnt_" --pmc $grp -d gpurun_out/pmc_reg/${cfg}_g$i -o run \
        --output-format csv -- python3 tools/exp_gen.py $cfg > gpurun_out/pmc_reg/${cfg}_g$i.log 2>&1 \
        || { echo "pass $cfg $i failed: $grp"; tail -5 gpurun_out/pmc_reg/${cfg}_g$i.log; exit 1; }
    echo "pass $cfg $i ok: $grp"
  done
done
