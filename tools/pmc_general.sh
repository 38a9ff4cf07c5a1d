#!/bin/bash
# PMC counters + kernel traces of the NFA kernels the general-engine configs actually run (register-window
# k_cnt_* / k_abs_* / k_absd_* / k_chn_*, the interpreter k_gen_batch / k_gen_timers), one counter group per rocprofv3
# pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in passes of their own, <= 8 SQ counters per pass).
#   PMC_CFGS="C3 C3_min1 C4 C4_deep C4_deep_state" PMC_OUT=gpurun_out/pmc_gen tools/pmc_general.sh
# Summary: python tools/pmc_general_summary.py gpurun_out/pmc_gen
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export SG_EXP_STEPS=${SG_EXP_STEPS:-3}
OUT=${PMC_OUT:-gpurun_out/pmc_gen}
RX='k_cnt_|k_abs|k_chn_|k_gen_batch|k_gen_timers'
mkdir -p $OUT
for cfg in ${PMC_CFGS:-C3 C3_min1 C3_and P3 C4 C4_deep C4_deep_state}; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/${cfg}_trace -o run --output-format csv \
      -- python3 tools/exp_gen.py $cfg > $OUT/${cfg}_trace.log 2>&1 || { echo "trace $cfg failed"; tail -5 $OUT/${cfg}_trace.log; exit 1; }
  echo "trace $cfg ok"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --kernel-include-regex "$RX" --pmc $grp -d $OUT/${cfg}_g$i -o run \
        --output-format csv -- python3 tools/exp_gen.py $cfg > $OUT/${cfg}_g$i.log 2>&1 \
        || { echo "pass $cfg $i failed: $grp"; tail -5 $OUT/${cfg}_g$i.log; exit 1; }
    echo "pass $cfg $i ok: $grp"
  done
done
