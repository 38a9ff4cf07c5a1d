#!/bin/bash
# PMC counters + kernel traces of the C2 workload variants' advance kernels (staged pass k_adv_m, HBM passes
# k_adv_m_h / k_adv_m_k, the hot-key pipeline k_hot_*), one counter group per rocprofv3 pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in passes of their own, <= 8 SQ counters per pass).
#   PMC_OUT=gpurun_out/pmc_var tools/pmc_variants.sh
# Summary: python tools/pmc_general_summary.py gpurun_out/pmc_var --variants [--json tools/pmc_traffic_variants.json]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_var}
RX='k_adv_m|k_hot_'
mkdir -p $OUT
for v in ${PMC_VARIANTS:-zipf walk}; do
  cfg=C2_$v
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/${cfg}_trace -o run --output-format csv \
      -- python3 tools/exp_variants.py 24 4 $v > $OUT/${cfg}_trace.log 2>&1 || { echo "trace $cfg failed"; tail -5 $OUT/${cfg}_trace.log; exit 1; }
  echo "trace $cfg ok"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --kernel-include-regex "$RX" --pmc $grp -d $OUT/${cfg}_g$i -o run \
        --output-format csv -- python3 tools/exp_variants.py 24 4 $v > $OUT/${cfg}_g$i.log 2>&1 \
        || { echo "pass $cfg $i failed: $grp"; tail -5 $OUT/${cfg}_g$i.log; exit 1; }
    echo "pass $cfg $i ok: $grp"
  done
done
