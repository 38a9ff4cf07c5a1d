#!/bin/bash
# PMC counters of the C2 advance kernel, one counter group per rocprofv3 pass (MI355X_MICROARCH.md:
# FETCH_SIZE and WRITE_SIZE cannot share a pass; <= 8 SQ counters per pass).
# Output: gpurun_out/pmc/g*/.../*counter_collection.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true

i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_adv_m$" --pmc $grp -d gpurun_out/pmc/g$i -o run --output-format csv \
      -- python3 tools/prof_c2.py 3 > gpurun_out/pmc/g$i.log 2>&1 || { echo "pass $i failed: $grp"; tail -5 gpurun_out/pmc/g$i.log; continue; }
  echo "pass $i ok: $grp"
done
