#!/bin/bash
# PMC counters of the general kernel (k_gen_batch) on the C4 workload, one counter group per
# rocprofv3 pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in passes of their own).
# Output: gpurun_out/pmc_gen/g*/.../*counter_collection.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gen
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "k_gen_batch" --pmc $grp -d gpurun_out/pmc_gen/g$i -o run --output-format csv \
      -- python3 tools/exp_c4.py 1048576,1,4194304,16 > gpurun_out/pmc_gen/g$i.log 2>&1 || { echo "pass $i failed: $grp"; tail -5 gpurun_out/pmc_gen/g$i.log; exit 1; }
  echo "pass $i ok: $grp"
done
