#!/bin/bash
# SQ counters of the C2 advance kernel for JIT variants: tools/pmc_cmp.sh NAME=SG_JIT_EXTRA ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcc
for v in "$@"; do
  name=${v%%=*}; extra=${v#*=}
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
             "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_FLAT SQ_INST_LEVEL_LDS SQ_INSTS_FLAT"; do
    i=$((i+1))
    SG_JIT_EXTRA=$extra timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_adv_m$" --pmc $grp -d gpurun_out/pmcc/$name/g$i -o run --output-format csv \
        -- python3 tools/prof_c2.py 3 > gpurun_out/pmcc/$name.g$i.log 2>&1 || { echo "pass $name $i failed"; tail -5 gpurun_out/pmcc/$name.g$i.log; exit 1; }
  done
  echo "variant $name done"
done
