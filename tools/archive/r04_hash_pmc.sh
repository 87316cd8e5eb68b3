#!/bin/bash
# Round 4: where the hash kernel's time goes -- SQ counter sets over the hash
# bench (offsets API and packed keys), one rocprofv3 pass per set.
# usage: tools/r04_hash_pmc.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/hash_pmc}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" && mkdir -p "$out"
bash tools/pmc_sets.sh "$out" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH" \
  -- --hash --blocks 4194304 > "$out/sets.txt" 2>&1 &&
echo "all steps done"
