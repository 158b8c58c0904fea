#!/bin/bash
# PMC pass set on single ops (tools/profile_op.py): wave-state breakdown, MFMA busy, and
# GRBM_GUI_ACTIVE for the effective clock. One rocprofv3 --pmc run per counter group.
#   tools/pmc_pair.sh <outdir> <kind> <dims> [<kind> <dims> ...]
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
while [ $# -gt 1 ]; do
  kind=$1; dims=$2; shift 2
  i=$((i+1)); d="$out/op$i"; mkdir -p "$d"; echo "$kind $dims" > "$d/op.txt"
  g=0
  for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD"; do
    g=$((g+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$d/g$g" -o pmc -- \
      python3 tools/profile_op.py $kind $dims --iters 10 > "$d/g$g.log" 2>&1 || { echo "pass $g of $kind $dims failed"; tail -3 "$d/g$g.log"; exit 3; }
  done
done
