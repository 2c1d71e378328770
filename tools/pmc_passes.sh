#!/bin/bash
# Separate rocprofv3 --pmc passes (one run per counter set, per
# MI355X_MICROARCH.md "rocprofv3 PMC slots": <= 8 SQ, <= 4 TCC, <= 2 GRBM)
# over one command; CSVs land in OUTDIR/<set>/.
#   tools/pmc_passes.sh OUTDIR "SETS" -- python3 tools/eval_variants.py ...
# SETS: any of occ mfma valu lds write fetch ea, and trace (a --kernel-trace
# --stats run: kernel durations without counter collection)
set -e
out=$1; sets=$2; shift 3
export TMPDIR=/tmp
declare -A C
C[occ]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
C[mfma]="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
C[valu]="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"
C[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_WR SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
C[write]="WRITE_SIZE"
C[fetch]="FETCH_SIZE"
# round 6: the L2's memory-side write requests, their stalls (all DRAM
# credit stalls on gfx950) and the queue level per cycle
C[ea]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE"
# the identity of the library these counters are taken on (bench.py reports
# a table entry only when it matches the library it loaded)
mkdir -p "$out"
python3 -c "import sys, json; sys.path.insert(0, 'ska-sdp-screen-fitting_amd'); \
from ska_sdp_screen_fitting_amd._lib import library_identity; \
print(json.dumps(library_identity()))" > "$out/library.json"
for s in $sets; do
  mkdir -p "$out/$s"
  if [ "$s" = trace ]; then
    timeout -s KILL 150 rocprofv3 --kernel-trace --stats -f csv -d "$out/$s" -o t -- "$@" \
      > "$out/$s/run.log" 2>&1
  else
    timeout -s KILL 150 rocprofv3 --pmc ${C[$s]} -f csv -d "$out/$s" -o p -- "$@" \
      > "$out/$s/run.log" 2>&1
  fi
  echo "pass $s done"
done
