#!/bin/bash
# SQ stall anatomy of kbench kernels (3 passes of <= 8 SQ counters each): usage
#   ONLY=conv2_dgrad_bits,conv2_fwd_mask TUNE="stagger=0" bash tools/pmc_sq.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
rm -rf gpurun_out/pmc1; mkdir -p gpurun_out/pmc1
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH")
i=0
for s in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $s --output-format csv -d gpurun_out/pmc1 -o p$i -- python3 tools/kbench.py --reps 2 --only $ONLY --tune "${TUNE:-stagger=0}" ${KBARGS:-} > gpurun_out/pmc1/log$i.txt 2>&1
  rc=$?; echo "set $i: rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc1/log$i.txt; exit $rc; }
done
for k in ${ONLY//,/ }; do echo "== $k"; done
echo done
