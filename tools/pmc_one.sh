#!/bin/bash
# PMC counters for one kbench kernel under two libraries (A/B): usage
#   ONLY=fc_fwd LIBS="lib/libppo_hip.so" TUNES="x9=1 x9=0" bash tools/pmc_one.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc1
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"
      "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY TA_BUSY_avr TD_BUSY_avr")
i=0
for t in ${TUNES}; do
  for s in "${SETS[@]:${SET0:-0}:${NSET:-3}}"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $s --output-format csv -d gpurun_out/pmc1 -o p$i -- python3 tools/kbench.py --reps 2 --only $ONLY --tune $t > gpurun_out/pmc1/log$i.txt 2>&1
    rc=$?; echo "set $i ($t): rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc1/log$i.txt; exit $rc; }
  done
done
echo done
