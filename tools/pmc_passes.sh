#!/bin/bash
# PMC counter passes over tools/kbench.py (one rocprofv3 run per counter set:
# SQ counters fit 8 per pass, FETCH_SIZE and WRITE_SIZE each need their own).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
ONLY="${ONLY:-conv1_fwd,conv2_fwd,conv1_wgrad,conv2_dgrad,conv2_wgrad}"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc -o pass$i -- python3 tools/kbench.py --reps 1 --only $ONLY $KB_ARGS > gpurun_out/pmc_pass$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
