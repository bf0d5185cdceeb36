#!/bin/bash
# Round profile set (GPU box): default bench line, rocprofv3 kernel-trace stats
# of the same command, and FETCH_SIZE / WRITE_SIZE passes (separate runs) for
# the dominant kernel.  Outputs under gpurun_out/; copy summaries to profiles/.
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
K="${KERNEL_REGEX:-Conv2Dgrad}"
BENCH_ARGS="${BENCH_ARGS:-}"
step() { echo "== $1"; shift; "$@"; rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step bench timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench_full.log 2>&1
grep '^{' gpurun_out/bench_full.log
step stats timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-gae-roofline --no-boundary $BENCH_ARGS
step fetch timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcb -o fetch -- python3 bench.py --no-cpu-baseline --no-gae-roofline --no-boundary $BENCH_ARGS
step write timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d gpurun_out/pmcb -o write -- python3 bench.py --no-cpu-baseline --no-gae-roofline --no-boundary $BENCH_ARGS
# MFMA utilisation of every kernel: pipeline-busy SIMD-cycles / (SIMDs x active cycles)
step mfma timeout -k 10 900 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcb -o mfma -- python3 bench.py --no-cpu-baseline --no-gae-roofline --no-boundary --steps 1 --warmup 1 $BENCH_ARGS
echo done
