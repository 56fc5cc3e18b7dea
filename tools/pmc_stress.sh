#!/bin/bash
# usage: tools/pmc_stress.sh <tag>
# PMC passes over the configs[3] stress aggregation (tools/staged_probe.py,
# blocked numbering, C = 128): HBM-side bytes (FETCH_SIZE, WRITE_SIZE), the
# L1 -> L2 read requests (the gather), and the SQ wait / LDS profile of the
# register gather (k_gat_fwd_cp / _ep) and the staged kernel
# (k_gat_fwd_staged) and the ring kernel (k_gat_fwd_ring).  One rocprofv3 run
# per pass (tools/pmc_kernel.sh).
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
CMD="python3 $R/tools/staged_probe.py --orders blocked --channels 128 --reps 3"
RE='k_gat_fwd'
bash $R/tools/pmc_kernel.sh ${TAG}_fetch "$RE" "FETCH_SIZE" $CMD || exit $?
bash $R/tools/pmc_kernel.sh ${TAG}_write "$RE" "WRITE_SIZE" $CMD || exit $?
bash $R/tools/pmc_kernel.sh ${TAG}_sq "$RE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" $CMD || exit $?
bash $R/tools/pmc_kernel.sh ${TAG}_tcp "$RE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" $CMD
