#!/bin/bash
# wire lab breakdown + SQ instruction mix of the lab's base build
set -o pipefail
mkdir -p gpurun_out/wlab
timeout -k 10 300 bash tools/wire_lab.sh run || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 python tools/pmc_sq.py --tag lab_a --counters "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" --match k_frame_seg,k_parse -- tools/bin/wire_lab_base 3 || exit 1
timeout -s KILL 90 python tools/pmc_sq.py --tag lab_b --counters "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" --match k_frame_seg,k_parse -- tools/bin/wire_lab_base 3
echo pmc_b rc=$?
