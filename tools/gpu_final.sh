#!/bin/bash
# end-of-round pass: the standard measurement script, then the SQ mix of the wire lab's base build
set -o pipefail
bash tools/measure.sh m5 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 python tools/pmc_sq.py --tag lab_parse_a --counters "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" --match k_frame_seg,k_parse -- tools/bin/wire_lab_base 3 > /dev/null || exit 1
timeout -s KILL 90 python tools/pmc_sq.py --tag lab_parse_b --counters "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" --match k_frame_seg,k_parse -- tools/bin/wire_lab_base 3 > /dev/null
echo pmc rc=$?
