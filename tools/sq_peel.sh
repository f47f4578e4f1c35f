# SQ counters (two passes) of the full-plan decode kernels: peel, replay, encode
set -o pipefail
export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
timeout -s KILL 100 python tools/pmc_sq.py --tag peelA --counters "$A" --match k_peel_lds,k_recover_flat,k_encode_k16 -- python bench.py --no-cpu --full-plan --steps 3 --warmup 1 > /dev/null 2>&1 && \
timeout -s KILL 100 python tools/pmc_sq.py --tag peelB --counters "$B" --match k_peel_lds,k_recover_flat,k_encode_k16 -- python bench.py --no-cpu --full-plan --steps 3 --warmup 1 > /dev/null 2>&1
echo rc=$?
