# GPU box: PMC passes over the wire kernels (tools/wire_bench.py --reps 3), one rocprofv3 --pmc pass per
# counter set, each under its own kill-timeout; per (kernel, grid) means -> gpurun_out/pmc_sq/<tag>_*.json
set -o pipefail
TAG=${1:-wire6}
export TMPDIR=/tmp
P() { local name=$1; shift; timeout -s KILL 150 python tools/pmc_sq.py --by-grid --tag ${TAG}_$name --counters "$*" --match k_frame_seg_q,k_frame_fec_q,k_parse_q --timeout 140 -- python tools/wire_bench.py --reps 3; }
P sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES &&
P sq2 SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES &&
P fetch FETCH_SIZE &&
P write WRITE_SIZE
