#!/bin/bash
set -u
export TMPDIR=/tmp
timeout -k 10 150 python tools/pmc_sq.py --tag wire_fetch --counters "FETCH_SIZE" --match k_frame,k_parse -- python tools/wire_bench.py --reps 3 || exit 1
timeout -k 10 150 python tools/pmc_sq.py --tag wire_write --counters "WRITE_SIZE" --match k_frame,k_parse -- python tools/wire_bench.py --reps 3 || exit 1
timeout -k 10 150 python tools/pmc_sq.py --tag wire_sq --counters "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" --match k_frame,k_parse -- python tools/wire_bench.py --reps 3 || exit 1
cat gpurun_out/pmc_sq/wire_fetch.json gpurun_out/pmc_sq/wire_write.json gpurun_out/pmc_sq/wire_sq.json
