# UDP tests, then the list of available rocprofv3 counters on the box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sq1
timeout -k 10 300 python -u -m pytest tests/test_udp.py -q -rs --timeout 120 --timeout-method thread > gpurun_out/sq1/pytest_udp.log 2>&1; echo "udp rc=$?"; tail -3 gpurun_out/sq1/pytest_udp.log
timeout -s KILL 60 rocprofv3 -L > gpurun_out/sq1/avail.txt 2>&1; echo "list rc=$?"
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
timeout -s KILL 100 python tools/pmc_sq.py --tag wireA --counters "$A" --match k_frame_seg,k_frame_fec,k_parse -- python tools/wire_bench.py --reps 3 > gpurun_out/sq1/wireA.log 2>&1 && \
timeout -s KILL 100 python tools/pmc_sq.py --tag wireB --counters "$B" --match k_frame_seg,k_frame_fec,k_parse -- python tools/wire_bench.py --reps 3 > gpurun_out/sq1/wireB.log 2>&1 && \
timeout -s KILL 100 python tools/pmc_sq.py --tag benchA --counters "$A" --match k_encode_rows,k_decode_disjoint -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/sq1/benchA.log 2>&1 && \
timeout -s KILL 100 python tools/pmc_sq.py --tag benchB --counters "$B" --match k_encode_rows,k_decode_disjoint -- python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/sq1/benchB.log 2>&1
echo "pmc rc=$?"
tail -5 gpurun_out/sq1/*.log
