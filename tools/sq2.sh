# wire tests + instruction-mix counters of the wire kernels
set -o pipefail
export TMPDIR=/tmp
T=${1:-sq2}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_receiver.py tests/test_udp.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/$T/pytest.log
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
timeout -s KILL 100 python tools/pmc_sq.py --tag ${T}A --counters "$A" --match k_frame_seg,k_frame_fec,k_parse -- python tools/wire_bench.py --reps 3 > gpurun_out/$T/A.log 2>&1 && \
timeout -s KILL 100 python tools/pmc_sq.py --tag ${T}B --counters "$B" --match k_frame_seg,k_frame_fec,k_parse -- python tools/wire_bench.py --reps 3 > gpurun_out/$T/B.log 2>&1
echo "pmc rc=$?"
