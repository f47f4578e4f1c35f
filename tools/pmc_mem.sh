# GPU box: memory-path counters (TCC EA request sizes, TA stalls) of the wire kernels beside the headline encode
# (a kernel at its mix ceiling), one --pmc pass per set.  bash tools/pmc_mem.sh TAG
set -o pipefail
TAG=${1:-mem}
export TMPDIR=/tmp
W() { timeout -s KILL 150 python tools/pmc_sq.py --by-grid --tag ${TAG}_w_$1 --counters "$2" --match k_frame_seg_q,k_frame_fec_q,k_parse_q --timeout 140 -- python tools/wire_bench.py --reps 3; }
E() { timeout -s KILL 200 python tools/pmc_sq.py --tag ${TAG}_e_$1 --counters "$2" --match k_encode_out,k_decode_rows --timeout 190 -- python bench.py --c4-steps 0 --sub-steps 0 --no-wire --no-cpu --steps 10 --warmup 2; }
for s in "ea:TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
         "rd:TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_HIT_sum TCC_MISS_sum" \
         "ta:TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
         "tab:TA_BUFFER_COALESCED_READ_CYCLES_sum TA_BUFFER_COALESCED_WRITE_CYCLES_sum" \
         "busy:TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum"; do
  n=${s%%:*}; c=${s#*:}
  W $n "$c" || exit $?
  E $n "$c" || exit $?
done
