# GPU box: the c4_strong decode gap -- the headline with 2 vs 16 buffer sets (16 sets ~ c4's working set), kernel
# times and UTCL1 translation counters per launch.  bash tools/g_tlb.sh <tag>
set -o pipefail
TAG=${1:-tlb}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --c4-steps 0 --sub-steps 0 --no-wire --no-cpu --steps 40 --warmup 5"
for S in 2 16; do
  timeout -k 10 300 $B --sets $S > $OUT/bench_sets$S.log 2>&1 || exit $?
  timeout -s KILL 200 python tools/pmc_sq.py --tag ${TAG}_sets$S --counters "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_ON_TRANSLATION_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" --match k_encode_out,k_decode_rows --timeout 190 -- $B --sets $S || exit $?
done
timeout -k 10 300 python bench.py --no-wire --no-cpu --sub-steps 0 --steps 20 > $OUT/bench_c4.log 2>&1
