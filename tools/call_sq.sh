# SQ / TCC counter passes of the c3 and c3full decodes (GPU box)
export TMPDIR=/tmp
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
C2="TCC_HIT_sum TCC_MISS_sum"
for cfg in c3 c3full; do
  timeout -k 10 150 python tools/pmc_sq.py --tag ${cfg}_sq --counters "$C1" --match k_decode,k_encode -- python bench.py --config $cfg --no-cpu --steps 10 --warmup 2 --c4-steps 0 || exit 1
  timeout -k 10 150 python tools/pmc_sq.py --tag ${cfg}_tcc --counters "$C2" --match k_decode,k_encode -- python bench.py --config $cfg --no-cpu --steps 10 --warmup 2 --c4-steps 0 || exit 1
done
for f in gpurun_out/pmc_sq/*/..; do :; done
ls gpurun_out/pmc_sq/
cat gpurun_out/pmc_sq/*.json
