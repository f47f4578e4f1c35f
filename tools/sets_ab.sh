# bench with 1 / 2 / 3 rotated buffer sets, alternating; then PMC traffic at 2 sets
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sets
for rep in 1 2; do
for n in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu --sets $n --steps 60 > gpurun_out/sets/n$n.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/sets/n$n.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('sets $n', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
timeout -k 10 600 python tools/pmc_traffic.py --out gpurun_out/sets/traffic2.json -- --sets 2 --steps 20 > gpurun_out/sets/pmc.log 2>&1; echo pmc rc=$?
python -c "
import json; d=json.load(open('gpurun_out/sets/traffic2.json')); e=list(d.values())[0]
print({k:(v['hbm_read_bytes_corrected'], v['hbm_write_bytes']) for k,v in e['kernels'].items()})"
