# flat row encode: XCD-swizzled payload blocks (16384) vs plain order, rotated buffer sets
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/xab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "xcd or full_size" > gpurun_out/xab/pytest.log 2>&1 || { tail -20 gpurun_out/xab/pytest.log; exit 1; }
tail -1 gpurun_out/xab/pytest.log
for rep in 1 2 3; do
for t in 0 16384; do
  timeout -k 10 300 python bench.py --no-cpu --sets 2 --tuning $t --steps 60 > gpurun_out/xab/t$t.r$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/xab/t$t.r$rep.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tuning $t', d['value'], d['roofline']['launch_us_median'], d['decode_roofline']['launch_us_median'], d['verified'])"
done; done
timeout -k 10 600 python tools/pmc_traffic.py --out gpurun_out/xab/traffic.json -- --sets 2 --steps 20 --tuning 16384 > gpurun_out/xab/pmc.log 2>&1; echo pmc rc=$?
python -c "
import json; d=json.load(open('gpurun_out/xab/traffic.json')); e=list(d.values())[0]
print({k:(v['hbm_read_bytes_corrected'], v['hbm_write_bytes']) for k,v in e['kernels'].items()})"
