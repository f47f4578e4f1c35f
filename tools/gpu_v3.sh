mkdir -p gpurun_out/v3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs --timeout 120 --timeout-method thread -k "dense or disjoint or erasure_fixture_rows" > gpurun_out/v3/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -4 gpurun_out/v3/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/v3/bench_dense.json 2> gpurun_out/v3/bench_dense.err; echo b1 rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --in-place > gpurun_out/v3/bench_inplace.json 2>/dev/null; echo b2 rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/v3/bench_dense2.json 2>/dev/null; echo b3 rc=$?
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu > gpurun_out/v3/bench_c5.json 2>/dev/null; echo b4 rc=$?
for f in bench_dense bench_inplace bench_dense2 bench_c5; do python -c "
import json,sys; d=json.load(open('gpurun_out/v3/$f.json')); print('$f', d['value'], d['roofline']['launch_us'], d['roofline']['frac'], d['decode_roofline']['launch_us'], d['decode_roofline']['frac'], d['verified'])"; done
