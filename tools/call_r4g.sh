export TMPDIR=/tmp; O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo pytest rc=$?; tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo smoke rc=$?; tail -4 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; echo bench rc=$?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['launch_us'],d['decode_roofline']['launch_us'],d['c4_strong']['value'])"
bash tools/abn.sh r4g/task 3 - tools/bin/ab/librazor_fec_task.so -- --config c3full
bash tools/abn.sh r4g/ppm 3 - tools/bin/ab/librazor_fec_ppm.so -- --c4-steps 0
timeout -k 10 400 bash tools/svc_ab.sh "plain prio_long plain_long" 3
timeout -k 10 300 python tools/e2e_step.py > $O/e2e.json; echo e2e rc=$?; cat $O/e2e.json
