#!/bin/bash
# XCD-swizzled output-mapped encode / row decode (A/B): parity tests, timing, HBM traffic
set -u
OUT=gpurun_out/xcd; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "xcd or dense or disjoint" > $OUT/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/step_ab.py --cold --rounds 6 --reps 10 --variants default --extra "xcd=16384:16384;dec xcd=0:16384;xcd2=16384:16384" --out $OUT/c3.json > $OUT/c3.txt 2>&1; echo ab rc=$?; cat $OUT/c3.txt
timeout -k 10 600 python tools/pmc_traffic.py --out $OUT/traffic_xcd.json -- --tuning 16384 --steps 10 --warmup 2 --no-cpu > $OUT/pmc.log 2>&1; echo pmc rc=$?
python -c "
import json; d=json.load(open('$OUT/traffic_xcd.json'))
for k,v in d.items(): print(k, {kk:vv for kk,vv in v.items() if 'over' in kk})"
