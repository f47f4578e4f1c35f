#!/bin/bash
# small-slot decode: parity tests, then the c5 A/B (header work in the payload lanes vs header blocks)
mkdir -p gpurun_out/v4
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs --timeout 120 --timeout-method thread -k "dense or disjoint or erasure_fixture_rows or long_sched"  tests/test_receiver.py > gpurun_out/v4/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -4 gpurun_out/v4/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/step_ab.py --k 32 --payload 256 --col 4 --cold --rounds 6 --reps 10 --variants default \
  --extra "dec split_hdr=0:4194304;dec small_b2=0:8388608;dec nohdr=0:1048576" --out gpurun_out/v4/c5.json > gpurun_out/v4/c5.txt 2>&1; echo c5 rc=$?; cat gpurun_out/v4/c5.txt
