#!/bin/bash
# c5 / c3 decode A/B: header-work cost (DIAGNOSTIC no-header flag), flat vs output-mapped, header blocks head vs spread
mkdir -p gpurun_out/c5ab
timeout -k 10 300 python tools/step_ab.py --k 32 --payload 256 --col 4 --cold --rounds 5 --reps 10 --variants default \
  --extra "dec nohdr=0:1048576;dec hdrhead=0:524288;dec out=0:2097152;dec out nohdr=0:3145728" \
  --out gpurun_out/c5ab/c5.json > gpurun_out/c5ab/c5.txt 2>&1; echo c5 rc=$?; cat gpurun_out/c5ab/c5.txt
timeout -k 10 300 python tools/step_ab.py --cold --rounds 5 --reps 10 --variants default \
  --extra "dec nohdr=0:1048576;dec flat=0:262144;dec hdrhead=0:524288" \
  --out gpurun_out/c5ab/c3.json > gpurun_out/c5ab/c3.txt 2>&1; echo c3 rc=$?; cat gpurun_out/c5ab/c3.txt
