# encode -> decode step timing at the packed 1200-B slot stride vs a line-aligned 1280-B stride
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/st
timeout -k 10 300 python tools/ab_encode.py --step-only --rounds 5 --out gpurun_out/st/s1200.json > gpurun_out/st/s1200.log 2>&1 && \
timeout -k 10 300 python tools/ab_encode.py --step-only --rounds 5 --stride 1280 --out gpurun_out/st/s1280.json > gpurun_out/st/s1280.log 2>&1 && \
timeout -k 10 300 python tools/ab_encode.py --step-only --rounds 5 --stride 1216 --out gpurun_out/st/s1216.json > gpurun_out/st/s1216.log 2>&1
echo rc=$?
