# bench.py at slot stride 1200 vs 1216, alternating (same box, same process image)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sb
for i in 1 2 3; do
  for s in 1200 1216; do
    timeout -k 10 200 python bench.py --no-cpu --stride $s > gpurun_out/sb/b_${s}_$i.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sb/b_${s}_$i.log') if l.startswith('{')][-1]); print($s, d['value'], d['encode_gibps'], d['decode_gibps'], d['roofline']['launch_us'], d['decode_roofline']['launch_us'])"
  done
done
