# sender bench (pinned vs pageable outputs) and bench.py through the driver's torchrun launcher at N=1
set -o pipefail
export TMPDIR=/tmp
T=${1:-mc}
mkdir -p gpurun_out/$T
timeout -k 10 300 python tools/send_bench.py --out gpurun_out/$T/send_pinned.json > gpurun_out/$T/send_pinned.log 2>&1; echo "send pinned rc=$?"
timeout -k 10 300 python tools/send_bench.py --pageable --out gpurun_out/$T/send_pageable.json > gpurun_out/$T/send_pageable.log 2>&1; echo "send pageable rc=$?"
grep -E "d2h_us|wall_s|datagrams_per_s|verified" gpurun_out/$T/send_pinned.json gpurun_out/$T/send_pageable.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu > gpurun_out/$T/torchrun1.log 2>&1; echo "torchrun rc=$?"
tail -2 gpurun_out/$T/torchrun1.log | cut -c1-400
