# GPU box: kernel trace of the receiver session (async, 16 shards)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RFEC_RX_SPIN_US=0 RFEC_RX_ARENA_ROWS=1048576 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/rxprof -o rx -- python3 tools/rx_session_bench.py --frames 32768 --threads 16 --modes async --reps 1 > gpurun_out/rxprof.log 2>&1
