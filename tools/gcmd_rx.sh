# GPU box: the receiver session (async, c3 stream, eviction per batch): thread sweep and variants, then a kernel +
# memory-copy trace of the T8 run.  bash tools/gcmd_rx.sh <tag>
set -o pipefail
TAG=${1:-rx}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
LOCAL=$(bash tools/gpu_local_cpus.sh)
PIN=(); [ -n "$LOCAL" ] && PIN=(taskset -c "$LOCAL")
run() { local name=$1 envs=$2; shift 2; timeout -k 10 300 env $envs "${PIN[@]}" python3 tools/rx_session_bench.py --frames 32768 --reps 3 "$@" --out $OUT/$name.json > $OUT/$name.log 2>&1; }
run rx_session RX=1 --threads ${RX_THREADS:-1,4,8} --modes async,sync &&
run rx_caller0 RFEC_RX_CALLER=0 --threads 4,8 --modes async &&
run rx_spin400 RFEC_RX_SPIN_US=400 --threads 4,8 --modes async &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/rxprof -o rx -- python3 tools/rx_session_bench.py --frames 32768 --threads 8 --modes async --reps 1 > $OUT/rxprof.log 2>&1
