# GPU box: receiver-session variants (async T8 unless RX_THREADS), one log per variant: bash tools/gcmd_rx_var.sh <tag> "<name>:<ENV=..>" ...
set -o pipefail
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp RFEC_RX_TRACE=1
LOCAL=$(bash tools/gpu_local_cpus.sh)
PIN=(); [ -n "$LOCAL" ] && PIN=(taskset -c "$LOCAL")
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  timeout -k 10 200 env $envs "${PIN[@]}" python3 tools/rx_session_bench.py --frames 32768 --reps 3 --threads ${RX_THREADS:-8} --modes async --out $OUT/rx_$name.json > $OUT/rx_$name.log 2>&1 || exit $?
done
