# Round 5: run a list of recipes in one call, with a heartbeat (a long CPU-oracle phase prints nothing for minutes)
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do echo "heartbeat $(date +%T)" >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap "kill $HB" EXIT
for s in "$@"; do
  bash "$s" || { echo "RECIPE $s FAILED"; exit 1; }
done
