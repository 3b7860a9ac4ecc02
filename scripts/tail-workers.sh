#!/usr/bin/env bash
# Follow the journals of every worker's thinvids units with host prefixes (reference tail-workers.sh).
set -Eeuo pipefail
source "$(dirname "$0")/_hosts.sh"
UNITS=${UNITS:-"thinvids-worker-encode@* thinvids-worker-pipeline thinvids-agent"}
FOLLOW=${FOLLOW:--f}
args=(); for u in $UNITS; do args+=(-u "$u"); done
pids=()
for h in "${HOSTS[@]}"; do
  valid_host "$h" || continue
  ssh "thinvids@$h" "journalctl ${args[*]} -n 50 $FOLLOW -o short-iso" | sed -u "s/^/[$h] /" &
  pids+=($!)
done
trap 'kill "${pids[@]}" 2>/dev/null' INT TERM EXIT
wait
