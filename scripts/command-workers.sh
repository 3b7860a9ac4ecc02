#!/usr/bin/env bash
# Remove stale UUID scratch dirs on every worker and show disk usage (reference command-workers.sh).
set -Eeuo pipefail
source "$(dirname "$0")/_hosts.sh"
SCRATCH=${SCRATCH:-/projects}
for h in "${HOSTS[@]}"; do
  valid_host "$h" || { echo "skip $h" >&2; continue; }
  echo "== $h: clean $SCRATCH"
  ssh "thinvids@$h" "find $SCRATCH -mindepth 1 -maxdepth 1 -type d -regextype posix-extended -regex '.*/[0-9A-Fa-f]{8}(-[0-9A-Fa-f]{4}){3}-[0-9A-Fa-f]{12}$' -exec rm -rf {} + ; df -h $SCRATCH"
done
