#!/usr/bin/env bash
# Suspend every worker (reference nodes-suspend.sh); wake them with POST /nodes/wake_all.
set -Eeuo pipefail
source "$(dirname "$0")/_hosts.sh"
for h in "${HOSTS[@]}"; do
  valid_host "$h" || continue
  echo "$h"; ssh "thinvids@$h" "sudo -n systemctl suspend" || true
done
