#!/usr/bin/env bash
# udev-triggered launcher: one rip per drive (flock), settle delay, disc type + label from
# udev, then the rip/queue tool (reference rips/auto_dvd/thinvids-dvd-auto.sh).
set -Eeuo pipefail
dev="${1:?device name, e.g. sr0}"
exec 9>"/run/lock/thinvids-dvd-${dev}.lock"
flock -n 9 || { echo "rip already running on ${dev}"; exit 0; }
sleep "${THINVIDS_DVD_SETTLE_SEC:-8}"
props=$(udevadm info --query=property --name="/dev/${dev}" || true)
grep -q '^ID_CDROM_MEDIA_DVD=1' <<<"$props" || grep -q '^ID_CDROM_MEDIA_BD=1' <<<"$props" || { echo "no DVD/BD media"; exit 0; }
label=$(sed -n 's/^ID_FS_LABEL=//p' <<<"$props" | head -n1)
exec /opt/thinvids/venv/bin/python -m thinvids_amd.rips --source "dev:/dev/${dev}" --disc-label "${label}"
