#!/usr/bin/env bash
# List the amdgpu RAS / ECC sysfs files of GPU card devices and their contents (read-only).
set -u
for c in /sys/class/drm/card*/device; do
  [ -e "$c/vendor" ] || continue
  [ "$(cat "$c/vendor" 2>/dev/null)" = "0x1002" ] || continue
  echo "== $c"
  ls "$c" | grep -i -E "ras|ecc|err|reset|throttle|gpu_metrics|unique_id|serial|product|thermal" || true
  if [ -d "$c/ras" ]; then
    for f in "$c"/ras/*; do echo "-- $f"; head -c 400 "$f" 2>/dev/null; echo; done
  fi
  break
done
