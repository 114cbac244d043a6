#!/usr/bin/env bash
# Capture the KFD topology sysfs tree (node properties + io_links) and the DRM
# card <-> KFD node mapping on a GPU box, for the exporter's sysfs-only mode.
# Names and numbers only; serials / unique ids are dropped.
#
#   gpurun -- 'bash tools/capture_kfd.sh'
set -u
OUT=gpurun_out/capture_kfd
mkdir -p "$OUT"
T=/sys/class/kfd/kfd/topology
{
  echo "# generation_id $(cat $T/generation_id 2>/dev/null)"
  for n in $T/nodes/*; do
    [ -d "$n" ] || continue
    echo "== node $(basename "$n")"
    echo "gpu_id $(cat "$n/gpu_id" 2>/dev/null)"
    echo "name $(cat "$n/name" 2>/dev/null)"
    grep -Ev '^(unique_id|serial)' "$n/properties" 2>/dev/null
    for l in "$n"/io_links/* "$n"/p2p_links/*; do
      [ -f "$l/properties" ] || continue
      echo "-- $(basename "$(dirname "$l")")/$(basename "$l")"
      cat "$l/properties"
    done
  done
} >"$OUT/kfd_topology.txt" 2>"$OUT/kfd_topology.err"
for c in /sys/class/drm/card*/device; do
  [ -e "$c/vendor" ] || continue
  echo "$c vendor=$(cat "$c/vendor") device=$(cat "$c/device") bdf=$(basename "$(readlink -f "$c")") render=$(ls "$(dirname "$c")"/../ 2>/dev/null | tr '\n' ' ')"
done >"$OUT/drm_cards.txt" 2>&1
ls -l /dev/kfd /dev/dri >"$OUT/dev_nodes.txt" 2>&1
id >>"$OUT/dev_nodes.txt" 2>&1
wc -l "$OUT"/*.txt
