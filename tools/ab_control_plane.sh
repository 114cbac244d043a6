#!/usr/bin/env bash
# A/B of bench.py's fake control plane placement (thread of rank 0 vs child
# process), interleaved, on one GPU box. Results: gpurun_out/<tag>/cp_*.json.
#   gpurun --timeout 900 -- 'bash tools/ab_control_plane.sh cp'
set -u
TAG=${1:-cp}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2; do
  for cp in thread process; do
    timeout -k 10 240 python bench.py --steps 30 --warmup 5 --control-plane $cp --out "$OUT/cp_${cp}_$i.json" \
      >"$OUT/cp_${cp}_$i.log" 2>&1
    rc=$?
    echo "$cp $i rc=$rc $(tail -1 "$OUT/cp_${cp}_$i.log" | cut -c1-140)"
    [ $rc -eq 0 ] || exit $rc
  done
done
