#!/usr/bin/env bash
# Scaling sweep on the GPU box: BASELINE configs + --beyond points, with
# bench progress streamed into gpurun_out/<tag>/progress.log.
#   gpurun --timeout 1200 -- 'bash tools/gpu_sweep.sh r3c 16,64,256,1000,h256'
set -u
TAG=${1:-sweep}
BEYOND=${2:-16,64,256,1000,h256}
EXTRA=${3:-}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 1100 python -u tools/sweep.py --steps 20 --warmup 3 --beyond "$BEYOND" $EXTRA --out "$OUT" \
  >"$OUT/sweep.log" 2>"$OUT/progress.log"
rc=$?
echo "sweep rc=$rc"
tail -40 "$OUT/sweep.log"
exit $rc
