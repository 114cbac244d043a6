#!/usr/bin/env bash
# One GPU-box pass: GPU tests, smoke(), 1-GPU bench, rocprofv3 kernel stats of
# the bench run. Results land in gpurun_out/<tag>/. Every GPU step has its own
# time limit; a timeout / abort / segfault ends the script (no further GPU work).
# Extensions are built beforehand on the CPU container (they travel in-tree).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_check.sh r2a'
set -u
TAG=${1:-check}
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" >"$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in
    0) ;;
    *) echo "stopping after $name (rc=$rc)"; tail -30 "$OUT/$name.log"; exit $rc ;;
  esac
}

step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -u -c 'import __graft_entry__ as g; g.smoke()'
step bench 600 python -u bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o kern -- python3 "$ROOT/bench.py" --steps 10 --warmup 2
cd "$ROOT"
tail -3 "$OUT/pytest_gpu.log"
tail -1 "$OUT/bench.log"
echo done
