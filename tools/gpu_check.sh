#!/usr/bin/env bash
# One GPU-box pass: build, GEMM A/B, GPU tests, 1-GPU bench, rocprofv3 kernel
# stats. Results land in gpurun_out/<tag>/. Every GPU step has its own time
# limit; a timeout / abort / segfault ends the script (no further GPU work).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_check.sh r1b'
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
    124 | 134 | 137 | 139) echo "stopping after $name (rc=$rc)"; tail -20 "$OUT/$name.log"; exit $rc ;;
  esac
  return 0
}

python -m headlamp_intel_gpu_plugin_amd.ops.build >"$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 1; }
step gemm_ab 600 python tools/gemm_ab.py --sizes 2048 4096 8192 --out "$OUT/gemm_ab.json"
step pytest_gpu 900 python -m pytest tests -m gpu -q
step bench 600 python bench.py --steps 30 --warmup 5 --out "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o kern -- python3 "$ROOT/profiles/run_kernels.py"
cd "$ROOT"
tail -3 "$OUT/pytest_gpu.log"
tail -1 "$OUT/bench.log"
echo done
