#!/usr/bin/env bash
# PMC counters for the workload kernels (own run: --pmc with kernel trace only).
#   gpurun -- 'bash tools/pmc_box.sh'
set -u
ROOT=$PWD
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
python -m headlamp_intel_gpu_plugin_amd.ops.build >"$OUT/build.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L >"$OUT/counters.txt" 2>&1
echo "list rc=$?"
run() {  # run <name> <counters...>
  local name=$1
  shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o "$name" -- python3 "$ROOT/profiles/run_gemm_pmc.py" >"$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124 | 134 | 137 | 139) exit $rc ;; esac
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY
run mem TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum
echo done
