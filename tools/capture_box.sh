#!/usr/bin/env bash
# Capture ground-truth MI355X telemetry/topology fixtures on a GPU box.
#
#   gpurun -- 'bash tools/capture_box.sh'
#
# Writes gpurun_out/capture/: the native exporter's scrape, amd-smi /
# rocm-smi JSON (static info, metrics, xGMI topology) and the amdgpu
# sysfs/hwmon file names the probe reads. Each step has its own time limit;
# a step that times out or crashes ends the script.
set -u
OUT=gpurun_out/capture
mkdir -p "$OUT"

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" >"$OUT/$name" 2>"$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in
    124 | 134 | 137 | 139) echo "stopping after $name (rc=$rc)"; exit $rc ;;
  esac
  return 0
}

python -m headlamp_intel_gpu_plugin_amd.ops.build >"$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 1; }
EXE=headlamp_intel_gpu_plugin_amd/ops/bin/amdgpu-exporter
step exporter_once.prom 60 "$EXE" --once --hostname mi355x-node-0
step amd_smi_static.json 60 amd-smi static --json
step amd_smi_metric.json 90 amd-smi metric --json
step amd_smi_topology.json 60 amd-smi topology --json
step amd_smi_list.json 60 amd-smi list --json
step rocm_smi_showtopo.json 60 rocm-smi --showtopo --json
step rocm_smi_info.json 60 rocm-smi --showproductname --showpower --showmeminfo vram --showuse --json
# sysfs names only (no values that identify the machine).
ls /sys/class/drm >"$OUT/sysfs_drm.txt" 2>&1 || true
for c in /sys/class/drm/card*/device; do
  [ -e "$c/vendor" ] || continue
  echo "== $c vendor=$(cat "$c/vendor" 2>/dev/null) device=$(cat "$c/device" 2>/dev/null)"
  ls "$c" | grep -E '^(mem_info|gpu_busy|power|current_|pp_|hwmon|xgmi)' || true
  ls "$c"/hwmon/hwmon*/ 2>/dev/null | grep -E '^(power|temp|energy|freq)' || true
done >"$OUT/sysfs_amdgpu.txt" 2>&1
echo done
