// MI355X telemetry probe — native half of the plugin's metrics path.
//
// The reference plugin reads GPU power that node-exporter's hwmon collector
// scrapes from i915 sysfs (reference src/components/MetricsPage.tsx:4-27,
// src/api/metrics.ts:1-13). On AMD the same information — and more — lives
// in amdgpu sysfs and the HIP runtime. This probe reads it directly:
//
//   * HIP runtime   device inventory: name, gfx arch, HBM bytes, CUs, LDS,
//                   L2, clocks, PCI BDF, UUID; xGMI link type + hop count
//                   between every device pair (hipExtGetLinkTypeAndHopCount).
//   * amdgpu sysfs  per device (/sys/bus/pci/devices/<bdf>/): power average /
//                   input and cap (hwmon power1_*), edge/junction/memory
//                   temperature (hwmon temp*_input + labels), SCLK/MCLK
//                   (hwmon freq*_input), GFX busy % (gpu_busy_percent),
//                   memory busy % (mem_busy_percent), VRAM used / total
//                   (mem_info_vram_*).
//
// and renders AMD Device Metrics Exporter style text exposition (`gpu_*`
// keyed by hostname + gpu_id) that the plugin's metrics client queries
// (src/api/metrics.js SERIES.exporter). Python binding: CPython C API module
// `_amdgpu_probe` (see bottom of file). Every sysfs field is optional: a
// missing file yields NaN / -1 and the exporter omits the series, which is
// how the plugin's "No data" states are reached.

#include <Python.h>

#include <mutex>

#include "probe_core.h"

namespace {

using namespace amdprobe;

// ---------------------------------------------------------------------------
// Python binding
// ---------------------------------------------------------------------------

PyObject* raise_hip() {
  const std::string e = last_error();  // a copy: another thread may set a new one meanwhile
  PyErr_SetString(PyExc_RuntimeError, e.empty() ? "HIP unavailable" : e.c_str());
  return nullptr;
}

PyObject* py_float_or_none(double v) {
  if (std::isnan(v)) Py_RETURN_NONE;
  return PyFloat_FromDouble(v);
}

PyObject* py_device_count(PyObject*, PyObject*) {
  if (!init_hip()) return PyLong_FromLong(0);
  return PyLong_FromLong(g_count);
}

PyObject* py_device_info(PyObject*, PyObject* args) {
  int dev;
  if (!PyArg_ParseTuple(args, "i", &dev)) return nullptr;
  if (!init_hip()) return raise_hip();
  if (dev < 0 || dev >= g_count) {
    PyErr_Format(PyExc_IndexError, "device %d out of range (count %d)", dev, g_count);
    return nullptr;
  }
  DeviceInfo i;
  if (!device_info(dev, &i)) return raise_hip();
  return Py_BuildValue(
      "{s:i,s:s,s:s,s:s,s:s,s:s,s:s,s:K,s:i,s:i,s:K,s:i,s:i,s:i,s:i}", "index", i.index, "name", i.name.c_str(), "arch",
      i.arch.c_str(), "bdf", i.bdf.c_str(), "uuid", i.uuid.c_str(), "serial", i.serial.c_str(), "device_id",
      i.device_id.c_str(), "hbm_bytes",
      static_cast<unsigned long long>(i.hbm_bytes), "compute_units", i.compute_units, "wavefront", i.wavefront,
      "lds_per_cu", static_cast<unsigned long long>(i.lds_per_cu), "l2_bytes", i.l2_bytes, "clock_khz", i.clock_khz,
      "mem_clock_khz", i.mem_clock_khz, "mem_bus_width", i.mem_bus_width);
}

PyObject* py_link(PyObject*, PyObject* args) {
  int a, b;
  if (!PyArg_ParseTuple(args, "ii", &a, &b)) return nullptr;
  if (!init_hip()) return raise_hip();
  if (a < 0 || b < 0 || a >= g_count || b >= g_count) {
    PyErr_SetString(PyExc_IndexError, "device out of range");
    return nullptr;
  }
  if (a == b) return Py_BuildValue("(sii)", "SELF", 0, 1);
  uint32_t type = 0, hops = 0;
  hipError_t err = hipExtGetLinkTypeAndHopCount(a, b, &type, &hops);
  int peer = 0;
  hipDeviceCanAccessPeer(&peer, a, b);
  if (err != hipSuccess) return Py_BuildValue("(sii)", "UNKNOWN", -1, peer);
  const char* name = type == kLinkTypeXgmi ? "XGMI" : type == kLinkTypePcie ? "PCIE" : "OTHER";
  return Py_BuildValue("(sii)", name, static_cast<int>(hops), peer);
}

// PCI address per device, resolved once. sample() used to call
// hipGetDeviceProperties on every call only to learn the BDF; the inventory
// never changes while the process lives.
std::mutex g_bdf_mu;
std::vector<std::string> g_bdf;

bool cached_bdf(int dev, std::string* bdf) {
  {
    std::lock_guard<std::mutex> lk(g_bdf_mu);
    if (dev < static_cast<int>(g_bdf.size()) && !g_bdf[dev].empty()) {
      *bdf = g_bdf[dev];
      return true;
    }
  }
  DeviceInfo i;
  if (!device_info(dev, &i)) return false;
  std::lock_guard<std::mutex> lk(g_bdf_mu);
  if (static_cast<int>(g_bdf.size()) <= dev) g_bdf.resize(dev + 1);
  g_bdf[dev] = i.bdf;
  *bdf = i.bdf;
  return true;
}

PyObject* py_sample(PyObject*, PyObject* args) {
  int dev;
  if (!PyArg_ParseTuple(args, "i", &dev)) return nullptr;
  if (!init_hip()) return raise_hip();
  if (dev < 0 || dev >= g_count) {
    PyErr_Format(PyExc_IndexError, "device %d out of range (count %d)", dev, g_count);
    return nullptr;
  }
  // The sysfs pass reads firmware-backed files (hwmon power, RAS aca_*) that
  // can block for hundreds of milliseconds; holding the GIL across it froze
  // every other Python thread in the process (the smoke's fake apiserver).
  std::string bdf;
  bool ok;
  Sample s;
  Py_BEGIN_ALLOW_THREADS
  ok = cached_bdf(dev, &bdf);
  if (ok) s = sample_sysfs(bdf);
  Py_END_ALLOW_THREADS
  if (!ok) return raise_hip();
  PyObject* d = PyDict_New();
  auto put = [&](const char* k, double v) {
    PyObject* o = py_float_or_none(v);
    PyDict_SetItemString(d, k, o);
    Py_DECREF(o);
  };
  put("power_w", s.power_w);
  put("power_cap_w", s.power_cap_w);
  put("temp_edge_c", s.temp_edge_c);
  put("temp_junction_c", s.temp_junction_c);
  put("temp_mem_c", s.temp_mem_c);
  put("temp_junction_slowdown_c", s.temp_junction_slowdown_c);
  put("temp_junction_shutdown_c", s.temp_junction_shutdown_c);
  put("temp_mem_slowdown_c", s.temp_mem_slowdown_c);
  put("sclk_mhz", s.sclk_mhz);
  put("mclk_mhz", s.mclk_mhz);
  put("gfx_busy_pct", s.gfx_busy_pct);
  put("mem_busy_pct", s.mem_busy_pct);
  put("vram_used_b", s.vram_used_b);
  put("vram_total_b", s.vram_total_b);
  put("ecc_correct", s.ecc_correct);
  put("ecc_uncorrect", s.ecc_uncorrect);
  put("ecc_deferred", s.ecc_deferred);
  put("ecc_retired_pages", s.ecc_retired_pages);
  auto put_str = [&](const char* k, const std::string& v) {
    PyObject* o = v.empty() ? (Py_INCREF(Py_None), Py_None) : PyUnicode_FromString(v.c_str());
    PyDict_SetItemString(d, k, o);
    Py_DECREF(o);
  };
  put_str("compute_partition", s.compute_partition);
  put_str("memory_partition", s.memory_partition);
  return d;
}

PyObject* py_render(PyObject*, PyObject* args) {
  const char* host = "localhost";
  int device = -1;
  const char* label = "";
  if (!PyArg_ParseTuple(args, "|sis", &host, &device, &label)) return nullptr;
  if (!init_hip()) return PyUnicode_FromString("");
  RenderOptions opt;
  opt.hostname = host;
  opt.only_device = device;
  opt.gpu_label = label;
  std::string s;
  Py_BEGIN_ALLOW_THREADS
  s = render(opt);
  Py_END_ALLOW_THREADS
  return PyUnicode_FromStringAndSize(s.data(), static_cast<Py_ssize_t>(s.size()));
}

PyObject* py_last_error(PyObject*, PyObject*) { return PyUnicode_FromString(last_error().c_str()); }

// RAS counters of a ras/ directory (no HIP needed: tests point it at a fixture tree).
PyObject* py_read_ras(PyObject*, PyObject* args) {
  const char* dir;
  if (!PyArg_ParseTuple(args, "s", &dir)) return nullptr;
  const RasCounts r = read_ras(dir);
  PyObject* ce = py_float_or_none(r.ce);
  PyObject* ue = py_float_or_none(r.ue);
  PyObject* de = py_float_or_none(r.de);
  PyObject* pages = py_float_or_none(r.retired_pages);
  PyObject* d = Py_BuildValue("{s:O,s:O,s:O,s:O,s:i}", "ce", ce, "ue", ue, "de", de, "retired_pages", pages,
                              "blocks", r.blocks);
  Py_DECREF(ce);
  Py_DECREF(ue);
  Py_DECREF(de);
  Py_DECREF(pages);
  return d;
}

PyMethodDef kMethods[] = {
    {"device_count", py_device_count, METH_NOARGS, "Number of HIP devices (0 if HIP is unavailable)."},
    {"device_info", py_device_info, METH_VARARGS, "Static inventory of one device."},
    {"link", py_link, METH_VARARGS, "(type, hops, can_access_peer) between two devices."},
    {"sample", py_sample, METH_VARARGS, "Current amdgpu sysfs telemetry of one device."},
    {"render_metrics", py_render, METH_VARARGS, "Exporter-format text exposition for every device."},
    {"read_ras", py_read_ras, METH_VARARGS, "Summed RAS error counters of one ras/ sysfs directory."},
    {"last_error", py_last_error, METH_NOARGS, "Last HIP error string."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_amdgpu_probe", "MI355X telemetry probe (HIP runtime + amdgpu sysfs).",
                       -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__amdgpu_probe(void) { return PyModule_Create(&kModule); }
