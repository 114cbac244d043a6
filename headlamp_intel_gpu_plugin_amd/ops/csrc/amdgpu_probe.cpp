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
#include <hip/hip_runtime.h>

#include <dirent.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

constexpr uint32_t kLinkTypeXgmi = 4;  // HSA_AMD_LINK_INFO_TYPE_XGMI
constexpr uint32_t kLinkTypePcie = 2;  // HSA_AMD_LINK_INFO_TYPE_PCIE

struct DeviceInfo {
  int index = -1;
  std::string name;
  std::string arch;
  std::string bdf;  // "0000:05:00.0"
  std::string uuid;
  size_t hbm_bytes = 0;
  int compute_units = 0;
  int wavefront = 0;
  size_t lds_per_cu = 0;
  int l2_bytes = 0;
  int clock_khz = 0;
  int mem_clock_khz = 0;
  int mem_bus_width = 0;
  int pci_domain = 0, pci_bus = 0, pci_device = 0;
};

struct Sample {
  double power_w = NAN;      // average (or instantaneous) board power
  double power_cap_w = NAN;  // power1_cap
  double temp_edge_c = NAN, temp_junction_c = NAN, temp_mem_c = NAN;
  double sclk_mhz = NAN, mclk_mhz = NAN;
  double gfx_busy_pct = NAN, mem_busy_pct = NAN;
  double vram_used_b = NAN, vram_total_b = NAN;
};

bool g_hip_ok = false;
int g_count = 0;
std::string g_error;

bool read_text(const std::string& path, std::string* out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  while (!out->empty() && (out->back() == '\n' || out->back() == ' ')) out->pop_back();
  return true;
}

bool read_double(const std::string& path, double* v) {
  std::string s;
  if (!read_text(path, &s) || s.empty()) return false;
  char* end = nullptr;
  double d = std::strtod(s.c_str(), &end);
  if (end == s.c_str()) return false;
  *v = d;
  return true;
}

std::string lower_bdf(const char* bus_id) {
  std::string s(bus_id);
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

std::vector<std::string> hwmon_dirs(const std::string& dev_dir) {
  std::vector<std::string> out;
  std::string base = dev_dir + "/hwmon";
  DIR* d = opendir(base.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (std::strncmp(e->d_name, "hwmon", 5) == 0) out.push_back(base + "/" + e->d_name);
  }
  closedir(d);
  return out;
}

bool init_hip() {
  if (g_hip_ok) return true;
  hipError_t err = hipGetDeviceCount(&g_count);
  if (err != hipSuccess) {
    g_error = std::string("hipGetDeviceCount: ") + hipGetErrorString(err);
    g_count = 0;
    return false;
  }
  g_hip_ok = true;
  return true;
}

bool device_info(int dev, DeviceInfo* out) {
  hipDeviceProp_t p;
  hipError_t err = hipGetDeviceProperties(&p, dev);
  if (err != hipSuccess) {
    g_error = std::string("hipGetDeviceProperties: ") + hipGetErrorString(err);
    return false;
  }
  out->index = dev;
  out->name = p.name;
  out->arch = p.gcnArchName;
  out->hbm_bytes = p.totalGlobalMem;
  out->compute_units = p.multiProcessorCount;
  out->wavefront = p.warpSize;
  out->lds_per_cu = p.maxSharedMemoryPerMultiProcessor;
  out->l2_bytes = p.l2CacheSize;
  out->clock_khz = p.clockRate;
  out->mem_clock_khz = p.memoryClockRate;
  out->mem_bus_width = p.memoryBusWidth;
  out->pci_domain = p.pciDomainID;
  out->pci_bus = p.pciBusID;
  out->pci_device = p.pciDeviceID;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) == hipSuccess) {
    out->bdf = lower_bdf(bus);
  } else {
    char tmp[64];
    std::snprintf(tmp, sizeof(tmp), "%04x:%02x:%02x.0", p.pciDomainID, p.pciBusID, p.pciDeviceID);
    out->bdf = tmp;
  }
  char hex[40] = {0};
  for (int i = 0; i < 16; ++i) std::snprintf(hex + 2 * i, 3, "%02x", static_cast<unsigned char>(p.uuid.bytes[i]));
  out->uuid = hex;
  return true;
}

Sample sample_sysfs(const std::string& bdf) {
  Sample s;
  const std::string dir = "/sys/bus/pci/devices/" + bdf;
  double v;
  if (read_double(dir + "/gpu_busy_percent", &v)) s.gfx_busy_pct = v;
  if (read_double(dir + "/mem_busy_percent", &v)) s.mem_busy_pct = v;
  if (read_double(dir + "/mem_info_vram_used", &v)) s.vram_used_b = v;
  if (read_double(dir + "/mem_info_vram_total", &v)) s.vram_total_b = v;
  for (const auto& h : hwmon_dirs(dir)) {
    // power: µW
    if (std::isnan(s.power_w) && read_double(h + "/power1_average", &v)) s.power_w = v / 1e6;
    if (std::isnan(s.power_w) && read_double(h + "/power1_input", &v)) s.power_w = v / 1e6;
    if (std::isnan(s.power_cap_w) && read_double(h + "/power1_cap", &v)) s.power_cap_w = v / 1e6;
    // temperatures: m°C, labelled edge / junction / mem
    for (int t = 1; t <= 4; ++t) {
      const std::string in = h + "/temp" + std::to_string(t) + "_input";
      if (!read_double(in, &v)) continue;
      std::string label;
      read_text(h + "/temp" + std::to_string(t) + "_label", &label);
      const double c = v / 1000.0;
      if (label == "edge") s.temp_edge_c = c;
      else if (label == "junction" || label == "hotspot") s.temp_junction_c = c;
      else if (label == "mem") s.temp_mem_c = c;
      else if (t == 1 && std::isnan(s.temp_edge_c)) s.temp_edge_c = c;
    }
    // clocks: Hz, freq1 = sclk, freq2 = mclk
    if (read_double(h + "/freq1_input", &v)) s.sclk_mhz = v / 1e6;
    if (read_double(h + "/freq2_input", &v)) s.mclk_mhz = v / 1e6;
  }
  return s;
}

void append_metric(std::string* out, const char* name, const std::string& labels, double v) {
  if (std::isnan(v)) return;
  char num[64];
  std::snprintf(num, sizeof(num), "%.6g", v);
  out->append(name).append("{").append(labels).append("} ").append(num).append("\n");
}

std::string escape_label(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '\\' || c == '"') o.push_back('\\');
    if (c == '\n') {
      o.append("\\n");
      continue;
    }
    o.push_back(c);
  }
  return o;
}

// Render every device in exporter format. Units follow the AMD Device Metrics
// Exporter conventions the plugin reads: watts, percent, MiB, °C, MHz.
std::string render(const std::string& hostname) {
  std::string out;
  out.reserve(4096);
  static const char* kHelp[][2] = {
      {"gpu_power_usage", "GPU board power (W)"},
      {"gpu_gfx_activity", "GFX engine busy (%)"},
      {"gpu_umc_activity", "HBM memory-controller busy (%)"},
      {"gpu_used_vram", "HBM in use (MiB)"},
      {"gpu_total_vram", "HBM capacity (MiB)"},
      {"gpu_edge_temperature", "edge temperature (C)"},
      {"gpu_junction_temperature", "junction temperature (C)"},
      {"gpu_memory_temperature", "HBM temperature (C)"},
      {"gpu_clock", "GFX clock (MHz)"},
      {"gpu_memory_clock", "memory clock (MHz)"},
      {"gpu_power_cap", "board power cap (W)"},
  };
  for (auto& h : kHelp) {
    out.append("# HELP ").append(h[0]).append(" ").append(h[1]).append("\n");
    out.append("# TYPE ").append(h[0]).append(" gauge\n");
  }
  for (int d = 0; d < g_count; ++d) {
    DeviceInfo info;
    if (!device_info(d, &info)) continue;
    Sample s = sample_sysfs(info.bdf);
    std::string labels = "hostname=\"" + escape_label(hostname) + "\",gpu_id=\"" + std::to_string(d) +
                         "\",card_model=\"" + escape_label(info.name) + "\",pci_bus=\"" + info.bdf + "\",serial_number=\"" +
                         info.uuid + "\"";
    const double mib = 1024.0 * 1024.0;
    append_metric(&out, "gpu_power_usage", labels, s.power_w);
    append_metric(&out, "gpu_power_cap", labels, s.power_cap_w);
    append_metric(&out, "gpu_gfx_activity", labels, s.gfx_busy_pct);
    append_metric(&out, "gpu_umc_activity", labels, s.mem_busy_pct);
    append_metric(&out, "gpu_used_vram", labels, std::isnan(s.vram_used_b) ? NAN : s.vram_used_b / mib);
    append_metric(&out, "gpu_total_vram", labels,
                  std::isnan(s.vram_total_b) ? static_cast<double>(info.hbm_bytes) / mib : s.vram_total_b / mib);
    append_metric(&out, "gpu_edge_temperature", labels, s.temp_edge_c);
    append_metric(&out, "gpu_junction_temperature", labels, s.temp_junction_c);
    append_metric(&out, "gpu_memory_temperature", labels, s.temp_mem_c);
    append_metric(&out, "gpu_clock", labels, s.sclk_mhz);
    append_metric(&out, "gpu_memory_clock", labels, s.mclk_mhz);
  }
  return out;
}

// ---------------------------------------------------------------------------
// Python binding
// ---------------------------------------------------------------------------

PyObject* raise_hip() {
  PyErr_SetString(PyExc_RuntimeError, g_error.empty() ? "HIP unavailable" : g_error.c_str());
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
      "{s:i,s:s,s:s,s:s,s:s,s:K,s:i,s:i,s:K,s:i,s:i,s:i,s:i}", "index", i.index, "name", i.name.c_str(), "arch",
      i.arch.c_str(), "bdf", i.bdf.c_str(), "uuid", i.uuid.c_str(), "hbm_bytes",
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

PyObject* py_sample(PyObject*, PyObject* args) {
  int dev;
  if (!PyArg_ParseTuple(args, "i", &dev)) return nullptr;
  if (!init_hip()) return raise_hip();
  if (dev < 0 || dev >= g_count) {
    PyErr_Format(PyExc_IndexError, "device %d out of range (count %d)", dev, g_count);
    return nullptr;
  }
  DeviceInfo i;
  if (!device_info(dev, &i)) return raise_hip();
  Sample s = sample_sysfs(i.bdf);
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
  put("sclk_mhz", s.sclk_mhz);
  put("mclk_mhz", s.mclk_mhz);
  put("gfx_busy_pct", s.gfx_busy_pct);
  put("mem_busy_pct", s.mem_busy_pct);
  put("vram_used_b", s.vram_used_b);
  put("vram_total_b", s.vram_total_b);
  return d;
}

PyObject* py_render(PyObject*, PyObject* args) {
  const char* host = "localhost";
  if (!PyArg_ParseTuple(args, "|s", &host)) return nullptr;
  if (!init_hip()) return PyUnicode_FromString("");
  std::string s;
  Py_BEGIN_ALLOW_THREADS
  s = render(host);
  Py_END_ALLOW_THREADS
  return PyUnicode_FromStringAndSize(s.data(), static_cast<Py_ssize_t>(s.size()));
}

PyObject* py_last_error(PyObject*, PyObject*) { return PyUnicode_FromString(g_error.c_str()); }

PyMethodDef kMethods[] = {
    {"device_count", py_device_count, METH_NOARGS, "Number of HIP devices (0 if HIP is unavailable)."},
    {"device_info", py_device_info, METH_VARARGS, "Static inventory of one device."},
    {"link", py_link, METH_VARARGS, "(type, hops, can_access_peer) between two devices."},
    {"sample", py_sample, METH_VARARGS, "Current amdgpu sysfs telemetry of one device."},
    {"render_metrics", py_render, METH_VARARGS, "Exporter-format text exposition for every device."},
    {"last_error", py_last_error, METH_NOARGS, "Last HIP error string."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_amdgpu_probe", "MI355X telemetry probe (HIP runtime + amdgpu sysfs).",
                       -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__amdgpu_probe(void) { return PyModule_Create(&kModule); }
