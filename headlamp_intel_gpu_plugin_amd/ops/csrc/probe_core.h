// probe_core.h — MI355X telemetry probe core (HIP runtime + amdgpu sysfs).
//
// Shared by the CPython module (amdgpu_probe.cpp) and the standalone exporter
// daemon (amdgpu_exporter.cpp). See amdgpu_probe.cpp for what is read and why.
#pragma once

#include <hip/hip_runtime.h>

#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <mutex>
#include <string>
#include <vector>

namespace amdprobe {


inline constexpr uint32_t kLinkTypeXgmi = 4;  // HSA_AMD_LINK_INFO_TYPE_XGMI
inline constexpr uint32_t kLinkTypePcie = 2;  // HSA_AMD_LINK_INFO_TYPE_PCIE

struct DeviceInfo {
  int index = -1;
  std::string name;
  std::string arch;
  std::string bdf;  // "0000:05:00.0"
  std::string uuid;    // 32 hex digits of the 16 raw uuid bytes
  std::string serial;  // ASIC serial (amd-smi asic_serial without "0x")
  std::string device_id;  // PCI device id, e.g. "0x75a3"
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

// PCI device ids confirmed on hardware (amd-smi static, tests/fixtures/mi355x).
inline const char* product_for_device_id(const std::string& id) {
  if (id == "0x75a3") return "AMD Instinct MI355X";
  return nullptr;
}

struct Sample {
  double power_w = NAN;      // average (or instantaneous) board power
  double power_cap_w = NAN;  // power1_cap
  double temp_edge_c = NAN, temp_junction_c = NAN, temp_mem_c = NAN;
  // hwmon tempN_crit / tempN_emergency: the slowdown and shutdown thresholds
  // (an MI355X reads 100 / 112 °C junction, 115 / 125 °C HBM: amd-smi static).
  double temp_junction_slowdown_c = NAN, temp_junction_shutdown_c = NAN, temp_mem_slowdown_c = NAN;
  double sclk_mhz = NAN, mclk_mhz = NAN;
  double gfx_busy_pct = NAN, mem_busy_pct = NAN;
  double vram_used_b = NAN, vram_total_b = NAN;
  std::string compute_partition, memory_partition;  // "SPX"/"CPX", "NPS1"/"NPS4"
  // RAS error counters summed over the IP blocks (NaN when the driver has no
  // ras/ directory): corrected, uncorrected, deferred; plus retired HBM pages.
  double ecc_correct = NAN, ecc_uncorrect = NAN, ecc_deferred = NAN, ecc_retired_pages = NAN;
};

inline bool g_hip_ok = false;
inline int g_count = 0;

// The last HIP error, written by whichever thread failed (device_info runs
// with the GIL released, in the exporter's request threads too) and read by
// another: every access goes through this mutex.
inline std::mutex g_error_mu;
inline std::string g_error;

inline void set_error(const std::string& e) {
  std::lock_guard<std::mutex> lk(g_error_mu);
  g_error = e;
}

inline std::string last_error() {
  std::lock_guard<std::mutex> lk(g_error_mu);
  return g_error;
}

// Root of the sysfs tree (tests point it at a captured copy:
// AMDGPU_EXPORTER_SYSFS_ROOT=/tmp/tree reads /tmp/tree/sys/...).
inline std::string sysfs_root() {
  const char* r = std::getenv("AMDGPU_EXPORTER_SYSFS_ROOT");
  return r ? std::string(r) : std::string();
}

inline std::string pci_dir(const std::string& bdf) { return sysfs_root() + "/sys/bus/pci/devices/" + bdf; }

inline bool read_text(const std::string& path, std::string* out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  while (!out->empty() && (out->back() == '\n' || out->back() == ' ')) out->pop_back();
  return true;
}

inline bool read_double(const std::string& path, double* v) {
  std::string s;
  if (!read_text(path, &s) || s.empty()) return false;
  char* end = nullptr;
  double d = std::strtod(s.c_str(), &end);
  if (end == s.c_str()) return false;
  *v = d;
  return true;
}

struct RasCounts {
  double ce = NAN, ue = NAN, de = NAN, retired_pages = NAN;
  int blocks = 0;  // IP blocks that reported counters
};

// One counter file: "ue: N\nce: N[\nde: N]" (ras/aca_<block> on MI300/MI355X,
// ras/<block>_err_count on older parts). Missing keys stay NaN.
inline void parse_ras_counter(const std::string& text, double* ue, double* ce, double* de) {
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {
    const size_t colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string key = line.substr(0, colon);
    while (!key.empty() && key.back() == ' ') key.pop_back();
    char* end = nullptr;
    const char* num = line.c_str() + colon + 1;
    const double v = std::strtod(num, &end);
    if (end == num) continue;
    if (key == "ue") *ue = v;
    else if (key == "ce") *ce = v;
    else if (key == "de") *de = v;
  }
}

inline void add_count(double* acc, double v) {
  if (std::isnan(v)) return;
  *acc = std::isnan(*acc) ? v : *acc + v;
}

// Sum a device's RAS counters. `ras_dir` is <pci device>/ras; the retired
// page table (gpu_vram_bad_pages) has one line per retired page. Per-block
// aca_* files are preferred; the legacy *_err_count files are read only when
// no aca_* file exists, so nothing is counted twice.
inline RasCounts read_ras(const std::string& ras_dir) {
  RasCounts r;
  DIR* d = opendir(ras_dir.c_str());
  if (!d) return r;
  std::vector<std::string> aca, legacy;
  while (dirent* e = readdir(d)) {
    const std::string n = e->d_name;
    if (n.rfind("aca_", 0) == 0) aca.push_back(n);
    else if (n.size() > 10 && n.compare(n.size() - 10, 10, "_err_count") == 0) legacy.push_back(n);
  }
  closedir(d);
  for (const auto& n : aca.empty() ? legacy : aca) {
    std::string text;
    if (!read_text(ras_dir + "/" + n, &text)) continue;
    double ue = NAN, ce = NAN, de = NAN;
    parse_ras_counter(text, &ue, &ce, &de);
    if (std::isnan(ue) && std::isnan(ce)) continue;
    add_count(&r.ue, ue);
    add_count(&r.ce, ce);
    add_count(&r.de, de);
    ++r.blocks;
  }
  std::string pages;
  if (read_text(ras_dir + "/gpu_vram_bad_pages", &pages)) {
    double n = 0;
    std::istringstream in(pages);
    std::string line;
    while (std::getline(in, line)) {
      if (line.find_first_not_of(" \t") != std::string::npos) n += 1;
    }
    r.retired_pages = n;
  }
  return r;
}

inline std::string lower_bdf(const char* bus_id) {
  std::string s(bus_id);
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

inline std::vector<std::string> hwmon_dirs(const std::string& dev_dir) {
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

inline bool init_hip() {
  if (g_hip_ok) return true;
  hipError_t err = hipGetDeviceCount(&g_count);
  if (err != hipSuccess) {
    set_error(std::string("hipGetDeviceCount: ") + hipGetErrorString(err));
    g_count = 0;
    return false;
  }
  g_hip_ok = true;
  return true;
}

inline bool device_info(int dev, DeviceInfo* out) {
  hipDeviceProp_t p;
  hipError_t err = hipGetDeviceProperties(&p, dev);
  if (err != hipSuccess) {
    set_error(std::string("hipGetDeviceProperties: ") + hipGetErrorString(err));
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
  // ROCm fills the uuid with the ASIC serial as ASCII hex digits (an MI355X
  // reads "cc63d7a5..." where amd-smi prints asic_serial 0xCC63D7A5...).
  out->serial.clear();
  for (int i = 0; i < 16; ++i) {
    const char c = p.uuid.bytes[i];
    if (c == 0) break;
    if (!std::isxdigit(static_cast<unsigned char>(c))) {
      out->serial.clear();
      break;
    }
    out->serial.push_back(static_cast<char>(std::toupper(static_cast<unsigned char>(c))));
  }
  if (out->serial.empty()) out->serial = out->uuid;
  const std::string dir = pci_dir(out->bdf);
  std::string s;
  if (read_text(dir + "/device", &s)) out->device_id = s;
  // The HIP device name is empty or generic on some ROCm builds. Prefer the
  // product name of a known device id ("AMD Instinct MI355X"), then the
  // board's FRU name (an MI355X reads "AMD Instinct MI355 OAM").
  if (const char* prod = product_for_device_id(out->device_id)) {
    out->name = prod;
  } else if (read_text(dir + "/product_name", &s) && !s.empty()) {
    out->name = s;
  } else if (out->name.empty() || out->name == "AMD Radeon Graphics") {
    out->name = "AMD Instinct (" + (out->device_id.empty() ? out->arch : out->device_id) + ")";
  }
  return true;
}

inline Sample sample_sysfs(const std::string& bdf) {
  Sample s;
  const std::string dir = pci_dir(bdf);
  double v;
  if (read_double(dir + "/gpu_busy_percent", &v)) s.gfx_busy_pct = v;
  if (read_double(dir + "/mem_busy_percent", &v)) s.mem_busy_pct = v;
  if (read_double(dir + "/mem_info_vram_used", &v)) s.vram_used_b = v;
  if (read_double(dir + "/mem_info_vram_total", &v)) s.vram_total_b = v;
  read_text(dir + "/current_compute_partition", &s.compute_partition);
  read_text(dir + "/current_memory_partition", &s.memory_partition);
  const RasCounts ras = read_ras(dir + "/ras");
  s.ecc_correct = ras.ce;
  s.ecc_uncorrect = ras.ue;
  s.ecc_deferred = ras.de;
  s.ecc_retired_pages = ras.retired_pages;
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
      const std::string base = h + "/temp" + std::to_string(t);
      double crit = NAN, emerg = NAN;
      if (read_double(base + "_crit", &v)) crit = v / 1000.0;
      if (read_double(base + "_emergency", &v)) emerg = v / 1000.0;
      if (label == "edge") {
        s.temp_edge_c = c;
      } else if (label == "junction" || label == "hotspot") {
        s.temp_junction_c = c;
        s.temp_junction_slowdown_c = crit;
        s.temp_junction_shutdown_c = emerg;
      } else if (label == "mem") {
        s.temp_mem_c = c;
        s.temp_mem_slowdown_c = crit;
      } else if (t == 1 && std::isnan(s.temp_edge_c)) {
        s.temp_edge_c = c;
      }
    }
    // clocks: Hz, freq1 = sclk, freq2 = mclk
    if (read_double(h + "/freq1_input", &v)) s.sclk_mhz = v / 1e6;
    if (read_double(h + "/freq2_input", &v)) s.mclk_mhz = v / 1e6;
  }
  return s;
}

// ---------------------------------------------------------------------------
// Device source without the HIP runtime (--sysfs-only): it needs no device
// node, so the exporter runs unprivileged with only /sys mounted read-only.
//   * GPUs are the DRM cards of vendor 0x1002 (/sys/class/drm/cardN/device),
//     in card order — the order the driver probed them, which is also the
//     KFD node order and so the HIP device order (no *_VISIBLE_DEVICES mask);
//   * telemetry comes from the same amdgpu sysfs / hwmon files as with HIP;
//   * xGMI links come from the KFD topology (/sys/class/kfd/kfd/topology):
//     io_links of type 11 (CRAT_IOLINK_TYPE_XGMI) between GPU nodes, 1 hop.
//     KFD shows a GPU node's properties only to a process whose device cgroup
//     admits that GPU's render node ("Operation not permitted" otherwise:
//     tests/fixtures/mi355x/kfd_topology.txt, captured in a 1-GPU container on
//     an 8 x MI355X host). A link is exported only when both ends are
//     readable; an unprivileged pod therefore exports no link series, and the
//     plugin says its xGMI matrix is the assumed MI355X mesh.
// ---------------------------------------------------------------------------

inline constexpr int kKfdIoLinkXgmi = 11;

// "key value" lines of a KFD properties file.
inline bool kfd_props(const std::string& path, std::vector<std::pair<std::string, double>>* out) {
  std::string text;
  if (!read_text(path, &text)) return false;
  std::istringstream in(text);
  std::string k;
  double v;
  while (in >> k >> v) out->emplace_back(k, v);
  return !out->empty();
}

inline double kfd_get(const std::vector<std::pair<std::string, double>>& p, const char* key, double dflt) {
  for (const auto& kv : p)
    if (kv.first == key) return kv.second;
  return dflt;
}

// Numeric suffixes of the entries of `dir` that start with `prefix` ("card3" → 3).
inline std::vector<int> numbered_entries(const std::string& dir, const char* prefix) {
  std::vector<int> out;
  DIR* d = opendir(dir.c_str());
  if (!d) return out;
  const size_t pl = std::strlen(prefix);
  while (dirent* e = readdir(d)) {
    if (std::strncmp(e->d_name, prefix, pl) != 0) continue;
    const char* num = e->d_name + pl;
    char* end = nullptr;
    const long n = std::strtol(num, &end, 10);
    if (end != num && *end == '\0') out.push_back(static_cast<int>(n));
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

inline std::string lower_hex(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

// PCI addresses of the AMD GPUs, in DRM card order.
inline std::vector<std::string> sysfs_gpu_bdfs() {
  std::vector<std::string> out;
  const std::string drm = sysfs_root() + "/sys/class/drm";
  for (int n : numbered_entries(drm, "card")) {
    const std::string dev = drm + "/card" + std::to_string(n) + "/device";
    std::string vendor;
    if (!read_text(dev + "/vendor", &vendor) || lower_hex(vendor) != "0x1002") continue;
    char buf[4096];
    const ssize_t len = readlink(dev.c_str(), buf, sizeof(buf) - 1);
    if (len <= 0) continue;
    buf[len] = 0;
    std::string bdf = buf;
    const size_t slash = bdf.rfind('/');
    if (slash != std::string::npos) bdf = bdf.substr(slash + 1);
    bdf = lower_hex(bdf);
    if (std::find(out.begin(), out.end(), bdf) == out.end()) out.push_back(bdf);
  }
  return out;
}

inline std::string kfd_bdf(long long domain, long long location_id) {
  char b[32];
  std::snprintf(b, sizeof(b), "%04llx:%02llx:%02llx.%llx", domain, (location_id >> 8) & 0xff,
                (location_id >> 3) & 0x1f, location_id & 0x7);
  return b;
}

// One direct xGMI link between GPU ordinals, and its position among the
// source node's xGMI io_links in io_link number order (io_links/0, /1, ...,
// counting links to GPUs this process cannot read too): the neighbour order
// the exporter publishes as the `neighbor` label, so a consumer can place a
// per-neighbour series (xgmi_neighbor_<k>_*) on its peer.
struct XgmiLink {
  int from;
  int to;
  int neighbor;
};

// Direct xGMI links between GPU ordinals (indices into `bdfs`), one per
// direction, from the KFD nodes this process may read.
inline std::vector<XgmiLink> kfd_xgmi_links(const std::vector<std::string>& bdfs) {
  const std::string base = sysfs_root() + "/sys/class/kfd/kfd/topology/nodes";
  std::vector<int> ordinal_of_node;  // KFD node → GPU ordinal (-1: CPU or unreadable)
  std::vector<std::vector<std::pair<int, int>>> links;  // per node: (type, node_to), in io_link order
  for (int n : numbered_entries(base, "")) {
    if (n >= static_cast<int>(ordinal_of_node.size())) {
      ordinal_of_node.resize(n + 1, -1);
      links.resize(n + 1);
    }
    const std::string nd = base + "/" + std::to_string(n);
    std::vector<std::pair<std::string, double>> p;
    if (!kfd_props(nd + "/properties", &p) || kfd_get(p, "simd_count", 0) <= 0) continue;
    const std::string bdf = kfd_bdf(static_cast<long long>(kfd_get(p, "domain", 0)),
                                    static_cast<long long>(kfd_get(p, "location_id", 0)));
    const auto it = std::find(bdfs.begin(), bdfs.end(), bdf);
    if (it == bdfs.end()) continue;
    ordinal_of_node[n] = static_cast<int>(it - bdfs.begin());
    for (int l : numbered_entries(nd + "/io_links", "")) {
      std::vector<std::pair<std::string, double>> lp;
      // An unreadable link keeps its place (type 0) so later neighbours keep their numbers.
      if (!kfd_props(nd + "/io_links/" + std::to_string(l) + "/properties", &lp)) lp.clear();
      links[n].emplace_back(static_cast<int>(kfd_get(lp, "type", 0)), static_cast<int>(kfd_get(lp, "node_to", -1)));
    }
  }
  std::vector<XgmiLink> out;
  for (size_t n = 0; n < links.size(); ++n) {
    if (ordinal_of_node[n] < 0) continue;
    int k = 0;
    for (const auto& tl : links[n]) {
      if (tl.first != kKfdIoLinkXgmi) continue;
      const int neighbor = k++;
      if (tl.second < 0 || tl.second >= static_cast<int>(ordinal_of_node.size())) continue;
      const int peer = ordinal_of_node[tl.second];
      if (peer >= 0 && peer != ordinal_of_node[n]) out.push_back({ordinal_of_node[n], peer, neighbor});
    }
  }
  return out;
}

// DeviceInfo from sysfs alone (no HIP): what the labels and HBM total need.
inline DeviceInfo sysfs_device_info(const std::string& bdf, int ordinal) {
  DeviceInfo d;
  d.index = ordinal;
  d.bdf = bdf;
  const std::string dir = pci_dir(bdf);
  std::string s;
  if (read_text(dir + "/device", &s)) d.device_id = lower_hex(s);
  if (read_text(dir + "/unique_id", &s) && !s.empty()) {
    d.serial = s;
    for (auto& c : d.serial) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
  }
  double v;
  if (read_double(dir + "/mem_info_vram_total", &v)) d.hbm_bytes = static_cast<size_t>(v);
  if (const char* prod = product_for_device_id(d.device_id)) d.name = prod;
  else if (read_text(dir + "/product_name", &s) && !s.empty()) d.name = s;
  else d.name = "AMD Instinct (" + (d.device_id.empty() ? std::string("unknown") : d.device_id) + ")";
  return d;
}

inline void append_metric(std::string* out, const char* name, const std::string& labels, double v) {
  if (std::isnan(v)) return;
  char num[64];
  std::snprintf(num, sizeof(num), "%.6g", v);
  out->append(name).append("{").append(labels).append("} ").append(num).append("\n");
}

inline std::string escape_label(const std::string& s) {
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

struct RenderOptions {
  std::string hostname = "localhost";
  int only_device = -1;      // export just this HIP device (-1 = all)
  std::string gpu_label;     // override the gpu_id label (with only_device)
  bool topology = true;      // emit xGMI link metrics between exported devices
  bool sysfs_only = false;   // enumerate devices from sysfs, links from the KFD topology (no HIP)
};

// Render devices in exporter format. Units follow the AMD Device Metrics
// Exporter conventions the plugin reads: watts, percent, MiB, °C, MHz.
inline std::string render(const RenderOptions& opt) {
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
      {"gpu_junction_temperature_slowdown", "junction temperature at which the GPU throttles (C)"},
      {"gpu_junction_temperature_shutdown", "junction temperature at which the GPU shuts down (C)"},
      {"gpu_memory_temperature_slowdown", "HBM temperature at which the GPU throttles (C)"},
      {"gpu_clock", "GFX clock (MHz)"},
      {"gpu_memory_clock", "memory clock (MHz)"},
      {"gpu_power_cap", "board power cap (W)"},
      {"gpu_xgmi_link_hops", "hops between two GPUs over xGMI (absent when not xGMI-connected)"},
      {"gpu_partition_info", "compute/memory partition mode of the GPU (value is always 1)"},
      {"gpu_ecc_correct_total", "corrected RAS errors since driver load, all IP blocks"},
      {"gpu_ecc_uncorrect_total", "uncorrected RAS errors since driver load, all IP blocks"},
      {"gpu_ecc_deferred_total", "deferred RAS errors since driver load, all IP blocks"},
      {"gpu_ecc_retired_pages", "HBM pages retired by the driver"},
  };
  for (auto& h : kHelp) {
    out.append("# HELP ").append(h[0]).append(" ").append(h[1]).append("\n");
    const std::string n = h[0];
    const bool counter = n.size() > 6 && n.compare(n.size() - 6, 6, "_total") == 0;
    out.append("# TYPE ").append(h[0]).append(counter ? " counter\n" : " gauge\n");
  }
  const double mib = 1024.0 * 1024.0;
  // Devices from HIP, or from sysfs alone (--sysfs-only).
  const bool from_sysfs = opt.sysfs_only;
  const std::vector<std::string> bdfs = from_sysfs ? sysfs_gpu_bdfs() : std::vector<std::string>();
  const int count = from_sysfs ? static_cast<int>(bdfs.size()) : g_count;
  for (int d = 0; d < count; ++d) {
    if (opt.only_device >= 0 && d != opt.only_device) continue;
    DeviceInfo info;
    if (from_sysfs) info = sysfs_device_info(bdfs[d], d);
    else if (!device_info(d, &info)) continue;
    Sample s = sample_sysfs(info.bdf);
    const std::string gid = (opt.only_device >= 0 && !opt.gpu_label.empty()) ? opt.gpu_label : std::to_string(d);
    std::string labels = "hostname=\"" + escape_label(opt.hostname) + "\",gpu_id=\"" + escape_label(gid) +
                         "\",card_model=\"" + escape_label(info.name) + "\",pci_bus=\"" + info.bdf +
                         "\",serial_number=\"" + escape_label(info.serial) + "\"";
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
    append_metric(&out, "gpu_junction_temperature_slowdown", labels, s.temp_junction_slowdown_c);
    append_metric(&out, "gpu_junction_temperature_shutdown", labels, s.temp_junction_shutdown_c);
    append_metric(&out, "gpu_memory_temperature_slowdown", labels, s.temp_mem_slowdown_c);
    append_metric(&out, "gpu_clock", labels, s.sclk_mhz);
    append_metric(&out, "gpu_memory_clock", labels, s.mclk_mhz);
    append_metric(&out, "gpu_ecc_correct_total", labels, s.ecc_correct);
    append_metric(&out, "gpu_ecc_uncorrect_total", labels, s.ecc_uncorrect);
    append_metric(&out, "gpu_ecc_deferred_total", labels, s.ecc_deferred);
    append_metric(&out, "gpu_ecc_retired_pages", labels, s.ecc_retired_pages);
    if (!s.compute_partition.empty() || !s.memory_partition.empty()) {
      append_metric(&out, "gpu_partition_info",
                    labels + ",compute_partition=\"" + escape_label(s.compute_partition) + "\",memory_partition=\"" +
                        escape_label(s.memory_partition) + "\"",
                    1.0);
    }
  }
  if (opt.topology && opt.only_device < 0) {
    // `neighbor` (sysfs mode): the link's place in the KFD io_link order of gpu_id's node.
    auto link = [&](int a, int b, double hops, int neighbor) {
      append_metric(&out, "gpu_xgmi_link_hops",
                    "hostname=\"" + escape_label(opt.hostname) + "\",gpu_id=\"" + std::to_string(a) +
                        "\",peer_gpu_id=\"" + std::to_string(b) + "\"" +
                        (neighbor >= 0 ? ",neighbor=\"" + std::to_string(neighbor) + "\"" : std::string()),
                    hops);
    };
    if (from_sysfs) {
      for (const auto& l : kfd_xgmi_links(bdfs)) link(l.from, l.to, 1.0, l.neighbor);
    } else {
      for (int a = 0; a < g_count; ++a) {
        for (int b = 0; b < g_count; ++b) {
          if (a == b) continue;
          uint32_t type = 0, hops = 0;
          if (hipExtGetLinkTypeAndHopCount(a, b, &type, &hops) != hipSuccess || type != kLinkTypeXgmi) continue;
          link(a, b, static_cast<double>(hops), -1);  // HIP reports no neighbour order
        }
      }
    }
  }
  return out;
}

inline std::string render(const std::string& hostname) {
  RenderOptions o;
  o.hostname = hostname;
  return render(o);
}

}  // namespace amdprobe
