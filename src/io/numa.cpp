// numa.cpp — sysfs NUMA resolution and thread binding (numa.hpp).
#include "numa.hpp"

#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace wc {

namespace {
bool read_text(const std::string& path, std::string& out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}
}  // namespace

std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    part.erase(std::remove_if(part.begin(), part.end(), [](unsigned char c) { return std::isspace(c); }), part.end());
    if (part.empty()) continue;
    char* end = nullptr;
    const long a = std::strtol(part.c_str(), &end, 10);
    if (end == part.c_str() || a < 0) continue;
    long b = a;
    if (*end == '-') {
      char* e2 = nullptr;
      b = std::strtol(end + 1, &e2, 10);
      if (e2 == end + 1 || *e2 || b < a) continue;
    } else if (*end) {
      continue;
    }
    for (long c = a; c <= b && c < 65536; ++c) out.push_back((int)c);
  }
  return out;
}

NumaNode numa_node_cpus(int node, const std::string& sysfs_root) {
  NumaNode n;
  if (node < 0) return n;
  std::string txt;
  if (!read_text(sysfs_root + "/devices/system/node/node" + std::to_string(node) + "/cpulist", txt)) return n;
  n.node = node;
  n.cpus = parse_cpulist(txt);
  return n;
}

NumaNode numa_of_pci(const std::string& bus_id, const std::string& sysfs_root) {
  std::string id = bus_id;
  for (char& c : id) c = (char)std::tolower((unsigned char)c);
  std::string txt;
  if (!read_text(sysfs_root + "/bus/pci/devices/" + id + "/numa_node", txt)) return NumaNode{};
  const int node = std::atoi(txt.c_str());
  return node >= 0 ? numa_node_cpus(node, sysfs_root) : NumaNode{};
}

NumaNode numa_of_device(int device) {
  if (const char* e = std::getenv("WC_NUMA_NODE"); e && *e) {
    if (std::strcmp(e, "off") == 0) return NumaNode{};
    return numa_node_cpus(std::atoi(e));
  }
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return NumaNode{};
  }
  return numa_of_pci(bus);
}

ScopedAffinity::ScopedAffinity(const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t old, want;
  CPU_ZERO(&want);
  int n = 0;
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) {
      CPU_SET(c, &want);
      ++n;
    }
  if (!n || sched_getaffinity(0, sizeof old, &old) != 0) return;
  if (sched_setaffinity(0, sizeof want, &want) != 0) return;  // e.g. CPUs outside the cgroup: stay unbound
  old_.assign(reinterpret_cast<const unsigned char*>(&old), reinterpret_cast<const unsigned char*>(&old) + sizeof old);
  active_ = true;
}

ScopedAffinity::~ScopedAffinity() {
  if (!active_) return;
  cpu_set_t old;
  std::memcpy(&old, old_.data(), sizeof old);
  (void)sched_setaffinity(0, sizeof old, &old);
}

}  // namespace wc
