// numa.hpp — host NUMA placement of the pinned staging memory and the host
// threads that feed a GPU (the 8-GPU host-staged config: each rank's pinned
// pool, its generator threads and its file-reader threads on the GPU's own
// socket, so H2D traffic never crosses the socket link).
//
// Reference: the reference copies its input with one blocking cudaMemcpy from
// unpinned memory (/root/reference/main.cu:143-147) and has no notion of
// placement.
#pragma once
#include <string>
#include <vector>

namespace wc {

struct NumaNode {
  int node = -1;          // -1: unknown (no sysfs entry, single-node host, or binding off)
  std::vector<int> cpus;  // the node's CPUs (empty: do not bind)
};

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}; malformed pieces are skipped.
std::vector<int> parse_cpulist(const std::string& s);
// CPUs of node `node` (root/devices/system/node/node<N>/cpulist).
NumaNode numa_node_cpus(int node, const std::string& sysfs_root = "/sys");
// Node of a PCI device (root/bus/pci/devices/<bus id>/numa_node) and its CPUs.
NumaNode numa_of_pci(const std::string& bus_id, const std::string& sysfs_root = "/sys");
// Node of a HIP device (its PCI bus id).  WC_NUMA_NODE=<n> forces node n (the
// local / remote H2D measurement), WC_NUMA_NODE=off disables binding.
NumaNode numa_of_device(int device);

// Binds the calling thread to `cpus` for the scope (threads it creates inherit
// the mask; pinned pages it allocates are placed by the kernel's local-node
// policy), then restores the previous mask.  No-op for an empty list.
class ScopedAffinity {
 public:
  explicit ScopedAffinity(const std::vector<int>& cpus);
  ~ScopedAffinity();
  ScopedAffinity(const ScopedAffinity&) = delete;
  ScopedAffinity& operator=(const ScopedAffinity&) = delete;
  bool active() const { return active_; }

 private:
  bool active_ = false;
  std::vector<unsigned char> old_;  // cpu_set_t bytes
};

}  // namespace wc
