// host_numa.h -- host topology for the C++ host layers: which NUMA node a GPU
// hangs off, which CPUs the process may use, and a scope that binds the
// calling thread's CPUs and page placement to one node.
//
// each GPU's shard is staged from pinned host memory local to
// that GPU's NUMA node.  The session of device d (host_session.h) allocates
// its pinned staging inside a NumaBind(node(d)) scope with
// hipHostMallocNumaUser, so the pages land on d's node; the worker pool keeps
// one group of threads per node and hands a session's copy jobs to its own
// node's group first; lsbm_crc32c_batch_host_multi binds each device's host
// thread to that device's node.  The reference runs its writer, compaction
// and reader threads concurrently in one process (util/env_posix.cc:546-586,
// lsbm/db_bench.cc:711-736); on a node with 8 GPUs over 2 sockets those
// threads reach 8 devices on two nodes.
//
// Everything degrades to "no NUMA information" (node -1: no binding, HIP's
// default placement) when sysfs or the syscalls are unavailable.
#pragma once
#include <sched.h>
#include <stddef.h>

#include <vector>

namespace lsbm {

// "0000:c1:00.0" (any case) -> the numa_node file under
// <sysfs_root>/bus/pci/devices/<bus id>/ ; -1 if absent or negative.
int pci_numa_node(const char* sysfs_root, const char* bus_id);

// The NUMA node of HIP device `device` (cached; -1 if unknown).
int device_numa_node(int device);

// "0-3,8,10-11" -> the CPUs; false on a malformed list.
bool parse_cpulist(const char* s, std::vector<int>* cpus);

// CPUs of `node` (<sysfs_root>/devices/system/node/node<N>/cpulist).
bool node_cpulist(const char* sysfs_root, int node, std::vector<int>* cpus);

// CPUs this process may run on, and the cgroup CPU quota in whole CPUs
// (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us; 0 if none).
std::vector<int> affinity_cpus();
int cgroup_cpu_quota(const char* cgroup_root);
// The quota of the process's own cgroup: its path from `proc_cgroup` (the
// text of /proc/self/cgroup: the v2 "0::<path>" line, else the v1 line whose
// controllers include cpu) under the mount `cgroup_root`, the smallest over
// that directory and its ancestors; the mount root's own quota when none is
// found there (a cgroup namespace shows its cgroup as "/").
int cgroup_cpu_quota_of(const char* cgroup_root, const char* proc_cgroup);

// Threads worth running at once: the affinity mask's CPUs, capped by the
// cgroup quota (the GPU box: 256 CPUs in the mask, a quota of 16).
// LSBM_HOST_THREADS overrides.
int usable_cores();

// The process's CPUs grouped by node: {node, cpus} for each node that has
// CPUs in the affinity mask (one group {-1, all} without NUMA information).
struct NodeCpus {
  int node;
  std::vector<int> cpus;
};
std::vector<NodeCpus> process_nodes();

// Binds the calling thread for the scope: its CPUs to node's CPUs within the
// process mask (bind_cpus) and its page placement to "prefer node"
// (bind_memory, set_mempolicy MPOL_PREFERRED).  Restores both on exit.
// node < 0, or a failing syscall, leaves that part unbound.
class NumaBind {
 public:
  NumaBind(int node, bool bind_cpus, bool bind_memory);
  ~NumaBind();
  NumaBind(const NumaBind&) = delete;
  NumaBind& operator=(const NumaBind&) = delete;
  bool cpus_bound() const { return cpus_bound_; }
  bool memory_bound() const { return mem_bound_; }

 private:
  bool cpus_bound_ = false, mem_bound_ = false;
  cpu_set_t old_cpus_;
  int old_mode_ = 0;
  unsigned long old_mask_[16] = {};
};

// Node of the page holding p (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR), or -1.
int page_node(const void* p);

}  // namespace lsbm
