// host_numa.cc -- see host_numa.h.
#include "host_numa.h"

#include <ctype.h>
#include <hip/hip_runtime_api.h>
#include <numaif.h>  // (MPOL_* constants only: the calls go through syscall(2))
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>

namespace lsbm {

namespace {
bool read_file(const std::string& path, std::string* out) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  *out = buf;
  return true;
}
}  // namespace

int pci_numa_node(const char* sysfs_root, const char* bus_id) {
  if (!bus_id || !*bus_id) return -1;
  std::string id(bus_id);
  for (char& c : id) c = (char)tolower((unsigned char)c);
  std::string s;
  if (!read_file(std::string(sysfs_root ? sysfs_root : "/sys") + "/bus/pci/devices/" + id + "/numa_node", &s))
    return -1;
  char* end = nullptr;
  const long v = strtol(s.c_str(), &end, 10);
  if (end == s.c_str() || v < 0 || v > 1023) return -1;
  return (int)v;
}

int device_numa_node(int device) {
  constexpr int kMax = 64;
  static std::atomic<int> cache[kMax];
  static std::once_flag once;
  std::call_once(once, [] {
    for (auto& c : cache) c.store(-2);
  });
  if (device < 0 || device >= kMax) return -1;
  int v = cache[device].load();
  if (v != -2) return v;
  char bus[64] = {0};
  v = -1;
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) == hipSuccess) v = pci_numa_node("/sys", bus);
  else (void)hipGetLastError();
  cache[device].store(v);
  return v;
}

bool parse_cpulist(const char* s, std::vector<int>* cpus) {
  cpus->clear();
  if (!s) return false;
  const char* p = s;
  while (*p) {
    while (*p == ' ' || *p == '\n' || *p == ',') p++;
    if (!*p) break;
    if (!isdigit((unsigned char)*p)) return false;
    char* end;
    const long a = strtol(p, &end, 10);
    long b = a;
    p = end;
    if (*p == '-') {
      p++;
      if (!isdigit((unsigned char)*p)) return false;
      b = strtol(p, &end, 10);
      p = end;
    }
    if (b < a || b > 65535) return false;
    for (long c = a; c <= b; c++) cpus->push_back((int)c);
    if (*p && *p != ',' && *p != '\n' && *p != ' ') return false;
  }
  return true;
}

bool node_cpulist(const char* sysfs_root, int node, std::vector<int>* cpus) {
  std::string s;
  if (node < 0 ||
      !read_file(std::string(sysfs_root ? sysfs_root : "/sys") + "/devices/system/node/node" +
                     std::to_string(node) + "/cpulist",
                 &s))
    return false;
  return parse_cpulist(s.c_str(), cpus);
}

std::vector<int> affinity_cpus() {
  std::vector<int> out;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return out;
  for (int c = 0; c < CPU_SETSIZE; c++)
    if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

int cgroup_cpu_quota(const char* cgroup_root) {
  const std::string root(cgroup_root ? cgroup_root : "/sys/fs/cgroup");
  std::string s;
  if (read_file(root + "/cpu.max", &s)) {  // v2: "<quota|max> <period>"
    char q[32] = {0};
    long long period = 0;
    if (sscanf(s.c_str(), "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
      const long long quota = atoll(q);
      return quota > 0 ? (int)std::max<long long>(1, quota / period) : 0;
    }
    return 0;
  }
  std::string qs, ps;  // v1
  if (read_file(root + "/cpu/cpu.cfs_quota_us", &qs) && read_file(root + "/cpu/cpu.cfs_period_us", &ps)) {
    const long long quota = atoll(qs.c_str()), period = atoll(ps.c_str());
    if (quota > 0 && period > 0) return (int)std::max<long long>(1, quota / period);
  }
  return 0;
}

namespace {
// Quota of one cgroup directory: v2 cpu.max, else v1 cfs files (0: none).
int dir_quota(const std::string& dir, bool v2) {
  std::string s;
  if (v2) {
    char q[32] = {0};
    long long period = 0;
    if (read_file(dir + "/cpu.max", &s) && sscanf(s.c_str(), "%31s %lld", q, &period) == 2 &&
        strcmp(q, "max") != 0 && period > 0 && atoll(q) > 0)
      return (int)std::max<long long>(1, atoll(q) / period);
    return 0;
  }
  std::string ps;
  if (read_file(dir + "/cpu.cfs_quota_us", &s) && read_file(dir + "/cpu.cfs_period_us", &ps)) {
    const long long quota = atoll(s.c_str()), period = atoll(ps.c_str());
    if (quota > 0 && period > 0) return (int)std::max<long long>(1, quota / period);
  }
  return 0;
}

// The smallest quota on the way from `path` (a cgroup path, "/a/b") up to the
// hierarchy's root under `mount`: a parent's limit binds its children too.
int path_quota(const std::string& mount, std::string path, bool v2) {
  int best = 0;
  for (;;) {
    while (path.size() > 1 && path.back() == '/') path.pop_back();
    const int q = dir_quota(path == "/" ? mount : mount + path, v2);
    if (q > 0) best = best ? std::min(best, q) : q;
    const size_t cut = path.rfind('/');
    if (path.empty() || path == "/" || cut == std::string::npos) break;
    path = cut == 0 ? "/" : path.substr(0, cut);
  }
  return best;
}
}  // namespace

int cgroup_cpu_quota_of(const char* cgroup_root, const char* proc_cgroup) {
  const std::string root(cgroup_root ? cgroup_root : "/sys/fs/cgroup");
  std::string v2_path, v1_path;
  bool have_v2 = false, have_v1 = false;
  const char* p = proc_cgroup ? proc_cgroup : "";
  while (*p) {  // lines "<id>:<controllers>:<path>"
    const char* eol = strchr(p, '\n');
    const std::string line(p, eol ? eol - p : strlen(p));
    p = eol ? eol + 1 : p + line.size();
    const size_t a = line.find(':'), b = a == std::string::npos ? a : line.find(':', a + 1);
    if (b == std::string::npos) continue;
    const std::string id = line.substr(0, a), ctl = line.substr(a + 1, b - a - 1), path = line.substr(b + 1);
    if (id == "0" && ctl.empty()) {
      have_v2 = true;
      v2_path = path;
      continue;
    }
    for (size_t s = 0; s <= ctl.size();) {  // v1: "cpu" among the controllers
      size_t e = ctl.find(',', s);
      if (e == std::string::npos) e = ctl.size();
      if (ctl.compare(s, e - s, "cpu") == 0) {
        have_v1 = true;
        v1_path = path;
      }
      s = e + 1;
    }
  }
  int q = 0;
  if (have_v2) q = path_quota(root, v2_path, true);
  if (!q && have_v1) {
    q = path_quota(root + "/cpu", v1_path, false);
    if (!q) q = path_quota(root + "/cpu,cpuacct", v1_path, false);
  }
  return q ? q : cgroup_cpu_quota(cgroup_root);  // (the mount root: a cgroup namespace's own)
}

int usable_cores() {
  static const int n = [] {
    if (const char* v = getenv("LSBM_HOST_THREADS")) {
      const int t = atoi(v);
      if (t > 0) return std::min(t, 1024);
    }
    int c = (int)affinity_cpus().size();
    if (c <= 0) c = (int)std::max(1L, sysconf(_SC_NPROCESSORS_ONLN));
    std::string self;
    const int q = read_file("/proc/self/cgroup", &self) ? cgroup_cpu_quota_of(nullptr, self.c_str())
                                                         : cgroup_cpu_quota(nullptr);
    return q > 0 ? std::min(c, q) : c;
  }();
  return n;
}

std::vector<NodeCpus> process_nodes() {
  const std::vector<int> mine = affinity_cpus();
  std::vector<NodeCpus> out;
  std::string online;
  std::vector<int> nodes;
  if (read_file("/sys/devices/system/node/online", &online)) parse_cpulist(online.c_str(), &nodes);
  for (int node : nodes) {
    std::vector<int> cpus;
    if (!node_cpulist("/sys", node, &cpus)) continue;
    NodeCpus nc{node, {}};
    for (int c : cpus)
      if (std::binary_search(mine.begin(), mine.end(), c)) nc.cpus.push_back(c);
    if (!nc.cpus.empty()) out.push_back(std::move(nc));
  }
  if (out.empty()) out.push_back(NodeCpus{-1, mine});
  return out;
}

NumaBind::NumaBind(int node, bool bind_cpus, bool bind_memory) {
  CPU_ZERO(&old_cpus_);
  if (node < 0 || node >= 1024) return;
  if (bind_cpus) {
    std::vector<int> cpus;
    if (node_cpulist("/sys", node, &cpus) &&
        pthread_getaffinity_np(pthread_self(), sizeof(old_cpus_), &old_cpus_) == 0) {
      cpu_set_t set;
      CPU_ZERO(&set);
      int k = 0;
      for (int c : cpus)
        if (c < CPU_SETSIZE && CPU_ISSET(c, &old_cpus_)) CPU_SET(c, &set), k++;
      cpus_bound_ = k > 0 && pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
    }
  }
  if (bind_memory) {
    const long r = syscall(SYS_get_mempolicy, &old_mode_, old_mask_, (unsigned long)(sizeof(old_mask_) * 8),
                           nullptr, 0UL);
    if (r == 0) {
      unsigned long mask[16] = {};
      mask[node / 64] = 1UL << (node % 64);
      mem_bound_ = syscall(SYS_set_mempolicy, MPOL_PREFERRED, mask, (unsigned long)(sizeof(mask) * 8)) == 0;
    }
  }
}

NumaBind::~NumaBind() {
  if (mem_bound_)
    (void)syscall(SYS_set_mempolicy, old_mode_, old_mode_ == MPOL_DEFAULT ? nullptr : old_mask_,
                  (unsigned long)(sizeof(old_mask_) * 8));
  if (cpus_bound_) (void)pthread_setaffinity_np(pthread_self(), sizeof(old_cpus_), &old_cpus_);
}

int page_node(const void* p) {
  int node = -1;
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, const_cast<void*>(p), (unsigned long)(MPOL_F_NODE | MPOL_F_ADDR)) != 0)
    return -1;
  return node;
}

}  // namespace lsbm

extern "C" {
__attribute__((visibility("default"))) int lsbm_device_numa_node(int device) {
  return lsbm::device_numa_node(device);
}
__attribute__((visibility("default"))) int lsbm_test_pci_numa_node(const char* sysfs_root, const char* bus_id) {
  return lsbm::pci_numa_node(sysfs_root, bus_id);
}
__attribute__((visibility("default"))) int lsbm_test_parse_cpulist(const char* list, int* cpus, int cap) {
  std::vector<int> v;
  if (!lsbm::parse_cpulist(list, &v)) return -1;
  for (size_t i = 0; i < v.size() && (int)i < cap; i++) cpus[i] = v[i];
  return (int)v.size();
}
__attribute__((visibility("default"))) int lsbm_test_cgroup_quota(const char* cgroup_root) {
  return lsbm::cgroup_cpu_quota(cgroup_root);
}
__attribute__((visibility("default"))) int lsbm_test_cgroup_quota_of(const char* cgroup_root,
                                                                     const char* proc_cgroup) {
  return lsbm::cgroup_cpu_quota_of(cgroup_root, proc_cgroup);
}
}  // extern "C"
