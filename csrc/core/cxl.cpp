// CXL tier: topology, pin budget, buffer registry.
#include "ogkm/cxl.hpp"

#include <dirent.h>
#include <numaif.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>

#include "ogkm/backend.hpp"

namespace ogkm {

uint64_t system_ram_bytes() {
  long pages = sysconf(_SC_PHYS_PAGES);
  long psz = sysconf(_SC_PAGE_SIZE);
  if (pages <= 0 || psz <= 0) return 0;
  return (uint64_t)pages * (uint64_t)psz;
}

static std::string read_line(const std::string& p) {
  std::ifstream f(p);
  std::string s;
  if (f) std::getline(f, s);
  return s;
}

static std::vector<std::string> list_dir(const std::string& p) {
  std::vector<std::string> out;
  DIR* d = opendir(p.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    out.push_back(e->d_name);
  }
  closedir(d);
  return out;
}

// Link speed string -> CXL version guess (the fork's heuristic, nv-p2p.c:1556-1609,
// extended with Gen6 -> CXL 3).
static int version_from_speed(const std::string& s) {
  double gts = atof(s.c_str());
  if (gts >= 64) return 3;
  if (gts >= 32) return 2;
  if (gts >= 16) return 1;
  return 0;
}

void CxlTopology::discover(int emulate_node, const std::string& root, uint64_t emulate_mask) {
  info_ = CxlInfo{};
  node_ids_.clear();
  distances_.clear();
  {
    // SLIT: node<N>/distance lists the distances to every online node in
    // ascending node-id order.
    std::string nodes = root + "/devices/system/node";
    for (auto& name : list_dir(nodes))
      if (name.rfind("node", 0) == 0 && name.size() > 4 && isdigit((unsigned char)name[4]))
        node_ids_.push_back(atoi(name.c_str() + 4));
    std::sort(node_ids_.begin(), node_ids_.end());
    for (int nid : node_ids_) {
      std::istringstream in(read_line(nodes + "/node" + std::to_string(nid) + "/distance"));
      std::vector<int> row;
      int v;
      while (in >> v) row.push_back(v);
      if (row.size() != node_ids_.size()) row.assign(node_ids_.size(), -1);
      distances_.push_back(row);
    }
  }
  // 1) CXL memory devices on the cxl bus.
  std::string bus = root + "/bus/cxl/devices";
  for (auto& name : list_dir(bus)) {
    if (name.rfind("mem", 0) != 0) continue;
    CxlDevice d;
    d.name = name;
    std::string base = bus + "/" + name;
    std::string ram = read_line(base + "/ram/size");
    d.bytes = ram.empty() ? 0 : strtoull(ram.c_str(), nullptr, 0);
    std::string nn = read_line(base + "/numa_node");
    d.numa_node = nn.empty() ? -1 : atoi(nn.c_str());
    std::string speed = read_line(base + "/../current_link_speed");
    std::string width = read_line(base + "/../current_link_width");
    d.version = version_from_speed(speed);
    d.link_up = atoi(width.c_str()) > 0 || speed.empty();
    info_.devices.push_back(d);
  }
  // 2) CPU-less NUMA nodes with memory = CXL.mem pools onlined as system RAM.
  std::string nodes = root + "/devices/system/node";
  for (auto& name : list_dir(nodes)) {
    if (name.rfind("node", 0) != 0) continue;
    int nid = atoi(name.c_str() + 4);
    std::string cpus = read_line(nodes + "/" + name + "/cpulist");
    bool cpuless = cpus.empty();
    if (!cpuless) continue;
    std::string mi = nodes + "/" + name + "/meminfo";
    std::ifstream f(mi);
    std::string line;
    uint64_t kb = 0;
    while (std::getline(f, line))
      if (line.find("MemTotal") != std::string::npos) {
        auto pos = line.find(':');
        kb = strtoull(line.c_str() + pos + 1, nullptr, 10);
      }
    if (kb == 0) continue;
    info_.numa_nodes.push_back(nid);
    bool matched = false;
    for (auto& d : info_.devices)
      if (d.numa_node == nid) matched = true;
    if (!matched) {
      CxlDevice d;
      d.name = "numa" + std::to_string(nid);
      d.numa_node = nid;
      d.bytes = kb << 10;
      d.link_up = true;
      d.version = 2;
      info_.devices.push_back(d);
    }
  }
  // 3) Emulation: ordinary NUMA nodes stand in for CXL pools (no CXL hardware).
  if (emulate_node >= 0 && emulate_node < 64) emulate_mask |= 1ull << emulate_node;
  if (info_.numa_nodes.empty() && emulate_mask) {
    info_.emulated = true;
    for (int nid = 0; nid < 64; ++nid) {
      if (!((emulate_mask >> nid) & 1)) continue;
      info_.numa_nodes.push_back(nid);
      CxlDevice d;
      d.name = "emulated-node" + std::to_string(nid);
      d.numa_node = nid;
      d.link_up = true;
      d.version = 2;
      info_.devices.push_back(d);
    }
  }
  info_.num_devices = (uint32_t)info_.devices.size();
  info_.max_links = info_.num_devices;
  for (size_t i = 0; i < info_.devices.size() && i < 32; ++i)
    if (info_.devices[i].link_up) info_.link_mask |= 1u << i;
  info_.link_up = info_.link_mask != 0;
  info_.memory_expander = !info_.numa_nodes.empty() || !info_.devices.empty();
  for (auto& d : info_.devices) info_.cxl_version = std::max<uint32_t>(info_.cxl_version, (uint32_t)d.version);
}

int CxlTopology::distance(int from, int to) const {
  size_t i = std::find(node_ids_.begin(), node_ids_.end(), from) - node_ids_.begin();
  size_t j = std::find(node_ids_.begin(), node_ids_.end(), to) - node_ids_.begin();
  if (i >= node_ids_.size() || j >= node_ids_.size()) return -1;
  return distances_[i][j];
}

int CxlTopology::nearest_node(int from) const {
  int best = first_node(), best_d = -1;
  for (int n : info_.numa_nodes) {
    // A pool on the asking node itself is that node's DRAM (an emulated pool
    // over a CPU node): never a farther tier while another pool exists.
    if (n == from && info_.numa_nodes.size() > 1) continue;
    int d = distance(from, n);
    if (d < 0) continue;
    if (best_d < 0 || d < best_d || (d == best_d && n < best)) {
      best = n;
      best_d = d;
    }
  }
  return best;
}

bool CxlTopology::is_cxl_node(int nid) const {
  for (int n : info_.numa_nodes)
    if (n == nid) return true;
  return false;
}

// ------------------------------------------------------------------ pins
void PinTracker::init(uint64_t max_bytes, uint32_t max_buffers) {
  max_bytes_ = max_bytes;
  max_buffers_ = max_buffers;
  pinned_ = 0;
  buffers_ = 0;
}

Status PinTracker::reserve(uint64_t bytes) {
  if (buffers_ >= max_buffers_) return Status::LIMIT_EXCEEDED;
  if (pinned_ + bytes > max_bytes_ || pinned_ + bytes < pinned_) return Status::LIMIT_EXCEEDED;
  pinned_ += bytes;
  buffers_++;
  return Status::OK;
}

void PinTracker::release(uint64_t bytes) {
  pinned_ -= std::min(pinned_, bytes);
  if (buffers_) buffers_--;
}

// ------------------------------------------------------------------ registry
CxlRegistry::~CxlRegistry() {
  for (auto& b : slots_)
    if (b.handle && b.registered_with_device) be_->host_unregister((void*)b.base);
}

void CxlRegistry::init(uint64_t pin_budget, uint32_t max_buffers, uint64_t max_buffer_bytes) {
  std::lock_guard<OrderedMutex> g(m_);
  pins_.init(pin_budget, max_buffers);
  max_buffer_bytes_ = max_buffer_bytes;
  slots_.assign(max_buffers, CxlBuffer{});
  gens_.assign(max_buffers, 1);
}

// Backing of the mapping that contains `addr` (/proc/self/smaps): the kernel
// page size (hugetlbfs mappings report 2 MB / 1 GB) and the bytes of it mapped
// by transparent huge pages. Huge-page pinning is then a property
// that is measured, not a label guessed from the buffer's alignment.
static void backing_of(uint64_t addr, uint64_t* kernel_page, uint64_t* thp_bytes) {
  *kernel_page = kPageSize;
  *thp_bytes = 0;
  FILE* f = fopen("/proc/self/smaps", "r");
  if (!f) return;
  char line[512];
  bool in = false;
  while (fgets(line, sizeof line, f)) {
    unsigned long lo = 0, hi = 0;
    char c = 0;
    if (sscanf(line, "%lx-%lx %c", &lo, &hi, &c) == 3 && strchr(line, '-') < strchr(line, ' ')) {
      if (in) break;  // past the mapping
      in = addr >= lo && addr < hi;
      continue;
    }
    if (!in) continue;
    unsigned long kb = 0;
    if (sscanf(line, "KernelPageSize: %lu kB", &kb) == 1) *kernel_page = (uint64_t)kb << 10;
    else if (sscanf(line, "AnonHugePages: %lu kB", &kb) == 1 || sscanf(line, "ShmemPmdMapped: %lu kB", &kb) == 1 ||
             sscanf(line, "FilePmdMapped: %lu kB", &kb) == 1)
      *thp_bytes += (uint64_t)kb << 10;
  }
  fclose(f);
}

Status CxlRegistry::register_buffer(uint64_t base, uint64_t size, int version, uint64_t* handle) {
  if (!base || size == 0 || version < 1 || version > 3) return Status::INVALID_ARGUMENT;
  if (base + size < base) return Status::INVALID_ARGUMENT;  // overflow
  if (size > max_buffer_bytes_) return Status::LIMIT_EXCEEDED;
  if ((base & (kPageSize - 1)) || (size & (kPageSize - 1))) return Status::INVALID_ARGUMENT;
  std::lock_guard<OrderedMutex> g(m_);
  int slot = -1;
  for (size_t i = 0; i < slots_.size(); ++i) {
    if (!slots_[i].handle) {
      if (slot < 0) slot = (int)i;
    } else if (base < slots_[i].base + slots_[i].size && slots_[i].base < base + size) {
      return Status::BUSY;  // overlaps a registered buffer
    }
  }
  if (slot < 0) return Status::LIMIT_EXCEEDED;
  Status st = pins_.reserve(size);
  if (st != Status::OK) return st;
  CxlBuffer b;
  b.base = base;
  b.size = size;
  b.version = version;
  // 2 MB extents when the buffer is 2 MB aligned in address and size (A4, with
  // the page counting done in base pages, not in huge pages).
  b.page_size = ((base | size) & (kBlockSize - 1)) == 0 ? kBlockSize : kPageSize;
  backing_of(base, &b.backing_page, &b.thp_bytes);
  if (b.backing_page > kBlockSize && b.page_size == kBlockSize) b.page_size = kBlockSize;  // 1 GB pages: 2 MB extents
  int node = -1;
  if (get_mempolicy(&node, nullptr, 0, (void*)base, MPOL_F_NODE | MPOL_F_ADDR) != 0) node = -1;
  b.numa_node = node;
  // IOMMU-correct pin + device mapping (identity VA), instead of raw phys.
  st = be_->host_register((void*)base, size);
  if (st != Status::OK) {
    pins_.release(size);
    return st;
  }
  b.registered_with_device = true;
  b.extents.push_back(CxlExtent{base, size});
  b.handle = ((uint64_t)gens_[slot] << 32) | (uint64_t)(slot + 1);
  slots_[slot] = b;
  *handle = b.handle;
  RT_INFO("cxl: registered buffer %#llx size %llu ver %d page %llu (backing %llu, thp %llu B) node %d",
          (unsigned long long)base, (unsigned long long)size, version, (unsigned long long)b.page_size,
          (unsigned long long)b.backing_page, (unsigned long long)b.thp_bytes, node);
  return Status::OK;
}

Status CxlRegistry::unregister_buffer(uint64_t handle) {
  std::lock_guard<OrderedMutex> g(m_);
  uint32_t s = cxl_handle_slot(handle);
  if (s >= slots_.size() || slots_[s].handle != handle) return Status::NOT_FOUND;
  if (slots_[s].page_refs) return Status::BUSY;
  if (slots_[s].registered_with_device) be_->host_unregister((void*)slots_[s].base);
  pins_.release(slots_[s].size);
  slots_[s] = CxlBuffer{};
  gens_[s]++;
  return Status::OK;
}

Status CxlRegistry::lookup(uint64_t handle, CxlBuffer* out) {
  std::lock_guard<OrderedMutex> g(m_);
  uint32_t s = cxl_handle_slot(handle);
  if (s >= slots_.size() || slots_[s].handle != handle || !handle) return Status::NOT_FOUND;
  *out = slots_[s];
  return Status::OK;
}

Status CxlRegistry::pages(uint64_t handle, uint64_t off, uint64_t len, std::vector<CxlExtent>* out) {
  std::lock_guard<OrderedMutex> g(m_);
  uint32_t s = cxl_handle_slot(handle);
  if (s >= slots_.size() || slots_[s].handle != handle || !handle) return Status::NOT_FOUND;
  CxlBuffer& b = slots_[s];
  if (len == 0 || off > b.size || len > b.size - off) return Status::INVALID_ARGUMENT;
  out->clear();
  // Split at page_size boundaries so importers see the pinning granularity.
  uint64_t pos = off;
  while (pos < off + len) {
    uint64_t next = std::min(off + len, align_down(pos, b.page_size) + b.page_size);
    if (!out->empty() && out->back().addr + out->back().bytes == b.base + pos && out->size() > 4096) {
      out->back().bytes += next - pos;
    } else {
      out->push_back(CxlExtent{b.base + pos, next - pos});
    }
    pos = next;
  }
  b.page_refs++;
  return Status::OK;
}

Status CxlRegistry::put_pages(uint64_t handle) {
  std::lock_guard<OrderedMutex> g(m_);
  uint32_t s = cxl_handle_slot(handle);
  if (s >= slots_.size() || slots_[s].handle != handle || !handle) return Status::NOT_FOUND;
  if (!slots_[s].page_refs) return Status::INVALID_ARGUMENT;
  slots_[s].page_refs--;
  return Status::OK;
}

uint32_t CxlRegistry::count() {
  std::lock_guard<OrderedMutex> g(m_);
  return pins_.buffers();
}

}  // namespace ogkm
