// The node side of the batched externals (Part 2 of include/ziria_rx.h): one call is split
// into contiguous packet ranges, one per logical shard, and every shard runs the chunked host
// pipeline of zrx_hostio.hpp on its own device, context, copy streams and host thread.
//
//   caller arrays (host) ──┬── packets [cut[0], cut[1]) ── shard 0: ctx on GPU d0, PCIe link 0
//                          ├── packets [cut[1], cut[2]) ── shard 1: ctx on GPU d1, PCIe link 1
//                          └── ...                                                    ...
//
// Every packet is independent, so there is no exchange between shards:
// each writes its packets' outputs straight into the caller's arrays at their own indices,
// and host memory is the gather.  The reference decodes in one process from one thread
// (csrc/driver.cpp:282, wpl_go; the externals of lib/externals.blk:201-217), which is
// exactly the caller this serves: one call, all GPUs of the node behind it.
//
// Also here: the registry of caller arrays the library page-locked (hipHostRegister) because
// they come back call after call (wplc emits its arrays as static globals: the same pointer
// every call), so their copies run from the caller's memory instead of through pinned slots.
#pragma once
#include <hip/hip_runtime.h>
#include <link.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "zrx_hostio.hpp"

namespace zrx_shard {

// The calling thread's current device is restored on scope exit: the externals (and the
// context / copy-stream setup they do) must not change the caller's device as a side effect.
class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    if (dev >= 0 && dev != prev_) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev_ >= 0 && (hipGetDevice(&cur) != hipSuccess || cur != prev_)) (void)hipSetDevice(prev_);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_ = -1;
};

// Below this much input per shard a call is not spread further (a shard's fixed cost, one
// chain launch and one round trip over its link, is ~0.2 ms; 16 MiB of config-3 symbols is
// ~1100 packets, ~0.3 ms of transfer at PCIe 5.0 x16).  zrx_set_devices overrides it.
constexpr int64_t kMinShardBytes = int64_t(16) << 20;

// Contiguous packet ranges [cut[k], cut[k+1]) of nearly equal weight: packet i weighs
// prefix[i+1] - prefix[i] (bytes it brings; monotone prefix, prefix[0] = base).  Shard s
// starts at the packet boundary nearest to base + s * total / k, so every packet belongs to
// exactly one shard, the shards follow packet order and none carries more than its share
// plus one packet.  k = min(nshards, np, max(1, total / min_bytes)); no shard is empty.
template <class Prefix>
std::vector<int> split(int np, Prefix prefix, int nshards, int64_t min_bytes) {
  std::vector<int> cut{0};
  if (np <= 0) {
    cut.push_back(0);
    return cut;
  }
  const int64_t base = prefix(0), total = prefix(np) - base;
  int64_t k = std::max(1, nshards);
  k = std::min<int64_t>(k, np);
  if (min_bytes > 0) k = std::min<int64_t>(k, std::max<int64_t>(1, total / min_bytes));
  if (total == 0) {                                             // weightless packets: split by count
    for (int64_t s = 1; s < k; s++) cut.push_back((int)(np * s / k));
    cut.push_back(np);
    return cut;
  }
  int i = 0;
  for (int64_t s = 1; s < k; s++) {
    // shard s starts at the packet boundary nearest to its share, leaving at least one packet
    // for this shard and for each one after it
    const int64_t target = base + total * s / k;
    const int lo = cut.back() + 1, hi = np - (int)(k - s);
    i = std::max(i, lo);
    while (i < hi && prefix(i) < target) i++;
    if (i > lo && target - prefix(i - 1) < prefix(i) - target) i--;
    cut.push_back(std::min(std::max(i, lo), hi));
  }
  cut.push_back(np);
  return cut;
}

// Runs body(k, cut[k], cut[k + 1]) for every shard k, shard 0 on the calling thread and the
// others on the pool's threads, and merges the results: the first negative one (in shard
// order) is the call's error code, otherwise their sum (packets decoded, CRC passes, samples
// written: each body counts only its own range).  Every body has returned when this does.
template <class Body>
int run(zrx_io::Pool* pool, const std::vector<int>& cut, Body&& body) {
  const int ns = (int)cut.size() - 1;
  if (ns <= 0) return 0;
  std::vector<int64_t> rc((size_t)ns, 0);
  auto task = [&](int k) { rc[(size_t)k] = body(k, cut[(size_t)k], cut[(size_t)k + 1]); };
  if (ns == 1 || !pool) {
    for (int k = 0; k < ns; k++) task(k);
  } else {
    pool->run(ns, task);
  }
  int64_t sum = 0;
  for (int k = 0; k < ns; k++) {
    if (rc[(size_t)k] < 0) return (int)rc[(size_t)k];
    sum += rc[(size_t)k];
  }
  return (int)sum;
}

// When [p, p + n) lies in the main program's static storage -- the writable part (.data,
// .bss; past the RELRO pages the loader makes read-only) of one of its load segments, mapped
// for the whole life of the process -- returns that whole part, page-aligned, in [*s, *e).
// wplc emits a Ziria program's arrays as such globals: they come back at the same address
// every call and are never unmapped, so one registration of the segment covers all of them.
inline bool static_storage(const void* p, size_t n, uintptr_t* s_out, uintptr_t* e_out) {
  struct Q {
    uintptr_t a, b, s, e;
    bool hit;
  } q{(uintptr_t)p, (uintptr_t)p + n, 0, 0, false};
  dl_iterate_phdr(
      [](struct dl_phdr_info* info, size_t, void* d) -> int {
        Q* q = (Q*)d;
        if (info->dlpi_name && info->dlpi_name[0]) return 0;   // (the main program has no name)
        const uintptr_t pg = 4096;
        uintptr_t relro_end = 0;
        for (int i = 0; i < info->dlpi_phnum; i++) {
          const ElfW(Phdr)& ph = info->dlpi_phdr[i];
          if (ph.p_type == PT_GNU_RELRO) relro_end = info->dlpi_addr + ph.p_vaddr + ph.p_memsz;
        }
        for (int i = 0; i < info->dlpi_phnum; i++) {
          const ElfW(Phdr)& ph = info->dlpi_phdr[i];
          if (ph.p_type != PT_LOAD || !(ph.p_flags & PF_W)) continue;
          uintptr_t s = info->dlpi_addr + ph.p_vaddr;
          const uintptr_t e = (s + ph.p_memsz + pg - 1) / pg * pg;
          if (relro_end > s && relro_end < e) s = relro_end;
          s = (s + pg - 1) / pg * pg;
          if (s <= q->a && q->b <= e) {
            q->s = s;
            q->e = e;
            q->hit = true;
          }
        }
        return 1;
      },
      &q);
  *s_out = q.s;
  *e_out = q.e;
  return q.hit;
}

// Caller arrays the library page-locked (hipHostRegister, portable: every device of the node
// may DMA from them), so that their copies run from the caller's memory instead of through
// pinned slots.  ensure(p, n) says whether [p, p + n) is page-locked after the call:
//   - memory the caller pinned itself (hipHostMalloc / hipHostRegister) is used as it is;
//   - mode 1 (the default): the first array met in the main program's static storage gets
//     that storage (its .data/.bss segment) registered whole, once, for good (a wplc
//     program's arrays: same addresses every call, never unmapped);
//   - mode 2 (opt-in): any array of at least kMinRegister bytes is registered on first use;
//     the caller keeps such arrays mapped until it calls zrx_set_host_register(0), which
//     releases every registration (a page-lock must never outlive its mapping: the GPU would
//     copy through a stale translation);
//   - mode 0 (ZRX_HOST_REGISTER=0): nothing is registered.
// A failed registration is harmless (the call stages through pinned slots as before).  At most
// kMaxEntries ranges / kMaxBytes are held (least recently used go first), and a range of ours
// that a new array overlaps without containing it is dropped first.
class HostRegistry {
 public:
  static constexpr size_t kMinRegister = size_t(32) << 10;
  static constexpr int kMaxEntries = 64;
  static constexpr size_t kMaxBytes = size_t(64) << 30;

  int mode() {
    if (mode_ < 0) {
      const char* v = std::getenv("ZRX_HOST_REGISTER");
      mode_ = v && *v ? std::max(0, std::min(2, std::atoi(v))) : 1;
    }
    return mode_;
  }
  void set_mode(int m) {
    mode_ = std::max(0, std::min(2, m));
    if (mode_ != 2) {                          // (mode 2's heap ranges are the caller's to keep mapped)
      for (size_t i = 0; i < e_.size();)
        if (mode_ == 0 || !e_[i].is_static) drop(i);
        else i++;
    }
  }

  bool ensure(const void* p, size_t n, bool (*is_pinned)(const void*, size_t)) {
    if (!p || n == 0) return false;
    const uintptr_t a = (uintptr_t)p, b = a + n;
    tick_++;
    for (Entry& e : e_)
      if (e.a <= a && b <= e.b) {
        e.used = tick_;
        hits_++;
        return true;
      }
    for (size_t i = 0; i < e_.size();)
      if (e_[i].a < b && a < e_[i].b) drop(i);
      else i++;
    if (is_pinned(p, n)) return true;                           // the caller's own pinned memory
    const int m = mode();
    if (m == 0) return false;
    uintptr_t ra = a, rb = b;                                   // the range to register
    const bool st = static_storage(p, n, &ra, &rb) && rb - ra <= kMaxBytes;
    if (!st) {
      ra = a;
      rb = b;
      if (m != 2 || n < kMinRegister) return false;
    } else {
      for (size_t i = 0; i < e_.size();)                        // (arrays of this segment registered alone)
        if (e_[i].a < rb && ra < e_[i].b) drop(i);
        else i++;
    }
    n = rb - ra;
    while (!e_.empty() && ((int)e_.size() >= kMaxEntries || bytes_ + n > kMaxBytes)) {
      size_t lru = 0;
      for (size_t i = 1; i < e_.size(); i++)
        if (e_[i].used < e_[lru].used) lru = i;
      drop(lru);
    }
    if (hipHostRegister((void*)ra, n, hipHostRegisterPortable) != hipSuccess) {
      (void)hipGetLastError();
      fails_++;
      return false;
    }
    e_.push_back(Entry{ra, rb, tick_, st});
    bytes_ += n;
    registered_++;
    return true;
  }
  void release_all() {
    while (!e_.empty()) drop(e_.size() - 1);
  }
  // {mode, ranges held, bytes held, registrations made, hits, failures}
  void stats(int64_t* s6) {
    s6[0] = mode();
    s6[1] = (int64_t)e_.size();
    s6[2] = (int64_t)bytes_;
    s6[3] = registered_;
    s6[4] = hits_;
    s6[5] = fails_;
  }

 private:
  struct Entry {
    uintptr_t a, b;
    uint64_t used;
    bool is_static;
  };
  void drop(size_t i) {
    (void)hipHostUnregister((void*)e_[i].a);
    (void)hipGetLastError();
    bytes_ -= e_[i].b - e_[i].a;
    e_.erase(e_.begin() + (ptrdiff_t)i);
  }
  std::vector<Entry> e_;
  size_t bytes_ = 0;
  uint64_t tick_ = 0;
  int64_t registered_ = 0, hits_ = 0, fails_ = 0;
  int mode_ = -1;
};

// ZRX_DEVICES: a comma-separated device list ("0,1,2,3"; a device may repeat, giving it
// several logical shards) or empty / unset for every visible gfx950 device.
inline std::vector<int> parse_devices(const char* s) {
  std::vector<int> out;
  if (!s) return out;
  const char* p = s;
  while (*p) {
    while (*p == ' ' || *p == ',') p++;
    if (!*p) break;
    char* end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if (end == p) return {};                                    // malformed: the default list
    out.push_back((int)v);
    p = end;
  }
  return out;
}

}  // namespace zrx_shard
