// Host-array staging of the batched externals (Part 2 of include/ziria_rx.h).
//
// A wplc program hands __ext_wifi_rx_batch / __ext_viterbi_batch_decode plain host arrays
// ("declarable as `fun external` with arrays and scalars only"), usually
// pageable memory.  A config-3 batch is 239 MB of samples against ≈1.1 ms of kernels, so the
// copies decide what the caller sees (PCIe 5.0 x16: ≈55 GB/s, ≈4.4 ms for that batch).  The
// calls therefore cut a batch into chunks of whole packets and pipeline them:
//
//   host:   [copy chunk j+1 into pinned slot]  (pageable input only; a worker pool)
//   up:     [H2D chunk j]  [H2D chunk j+1] ...                (copy engine, own stream)
//   stream:        [chain chunk j]  [chain chunk j+1] ...     (the context's stream)
//   down:                 [D2H outputs j] ...                 (copy engine, own stream)
//   host:                        [scatter outputs j-1 to the caller] (pageable output only)
//
// so the link runs back to back and the kernels and the host copies hide under it.  A pinned
// caller buffer (hipHostMalloc / hipHostRegister, e.g. torch's pin_memory) is transferred in
// place: no host copy at all.  Two pinned slots per direction alternate; the host reuses a
// slot only after the event of its last transfer.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace zrx_io {

// Symbol bytes per chunk: large enough that a chunk's chain runs near its batch speed (a
// 2048-packet config-3 shard decodes at ≈125 Gbit/s, far above the link), small enough that
// the first upload and the last chunk's kernels and download (the pipeline's fill and drain)
// stay short.
constexpr size_t kChunkBytes = size_t(32) << 20;

// True when every byte of [p, p + n) is page-locked host memory the DMA engines can read in
// place (a hipHostMalloc'd or hipHostRegister'd allocation).  Pageable memory makes
// hipPointerGetAttributes fail; its error is cleared here.
inline bool is_pinned(const void* p, size_t n) {
  if (!p || n == 0) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (a.type != hipMemoryTypeHost) return false;
  // (the caller's array is one allocation: its last byte is locked too)
  hipPointerAttribute_t b;
  if (hipPointerGetAttributes(&b, (const uint8_t*)p + n - 1) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return b.type == hipMemoryTypeHost;
}

// A small persistent worker pool for the host-side copies (spawning threads per chunk would
// cost more than the copies).  run(n, f) calls f(i) for i in [0, n) on the workers and the
// caller, and returns when all are done.
class Pool {
 public:
  explicit Pool(int nthreads) {
    for (int t = 0; t < nthreads - 1; t++) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size() + 1; }
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (th_.empty() || n == 1) {
      for (int i = 0; i < n; i++) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      f_ = &f;
      n_ = n;
      next_.store(0);
      busy_ = (int)th_.size();
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return busy_ == 0; });
    f_ = nullptr;
  }

 private:
  void work() {
    for (int i; (i = next_.fetch_add(1)) < n_;) (*f_)(i);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* f_ = nullptr;
  int n_ = 0, busy_ = 0;
  std::atomic<int> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// memcpy of n bytes split over the pool in 1-MiB pieces
inline void par_copy(Pool& pool, void* dst, const void* src, size_t n) {
  constexpr size_t kPiece = size_t(1) << 20;
  const int pieces = (int)((n + kPiece - 1) / kPiece);
  pool.run(pieces, [&](int i) {
    const size_t a = (size_t)i * kPiece, m = std::min(kPiece, n - a);
    std::memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, m);
  });
}

// rows x width bytes between buffers of different pitches, split over the pool
inline void par_copy_2d(Pool& pool, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                        size_t rows) {
  if (rows == 0 || width == 0) return;
  const size_t per = std::max<size_t>(1, (size_t(1) << 20) / width);
  const int pieces = (int)((rows + per - 1) / per);
  pool.run(pieces, [&](int i) {
    const size_t r0 = (size_t)i * per, r1 = std::min(rows, r0 + per);
    for (size_t r = r0; r < r1; r++)
      std::memcpy((uint8_t*)dst + r * dpitch, (const uint8_t*)src + r * spitch, width);
  });
}

// Per-context state of the host pipelines: two copy streams (one per direction, so uploads
// and downloads use both link directions at once), two pinned slots per direction and the
// events that free them.
struct HostIO {
  int device = 0;
  hipStream_t up = nullptr, down = nullptr;
  uint8_t* in[2] = {nullptr, nullptr};
  uint8_t* out[2] = {nullptr, nullptr};
  size_t in_cap = 0, out_cap = 0;
  hipEvent_t up_done[2] = {nullptr, nullptr};     // slot's last upload finished (slot reusable)
  hipEvent_t down_done[2] = {nullptr, nullptr};   // slot's last download finished (outputs readable)
  hipEvent_t decoded = nullptr;                   // chunk decoded (the download waits on it)
  int32_t* flags = nullptr;                       // pinned: one plan word per chunk
  int flags_cap = 0;
  Pool* pool = nullptr;

  ~HostIO() {
    int prev = -1;
    if (hipGetDevice(&prev) == hipSuccess && prev != device) (void)hipSetDevice(device);
    else prev = -1;
    for (int s = 0; s < 2; s++) {
      if (in[s]) (void)hipHostFree(in[s]);
      if (out[s]) (void)hipHostFree(out[s]);
      if (up_done[s]) (void)hipEventDestroy(up_done[s]);
      if (down_done[s]) (void)hipEventDestroy(down_done[s]);
    }
    if (flags) (void)hipHostFree(flags);
    if (decoded) (void)hipEventDestroy(decoded);
    if (up) (void)hipStreamDestroy(up);
    if (down) (void)hipStreamDestroy(down);
    delete pool;
    if (prev >= 0) (void)hipSetDevice(prev);          // (the caller's device, as it was)
  }

  // on device `dev` (the caller's current device is left as it was), with a host pool of
  // `nthreads` threads for the pageable copies
  hipError_t init(int dev, int nthreads) {
    device = dev;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    const hipError_t e = init_on(dev, nthreads);
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    return e;
  }

  // pinned slots of at least `bytes` each (grown on demand; every slot idle when called)
  hipError_t reserve_in(size_t bytes) { return grow(in, in_cap, bytes); }
  hipError_t reserve_out(size_t bytes) { return grow(out, out_cap, bytes); }
  hipError_t reserve_flags(int n) {
    if (n <= flags_cap) return hipSuccess;
    if (flags) (void)hipHostFree(flags);
    flags = nullptr;
    flags_cap = 0;
    const hipError_t e = hipHostMalloc((void**)&flags, (size_t)std::max(n, 64) * 4, hipHostMallocDefault);
    if (e == hipSuccess) flags_cap = std::max(n, 64);
    return e;
  }

 private:
  hipError_t init_on(int dev, int nthreads) {
    hipError_t e;
    if ((e = hipSetDevice(dev)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&up, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&down, hipStreamNonBlocking)) != hipSuccess) return e;
    for (int s = 0; s < 2; s++) {
      if ((e = hipEventCreateWithFlags(&up_done[s], hipEventDisableTiming)) != hipSuccess) return e;
      if ((e = hipEventCreateWithFlags(&down_done[s], hipEventDisableTiming)) != hipSuccess) return e;
    }
    if ((e = hipEventCreateWithFlags(&decoded, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess)
      return e;
    pool = new Pool(std::max(1, nthreads));
    return hipSuccess;
  }
  static hipError_t grow(uint8_t* (&slot)[2], size_t& cap, size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    const size_t c = std::max(bytes, size_t(1) << 20);
    for (int s = 0; s < 2; s++) {
      if (slot[s]) (void)hipHostFree(slot[s]);
      slot[s] = nullptr;
    }
    cap = 0;
    for (int s = 0; s < 2; s++) {
      const hipError_t e = hipHostMalloc((void**)&slot[s], c, hipHostMallocDefault);
      if (e != hipSuccess) return e;
    }
    cap = c;
    return hipSuccess;
  }
};

// Packet ranges [cut[k], cut[k+1]) whose summed per-packet `bytes` stay near kChunkBytes
// (at least one packet per chunk); a batch under two chunks' worth is one chunk.
template <class BytesOf>
std::vector<int> chunk_cuts(int np, BytesOf bytes_of, size_t total) {
  std::vector<int> cut{0};
  if (total < 2 * kChunkBytes) {
    cut.push_back(np);
    return cut;
  }
  const int k = (int)((total + kChunkBytes - 1) / kChunkBytes);
  const size_t per = (total + k - 1) / k;
  size_t acc = 0;
  for (int i = 0; i < np; i++) {
    acc += bytes_of(i);
    if (acc >= per && i + 1 < np) {
      cut.push_back(i + 1);
      acc = 0;
    }
  }
  cut.push_back(np);
  return cut;
}

}  // namespace zrx_io
