// Staging and plan caching shared by the signal-chain bindings (integration/*_gpu.cpp). The reference's processors
// hand a binding host-side objects (resource grids, channel estimates, bit buffers); a binding stages what its kernel
// reads through pinned host memory into HBM, runs the cached srsgpu plan on its own stream and copies the results back
// the same way. Everything is grow-only and owned by one binding instance (one per processing thread, like the
// reference's own components), so steady state allocates nothing.
#pragma once

#include "gpu_context.h"
#include <algorithm>
#include <cstring>
#include <list>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace srsran {
namespace gpu {

/// A pinned host buffer and a device buffer of the same capacity (bytes).
class staged_buffer
{
public:
  explicit staged_buffer(const char* who_) : who(who_) {}
  staged_buffer(const staged_buffer&)            = delete;
  staged_buffer& operator=(const staged_buffer&) = delete;
  ~staged_buffer()
  {
    if (d != nullptr || h != nullptr) {
      std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());  // frees vs another thread's capture
      (void)hipFree(d);
      (void)hipHostFree(h);
    }
  }

  /// Makes room for n bytes (contents are not preserved when it grows).
  void reserve(size_t n)
  {
    if (n <= cap) {
      return;
    }
    std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());
    const size_t                          c = std::max(n, 2 * cap);
    (void)hipFree(d);
    (void)hipHostFree(h);
    d = nullptr;
    h = nullptr;
    cap = 0;
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&h), c), who, "pinned staging");
    hip_check(hipMalloc(reinterpret_cast<void**>(&d), c), who, "device buffer");
    cap = c;
  }

  template <typename T = uint8_t>
  T* host(size_t byte_offset = 0)
  {
    return reinterpret_cast<T*>(h + byte_offset);
  }
  template <typename T = uint8_t>
  T* dev(size_t byte_offset = 0)
  {
    return reinterpret_cast<T*>(d + byte_offset);
  }

  void upload(size_t offset, size_t n, hipStream_t s)
  {
    if (n != 0) {
      hip_check(hipMemcpyAsync(d + offset, h + offset, n, hipMemcpyHostToDevice, s), who, "upload");
    }
  }
  void download(size_t offset, size_t n, hipStream_t s)
  {
    if (n != 0) {
      hip_check(hipMemcpyAsync(h + offset, d + offset, n, hipMemcpyDeviceToHost, s), who, "download");
    }
  }

private:
  const char* who;
  uint8_t*    h   = nullptr;
  uint8_t*    d   = nullptr;
  size_t      cap = 0;
};

/// Pinned host memory the GPU reads and writes in place (fine-grained, mapped): zero-copy staging. A kernel that reads
/// its input from here and writes its output here replaces an upload, the kernel and a download; below a few MB the
/// DMA engines' copies cost far more than the PCIe transfer itself (profiles/r5_pcie_probe.txt: a 142 KB
/// hipMemcpyAsync takes ~70 us, a kernel reads it in place in ~5 us).
class mapped_buffer
{
public:
  explicit mapped_buffer(const char* who_) : who(who_) {}
  mapped_buffer(const mapped_buffer&)            = delete;
  mapped_buffer& operator=(const mapped_buffer&) = delete;
  ~mapped_buffer()
  {
    if (h != nullptr) {
      std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());
      (void)hipHostFree(h);
    }
  }

  /// Makes room for n bytes (contents are not preserved when it grows).
  void reserve(size_t n)
  {
    if (n <= cap) {
      return;
    }
    std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());
    const size_t                          c = std::max(n, 2 * cap);
    (void)hipHostFree(h);
    h   = nullptr;
    d   = nullptr;
    cap = 0;
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&h), c, hipHostMallocCoherent | hipHostMallocMapped), who,
              "mapped staging");
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0), who, "mapped device pointer");
    cap = c;
  }

  template <typename T = uint8_t>
  T* host(size_t byte_offset = 0)
  {
    return reinterpret_cast<T*>(h + byte_offset);
  }
  /// The same bytes as the GPU addresses them.
  template <typename T = uint8_t>
  T* dev(size_t byte_offset = 0)
  {
    return reinterpret_cast<T*>(d + byte_offset);
  }

private:
  const char* who;
  uint8_t*    h   = nullptr;
  uint8_t*    d   = nullptr;
  size_t      cap = 0;
};

/// Appends the bytes of a POD value to a cache key.
template <typename T>
void key_append(std::vector<uint8_t>& key, const T& v)
{
  const auto* p = reinterpret_cast<const uint8_t*>(&v);
  key.insert(key.end(), p, p + sizeof(T));
}

/// Most-recently-used cache of srsgpu plans keyed by their configuration bytes (a cell's grants repeat slot after
/// slot): create() runs only on a miss; the least recently used plan is destroyed beyond `capacity`. Hashed lookup: a
/// slot's key is a few kilobytes and a frame's worth of slot-dependent plans stays resident.
template <typename Plan>
class plan_cache
{
public:
  plan_cache(void (*destroy_)(Plan*), size_t capacity_ = 64) : destroy(destroy_), capacity(capacity_) {}
  plan_cache(const plan_cache&)            = delete;
  plan_cache& operator=(const plan_cache&) = delete;
  ~plan_cache() { clear(); }

  template <typename Create>
  Plan* get(const std::vector<uint8_t>& key_bytes, Create&& create)
  {
    std::string key(key_bytes.begin(), key_bytes.end());
    auto        it = index.find(key);
    if (it != index.end()) {
      lru.splice(lru.begin(), lru, it->second);
      return lru.front().plan;
    }
    Plan* plan = nullptr;
    ++nof_misses;
    {
      std::lock_guard<std::recursive_mutex> lock(hip_setup_mutex());
      plan = create();
    }
    lru.push_front({key, plan});
    index.emplace(std::move(key), lru.begin());
    if (lru.size() > capacity) {
      destroy(lru.back().plan);
      index.erase(lru.back().key);
      lru.pop_back();
      ++nof_evictions;
    }
    return plan;
  }

  /// Plans destroyed so far (a captured graph that references a plan must not outlive it).
  uint64_t evictions() const { return nof_evictions; }
  /// Plans created so far (cache misses).
  uint64_t misses() const { return nof_misses; }

  void clear()
  {
    for (auto& e : lru) {
      destroy(e.plan);
    }
    lru.clear();
    index.clear();
  }

private:
  struct entry {
    std::string key;
    Plan*       plan;
  };
  void (*destroy)(Plan*);
  size_t                                                            capacity;
  std::list<entry>                                                  lru;
  std::unordered_map<std::string, typename std::list<entry>::iterator> index;
  uint64_t                                                          nof_evictions = 0;
  uint64_t                                                          nof_misses    = 0;
};

/// A HIP stream on the context's device, destroyed with its owner.
class owned_stream
{
public:
  owned_stream(srsgpu_context* ctx, const char* who)
  {
    hip_check(hipSetDevice(srsgpu_context_device(ctx)), who, "device");
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), who, "stream");
  }
  owned_stream(const owned_stream&)            = delete;
  owned_stream& operator=(const owned_stream&) = delete;
  ~owned_stream() { (void)hipStreamDestroy(s); }
  hipStream_t get() const { return s; }

private:
  hipStream_t s = nullptr;
};

/// Host blocks page-locked and mapped for the devices (hipHostRegister), shared by the components that hand them to
/// kernels in place. The PUSCH slot batch registers its uplink processor's resource grid (the reference's
/// resource_grid_impl tensor, one [port][symbol][subcarrier] block) and reads it in place; the lower PHY's sector group
/// finds the grid here and demodulates straight into its rows. The registering component unregisters the block before
/// its memory goes away.
class host_blocks
{
public:
  /// Registers [base, base + bytes) (the caller's device is current); the device address, or nullptr on failure.
  static const void* add(const void* base, size_t bytes)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    void*                       d = nullptr;
    if (hipHostRegister(const_cast<void*>(base), bytes, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    if (hipHostGetDevicePointer(&d, const_cast<void*>(base), 0) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipHostUnregister(const_cast<void*>(base));
      return nullptr;
    }
    r.blocks[reinterpret_cast<uintptr_t>(base)] = {bytes, reinterpret_cast<uintptr_t>(d)};
    return d;
  }

  static void remove(const void* base)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    if (r.blocks.erase(reinterpret_cast<uintptr_t>(base)) != 0) {
      (void)hipHostUnregister(const_cast<void*>(base));
    }
  }

  /// The device address of p when [p, p + bytes) lies inside a registered block, else nullptr.
  static void* find(const void* p, size_t bytes)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    const auto                  a  = reinterpret_cast<uintptr_t>(p);
    auto                        it = r.blocks.upper_bound(a);
    if (it == r.blocks.begin()) {
      return nullptr;
    }
    --it;
    if (a + bytes > it->first + it->second.first) {
      return nullptr;
    }
    return reinterpret_cast<void*>(it->second.second + (a - it->first));
  }

  /// An HBM twin of a registered block (the PUSCH slot batch's HBM slot of its uplink processor's grid, same layout):
  /// a writer that fills the block from the GPU (the lower PHY's demodulation) writes the twin too and sets one bit
  /// per OFDM symbol in `symbols`; the owner, which would otherwise copy the block to its twin over PCIe, skips the
  /// copy when every symbol's bit is set, and clears them.
  struct twin {
    uint8_t*               dev     = nullptr;
    size_t                 bytes   = 0;
    std::atomic<uint32_t>* symbols = nullptr;
  };
  static void set_twin(const void* base, const twin& t)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    r.twins[reinterpret_cast<uintptr_t>(base)] = t;
  }
  static void remove_twin(const void* base)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    r.twins.erase(reinterpret_cast<uintptr_t>(base));
  }
  /// The twin of the block that starts at base, if any (dev == nullptr: none).
  static twin find_twin(const void* base)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    auto                        it = r.twins.find(reinterpret_cast<uintptr_t>(base));
    return it == r.twins.end() ? twin() : it->second;
  }

private:
  static host_blocks& get()
  {
    static host_blocks r;
    return r;
  }
  std::mutex                                                 mtx;
  std::map<uintptr_t, std::pair<size_t, uintptr_t>>          blocks;  ///< base -> (bytes, device address)
  std::map<uintptr_t, twin>                                  twins;   ///< base -> HBM twin
};

/// HBM twins of downlink resource grids (the DL counterpart of host_blocks::twin), keyed by the grid's writer: when the
/// GPU PDxCH of a sector on the same device modulates the grid (it subscribes), the PDSCH slot batch leaves its slot's
/// PDSCH REs in the twin (a device copy of its sentinel-filled scratch grid) instead of downloading them into the host
/// grid, and the PDxCH modulates every RE from the twin unless it holds the sentinel, then from the host grid (the REs
/// the CPU channels wrote): the grid's PDSCH part crosses PCIe neither way. Stream-ordered on both sides: the producer
/// waits for the consumer's last read of the twin before its copy, the consumer for the producer's copy. A publication
/// is tagged with its slot, so a consumer never takes one meant for an earlier use of the same grid.
class dl_grid_twins
{
public:
  /// A consumer on `device` modulates the grid keyed `key`, whose [port][symbol][subcarrier] image has `bytes` bytes
  /// (idempotent).
  static void subscribe(const void* key, int device, size_t bytes)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    if (r.enabled) {
      r.entries[key].device = device;
      r.entries[key].want   = bytes;
    }
  }
  static void unsubscribe(const void* key)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    auto                        it = r.entries.find(key);
    if (it != r.entries.end()) {
      it->second.device = -1;
    }
  }
  /// Tests: false makes every producer download its grid (the path the twin replaces).
  static void set_enabled(bool on)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    r.enabled = on;
  }

  /// Producer (current device `device`): the twin buffer for `key` (grown to `bytes`) after `s` waits for the
  /// consumer's last read of it; nullptr when no consumer on `device` subscribed to `key` with that image size (then
  /// the producer writes the host grid as before).
  static uint8_t* begin(const void* key, int device, size_t bytes, hipStream_t s)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    auto                        it = r.entries.find(key);
    if (!r.enabled || it == r.entries.end() || it->second.device != device || it->second.want != bytes) {
      return nullptr;
    }
    entry& e = it->second;
    if (e.bytes < bytes) {
      std::lock_guard<std::recursive_mutex> setup(hip_setup_mutex());
      if (e.dev != nullptr) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(e.dev);
        e.dev = nullptr;
      }
      if (hipMalloc(&e.dev, bytes) != hipSuccess) {
        e.dev   = nullptr;
        e.bytes = 0;
        return nullptr;
      }
      e.bytes = bytes;
      if (e.ready == nullptr) {
        (void)hipEventCreateWithFlags(&e.ready, hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&e.consumed, hipEventDisableTiming);
      }
    }
    (void)hipStreamWaitEvent(s, e.consumed, 0);
    e.pending = false;
    return e.dev;
  }
  /// Producer: the twin of `key` holds slot `slot` once `s` reaches this point.
  static void publish(const void* key, uint32_t slot, hipStream_t s)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    entry&                      e = r.entries[key];
    (void)hipEventRecord(e.ready, s);
    e.slot    = slot;
    e.pending = true;
  }
  /// Consumer: the twin of `key` for `slot` with `bytes` bytes (`s` waits for it), or nullptr. release() follows
  /// the launch that reads it.
  static const uint8_t* take(const void* key, uint32_t slot, size_t bytes, hipStream_t s)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    auto                        it = r.entries.find(key);
    if (it == r.entries.end() || !it->second.pending || it->second.slot != slot || it->second.want != bytes) {
      return nullptr;
    }
    it->second.pending = false;
    (void)hipStreamWaitEvent(s, it->second.ready, 0);
    return it->second.dev;
  }
  static void release(const void* key, hipStream_t s)
  {
    auto&                       r = get();
    std::lock_guard<std::mutex> lock(r.mtx);
    auto                        it = r.entries.find(key);
    if (it != r.entries.end()) {
      (void)hipEventRecord(it->second.consumed, s);
    }
  }

private:
  struct entry {
    int        device   = -1;  ///< the subscribed consumer's device (-1: none)
    size_t     want     = 0;   ///< the subscribed consumer's image size
    uint8_t*   dev      = nullptr;
    size_t     bytes    = 0;
    hipEvent_t ready    = nullptr;
    hipEvent_t consumed = nullptr;
    uint32_t   slot     = 0;
    bool       pending  = false;
  };
  static dl_grid_twins& get()
  {
    static dl_grid_twins r;
    return r;
  }
  std::mutex                         mtx;
  bool                               enabled = true;
  std::map<const void*, entry>       entries;
};

} // namespace gpu
} // namespace srsran
