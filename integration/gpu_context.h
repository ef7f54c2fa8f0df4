// Shared pieces of the reference-side GPU bindings (integration/*.cpp): the per-device srsgpu context, owned jointly
// by every factory and by every object a factory creates, so that an object outlives the factory that made it (the
// reference's factories are routinely dropped right after create(), e.g. pusch_decoder_factory_hw, factories.cpp:122-
// 140, keeps only the accelerators it created), and the HIP error check the bindings share.
#pragma once

#include "srsgpu_phy.h"
#include <hip/hip_runtime.h>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>

namespace srsran {
namespace gpu {

/// Throws std::runtime_error naming the binding and the failed step when a HIP call fails.
inline void hip_check(hipError_t e, const char* who, const char* what)
{
  if (e != hipSuccess) {
    throw std::runtime_error(std::string(who) + ": " + what + ": " + hipGetErrorString(e));
  }
}

/// Throws std::runtime_error with the library's last error message when an srsgpu call fails.
inline void srsgpu_check(int r, const char* who)
{
  if (r != SRSGPU_OK) {
    throw std::runtime_error(std::string(who) + ": " + srsgpu_last_error());
  }
}

/// Makes the context's device current for the duration of a public entry point and restores the caller's device on
/// exit. The reference hands binding objects to arbitrary worker threads (its processor pools), whose current device
/// is whatever they used last, and a lazily grown buffer (staged_buffer::reserve, the HARQ arena) is allocated on the
/// calling thread's current device: without this, a grow on device != 0 would land on the wrong GPU.
class device_scope
{
public:
  device_scope(const srsgpu_context* ctx, const char* who)
  {
    hip_check(hipGetDevice(&prev), who, "current device");
    const int dev = srsgpu_context_device(ctx);
    if (dev != prev) {
      hip_check(hipSetDevice(dev), who, "device");
      changed = true;
    }
  }
  device_scope(const device_scope&)            = delete;
  device_scope& operator=(const device_scope&) = delete;
  ~device_scope()
  {
    if (changed) {
      (void)hipSetDevice(prev);
    }
  }

private:
  int  prev    = 0;
  bool changed = false;
};

/// The srsgpu context of `device`, one per process and device while anyone holds it: destroyed with its last owner.
inline std::shared_ptr<srsgpu_context> shared_context(int device)
{
  static std::mutex                     mtx;
  static std::weak_ptr<srsgpu_context> live[64];
  if (device < 0 || device >= 64) {
    throw std::invalid_argument("srsgpu: invalid device index " + std::to_string(device));
  }
  std::lock_guard<std::mutex> lock(mtx);
  if (std::shared_ptr<srsgpu_context> ctx = live[device].lock()) {
    return ctx;
  }
  srsgpu_context* raw = nullptr;
  srsgpu_check(srsgpu_context_create(device, &raw), "srsgpu_context_create");
  std::shared_ptr<srsgpu_context> ctx(raw, srsgpu_context_destroy);
  live[device] = ctx;
  return ctx;
}

/// Serialises the bindings' synchronous HIP set-up calls (allocations, plan creation, blocking copies) with stream
/// captures: HIP fails a synchronous call made while any thread of the process captures a stream, whatever the
/// capture mode. Held around every plan-cache miss, staging growth and graph capture (recursive: a capture path may
/// create a plan).
inline std::recursive_mutex& hip_setup_mutex()
{
  static std::recursive_mutex m;
  return m;
}

} // namespace gpu
} // namespace srsran
