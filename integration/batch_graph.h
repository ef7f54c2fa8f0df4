// Pieces shared by the slot batches of integration/upper_phy_gpu.cpp (DL) and integration/pusch_batch_gpu.cpp (UL):
// captured-graph helpers and the LDPC sizes of a transport block.
#pragma once

#include "gpu_staging.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc.h"

namespace srsran {
namespace gpu {

/// Capacity of the caches whose plans depend on the slot number (DM-RS sequences, and the slot graphs that run them):
/// a grant pattern repeats every frame, i.e. every 10 x 2^mu slots (40 at 60 kHz), so a few patterns of a frame stay
/// resident instead of every slot missing.
constexpr size_t SLOT_PLANS = 160;

inline void destroy_graph_exec(hipGraphExec_t x)
{
  (void)hipGraphExecDestroy(x);
}

/// Captures the queue operations `body` issues on `s` (relaxed mode; the caller holds gpu::hip_setup_mutex) into an
/// instantiated graph. A capture an error interrupts is ended, so the stream stays usable.
template <typename F>
hipGraphExec_t capture_graph(hipStream_t s, const char* who, F&& body)
{
  hip_check(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), who, "begin capture");
  struct capture_guard {
    hipStream_t s;
    bool        open = true;
    ~capture_guard()
    {
      if (open) {
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphDestroy(g);
      }
    }
  } guard{s};
  body();
  hipGraph_t g = nullptr;
  guard.open   = false;
  hip_check(hipStreamEndCapture(s, &g), who, "end capture");
  hipGraphExec_t   x = nullptr;
  const hipError_t r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  hip_check(r, who, "graph instantiate");
  return x;
}

inline uint8_t bg_number(ldpc_base_graph_type bg)
{
  return bg == ldpc_base_graph_type::BG1 ? 1 : 2;
}

/// Codeblock length N (soft bits kept for HARQ) and message bits K Z of a transport block's codeblocks.
inline void ldpc_lengths(units::bits tbs, ldpc_base_graph_type bg, unsigned& N, unsigned& KZ)
{
  const unsigned Z = ldpc::compute_lifting_size(tbs, bg, ldpc::compute_nof_codeblocks(tbs, bg));
  N                = (bg == ldpc_base_graph_type::BG1 ? 66 : 50) * Z;
  KZ               = (bg == ldpc_base_graph_type::BG1 ? 22 : 10) * Z;
}

} // namespace gpu
} // namespace srsran
