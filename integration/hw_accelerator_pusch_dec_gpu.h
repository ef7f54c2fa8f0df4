// Factories of the MI355X implementations of the reference's HAL accelerator interfaces (the headers a srsRAN
// maintainer adds next to include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_factories.h).
#pragma once

#include "srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc_factory.h"
#include "srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec_factory.h"
#include <memory>

namespace srsran {
namespace hal {

/// PUSCH decoder accelerator on GPU `device` (integration/hw_accelerator_pusch_dec_gpu.cpp). HARQ soft buffers are
/// resident in HBM for absolute codeblock identifiers 0..max_cb_ids-1 (25 KB each), one arena shared by every
/// accelerator of the factory. debug_mode: free_harq_context_entry() keeps the soft bits (the reference's
/// ext_harq_buffer_context_repository debug mode, "to enable HARQ unit testing": a retransmission after a passing TB CRC
/// still combines); otherwise a released entry combines as a new soft buffer.
std::shared_ptr<hw_accelerator_pusch_dec_factory>
create_hw_accelerator_pusch_dec_factory_gpu(int device, unsigned max_cb_ids, bool debug_mode = false);

/// PDSCH encoder accelerator on GPU `device` in transport-block mode (integration/hw_accelerator_pdsch_enc_gpu.cpp).
std::shared_ptr<hw_accelerator_pdsch_enc_factory> create_hw_accelerator_pdsch_enc_factory_gpu(int device);

} // namespace hal
} // namespace srsran
