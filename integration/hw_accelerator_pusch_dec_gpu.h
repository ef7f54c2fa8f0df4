// Factories of the MI355X implementations of the reference's HAL accelerator interfaces (the headers a srsRAN
// maintainer adds next to include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_factories.h).
#pragma once

#include "srsran/hal/phy/upper/channel_processors/hw_accelerator_pdsch_enc_factory.h"
#include "srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec_factory.h"
#include <memory>

namespace srsran {
namespace hal {

/// PUSCH decoder accelerator on GPU `device` (integration/hw_accelerator_pusch_dec_gpu.cpp). HARQ soft buffers are
/// resident in HBM for absolute codeblock identifiers 0..max_cb_ids-1 (25 KB each).
std::shared_ptr<hw_accelerator_pusch_dec_factory> create_hw_accelerator_pusch_dec_factory_gpu(int      device,
                                                                                              unsigned max_cb_ids);

/// PDSCH encoder accelerator on GPU `device` in transport-block mode (integration/hw_accelerator_pdsch_enc_gpu.cpp).
std::shared_ptr<hw_accelerator_pdsch_enc_factory> create_hw_accelerator_pdsch_enc_factory_gpu(int device);

} // namespace hal
} // namespace srsran
