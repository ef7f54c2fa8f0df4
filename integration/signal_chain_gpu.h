// Factories of the MI355X implementations of the reference's signal-chain interfaces (the declarations a srsRAN
// maintainer adds next to signal_processor_factories.h, pusch/factories.h, pdsch/factories.h and
// lower/modulation/modulation_factories.h). Each factory shares the device's srsgpu context with every object it
// creates (integration/gpu_context.h); objects are per processing thread like the reference's own components and
// stage the caller's host objects (resource grids, channel estimates, codewords, samples) through pinned memory.
#pragma once

#include "srsran/phy/lower/modulation/modulation_factories.h"
#include "srsran/phy/lower/processors/downlink/pdxch/pdxch_processor_factories.h"
#include "srsran/phy/lower/processors/uplink/puxch/puxch_processor_factories.h"
#include "srsran/phy/upper/channel_processors/pdsch/factories.h"
#include "srsran/phy/upper/channel_processors/pusch/factories.h"
#include "srsran/phy/upper/signal_processors/signal_processor_factories.h"
#include <cstdint>
#include <memory>

namespace srsran {
namespace gpu {

/// create_dmrs_pusch_estimator_factory_sw's strategy arguments (signal_processor_factories.h:74-80), as srsgpu codes.
struct pusch_estimator_options {
  uint8_t fd_smoothing   = 2;  ///< SRSGPU_CHEST_FD_*: 0 none, 1 mean, 2 filter (du_low default).
  uint8_t td_strategy    = 0;  ///< SRSGPU_CHEST_TD_*: 0 average (du_low default), 1 interpolate.
  bool    compensate_cfo = true;
};

/// create_pusch_demodulator_factory_sw's options (pusch/factories.h:92-99): the equalizer algorithm, whether an EVM
/// calculator is given, and enable_post_eq_sinr.
struct pusch_demodulator_options {
  uint8_t equalizer           = 0;  ///< SRSGPU_EQ_ZF (reference default) or SRSGPU_EQ_MMSE.
  bool    enable_evm          = true;
  bool    enable_post_eq_sinr = true;
};

/// Maps the reference's strategy enums onto pusch_estimator_options.
inline pusch_estimator_options make_pusch_estimator_options(port_channel_estimator_fd_smoothing_strategy     fd,
                                                            port_channel_estimator_td_interpolation_strategy td,
                                                            bool compensate_cfo)
{
  pusch_estimator_options o;
  o.fd_smoothing = fd == port_channel_estimator_fd_smoothing_strategy::none
                       ? 0
                       : (fd == port_channel_estimator_fd_smoothing_strategy::mean ? 1 : 2);
  o.td_strategy    = td == port_channel_estimator_td_interpolation_strategy::interpolate ? 1 : 0;
  o.compensate_cfo = compensate_cfo;
  return o;
}

} // namespace gpu

/// PUSCH DM-RS channel estimator on GPU `device` (integration/pusch_chain_gpu.cpp).
std::shared_ptr<dmrs_pusch_estimator_factory> create_dmrs_pusch_estimator_factory_gpu(int device,
                                                                                     const gpu::pusch_estimator_options& opts);

/// PUSCH demodulator on GPU `device` (integration/pusch_chain_gpu.cpp).
std::shared_ptr<pusch_demodulator_factory> create_pusch_demodulator_factory_gpu(int                                   device,
                                                                                const gpu::pusch_demodulator_options& opts);

/// PDSCH modulator on GPU `device` (integration/pdsch_chain_gpu.cpp).
std::shared_ptr<pdsch_modulator_factory> create_pdsch_modulator_factory_gpu(int device);

/// PDSCH DM-RS processor on GPU `device` (integration/pdsch_chain_gpu.cpp).
std::shared_ptr<dmrs_pdsch_processor_factory> create_dmrs_pdsch_processor_factory_gpu(int device);

/// OFDM modulator / demodulator on GPU `device` (integration/ofdm_gpu.cpp): slot objects (one launch per port and
/// slot) and symbol objects (one launch per port and symbol, synchronous: correct under the reference's own
/// pdxch_processor_impl / puxch_processor_impl, but the lower-PHY processors below are the GPU's throughput path).
std::shared_ptr<ofdm_modulator_factory>   create_ofdm_modulator_factory_gpu(int device);
std::shared_ptr<ofdm_demodulator_factory> create_ofdm_demodulator_factory_gpu(int device);

/// Lower-PHY PDxCH processor on GPU `device` (integration/lower_phy_gpu.cpp), the replacement of
/// create_pdxch_processor_factory_sw (pdxch_processor_factories.h:68; lower_phy_factory.cpp:70): each slot's grid is
/// modulated (all ports) asynchronously when the request arrives, process_symbol() hands out the symbol's samples.
std::shared_ptr<pdxch_processor_factory> create_pdxch_processor_factory_gpu(int device);

/// Lower-PHY PUxCH processor on GPU `device` (integration/lower_phy_gpu.cpp), the replacement of
/// create_puxch_processor_factory_sw (puxch_processor_factories.h:69; lower_phy_factory.cpp:84): every received symbol
/// (all ports) is demodulated by one asynchronous launch; up to `max_symbols_in_flight` symbols are outstanding before
/// process_symbol() waits. 0 (the default, the drop-in setting): each symbol is demodulated and on_rx_symbol notified
/// within its own process_symbol() call, the reference's timing (puxch_processor_impl.cpp:78). Above 0 the notification
/// of symbol l arrives during a later symbol's call (or at the end of the slot): more throughput per sector thread, but
/// an upper PHY that starts per-symbol work from on_rx_symbol sees it that much later.
std::shared_ptr<puxch_processor_factory> create_puxch_processor_factory_gpu(int device, unsigned max_symbols_in_flight = 0);

/// The sectors of one GPU as a group (integration/lower_phy_gpu.cpp). The reference runs one lower-PHY sector per cell,
/// each with its own processors driven by its own real-time thread (lib/ru/generic/ru_factory_generic_impl.cpp:75-90);
/// the processors made by a group's factories stay one per sector and keep the reference's per-sector behaviour and
/// notifications, but their OFDM work is batched: the symbols (UL) or slots (DL) the sectors submit at about the same
/// time run as ONE launch over every sector's ports, reading the samples (grids) and writing the grids (samples) in
/// place in mapped host memory. A launch goes out once every active sector has work waiting, or the gather window
/// after the oldest waiting work; no sector waits for a particular other one. Sectors batch when they share
/// numerology, cyclic prefix, DFT size (not the split sizes), bandwidth, DFT window offset and number of ports
/// (carrier frequencies may differ); a sector that cannot (or finds its staging full) runs on its own as the ungrouped
/// processors do.
struct lower_phy_group_configuration {
  int      device       = 0;
  unsigned nof_sectors  = 1;    ///< sectors of each direction the group takes (at most 32).
  unsigned ul_window_us = 50;   ///< how long a UL launch waits for active sectors still to submit.
  unsigned dl_window_us = 100;  ///< the same for DL launches (requests arrive slots ahead of transmission).
};
class lower_phy_sector_group;
std::shared_ptr<lower_phy_sector_group> create_lower_phy_sector_group(const lower_phy_group_configuration& config);
std::shared_ptr<pdxch_processor_factory> create_pdxch_processor_factory_gpu(std::shared_ptr<lower_phy_sector_group> group);
std::shared_ptr<puxch_processor_factory> create_puxch_processor_factory_gpu(std::shared_ptr<lower_phy_sector_group> group,
                                                                            unsigned max_symbols_in_flight = 0);

/// Launches a group made (UL, DL), the sector symbols / slots they ran, those that ran alone instead and the launches
/// the gather window sent (for tests and benchmarks).
struct lower_phy_group_counters {
  uint64_t ul_launches = 0, ul_batched = 0, ul_alone = 0, ul_windowed = 0;
  uint64_t dl_launches = 0, dl_batched = 0, dl_alone = 0, dl_windowed = 0;
};
lower_phy_group_counters get_lower_phy_group_counters(const lower_phy_sector_group& group);

} // namespace srsran
