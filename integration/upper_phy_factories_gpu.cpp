// Row b8: the GPU slot processors and channel processors behind the reference's factory interfaces. The classes here
// restate the factories of lib/phy/upper/upper_phy_factories.cpp (uplink_processor_base_factory :52-149,
// downlink_processor_single_executor_factory :153-259) and lib/phy/upper/channel_processors/pusch/factories.cpp
// (pusch_processor_factory_generic :208-270) / pdsch/factories.cpp (pdsch_processor_factory_sw :124-158), building the
// same reference processors, with the PUSCH / PDSCH work of each slot on the GPU (integration/upper_phy_gpu.h).
#include "upper_phy_gpu.h"

#include "lib/phy/upper/channel_processors/pdsch/pdsch_processor_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_processor_validator_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_processor_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_processor_validator_impl.h"
#include "lib/phy/upper/downlink_processor_single_executor_impl.h"
#include "lib/phy/upper/uplink_processor_impl.h"
#include "lib/phy/upper/upper_phy_pdu_validators.h"
#include "srsran/phy/support/resource_grid.h"
#include "srsran/srslog/srslog.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>

namespace srsran {
namespace gpu {

std::shared_ptr<pusch_gpu_service> get_pusch_gpu_service(const pusch_service_configuration& config)
{
  // One service per device and process while anything holds it (du_low's sectors on one GPU share it, which is what
  // aggregates their slots into one launch).
  static std::mutex                                    mtx;
  static std::map<int, std::weak_ptr<pusch_gpu_service>> services;
  std::lock_guard<std::mutex>                          lock(mtx);
  std::weak_ptr<pusch_gpu_service>&                    slot = services[config.device];
  std::shared_ptr<pusch_gpu_service>                   s    = slot.lock();
  if (!s) {
    s    = create_pusch_gpu_service(config);
    slot = s;
  }
  return s;
}

} // namespace gpu

namespace {

[[noreturn]] void invalid(const char* who, const std::string& what)
{
  throw std::invalid_argument(std::string(who) + ": " + what);
}

/// The HBM HARQ arena of the uplink processors that share `pool` (one sector, whichever factory made them): it is
/// indexed by the pool's absolute codeblock identifiers, so every processor of one pool must see the same soft bits.
std::shared_ptr<gpu::pusch_harq_arena> arena_for(int device, const rx_buffer_pool& pool, unsigned max_cb_ids)
{
  static std::mutex                                                                 mtx;
  static std::map<std::pair<int, const rx_buffer_pool*>, std::weak_ptr<gpu::pusch_harq_arena>> arenas;
  std::lock_guard<std::mutex>                                                       lock(mtx);
  std::weak_ptr<gpu::pusch_harq_arena>&  slot  = arenas[{device, &pool}];
  std::shared_ptr<gpu::pusch_harq_arena> arena = slot.lock();
  if (!arena) {
    arena = gpu::create_pusch_harq_arena(device, max_cb_ids);
    slot  = arena;
  }
  return arena;
}

// ---------------------------------------------------------------------------------------------------------------------
// PUSCH / PDSCH processor factories (per-PDU processors on the GPU signal chain)
// ---------------------------------------------------------------------------------------------------------------------

/// pusch_processor_factory_generic (pusch/factories.cpp:208-270) with the GPU estimator and demodulator factories.
class pusch_processor_factory_gpu : public pusch_processor_factory
{
  static constexpr const char* WHO = "pusch_processor_factory_gpu";

public:
  explicit pusch_processor_factory_gpu(const pusch_processor_factory_gpu_configuration& c) :
    decoder_factory(c.decoder_factory),
    ch_estimate_dimensions(c.ch_estimate_dimensions),
    dec_nof_iterations(c.dec_nof_iterations),
    dec_enable_early_stop(c.dec_enable_early_stop),
    csi_sinr_calc_method(c.csi_sinr_calc_method)
  {
    if (!c.demux_factory || !c.decoder_factory || !c.uci_dec_factory) {
      invalid(WHO, "invalid demultiplexer, decoder or UCI decoder factory");
    }
    if (c.max_nof_concurrent_threads == 0) {
      invalid(WHO, "at least one concurrent thread");
    }
    std::shared_ptr<dmrs_pusch_estimator_factory> est   = create_dmrs_pusch_estimator_factory_gpu(c.device, c.estimator);
    std::shared_ptr<pusch_demodulator_factory>    demod = create_pusch_demodulator_factory_gpu(c.device, c.demodulator);
    std::vector<std::unique_ptr<pusch_processor_impl::concurrent_dependencies>> deps(c.max_nof_concurrent_threads);
    for (auto& d : deps) {
      d = std::make_unique<pusch_processor_impl::concurrent_dependencies>(est->create(),
                                                                          demod->create(),
                                                                          c.demux_factory->create(),
                                                                          c.uci_dec_factory->create(),
                                                                          ch_estimate_dimensions);
    }
    dependencies_pool = std::make_shared<pusch_processor_impl::concurrent_dependencies_pool_type>(std::move(deps));
  }

  std::unique_ptr<pusch_processor> create() override
  {
    pusch_processor_impl::configuration config;
    config.thread_local_dependencies_pool = dependencies_pool;
    config.decoder                        = decoder_factory->create();
    config.dec_nof_iterations             = dec_nof_iterations;
    config.dec_enable_early_stop          = dec_enable_early_stop;
    config.csi_sinr_calc_method           = csi_sinr_calc_method;
    return std::make_unique<pusch_processor_impl>(config);
  }

  std::unique_ptr<pusch_pdu_validator> create_validator() override
  {
    return std::make_unique<pusch_processor_validator_impl>(ch_estimate_dimensions);
  }

private:
  std::shared_ptr<pusch_processor_impl::concurrent_dependencies_pool_type> dependencies_pool;
  std::shared_ptr<pusch_decoder_factory>                                   decoder_factory;
  channel_estimate::channel_estimate_dimensions                            ch_estimate_dimensions;
  unsigned                                                                 dec_nof_iterations;
  bool                                                                     dec_enable_early_stop;
  channel_state_information::sinr_type                                     csi_sinr_calc_method;
};

/// pdsch_processor_factory_sw (pdsch/factories.cpp:124-158) with the GPU modulator and DM-RS processor factories.
class pdsch_processor_factory_gpu : public pdsch_processor_factory
{
public:
  pdsch_processor_factory_gpu(int                                           device,
                              std::shared_ptr<pdsch_encoder_factory>        encoder_factory_,
                              std::shared_ptr<ptrs_pdsch_generator_factory> ptrs_factory_) :
    encoder_factory(std::move(encoder_factory_)),
    modulator_factory(create_pdsch_modulator_factory_gpu(device)),
    dmrs_factory(create_dmrs_pdsch_processor_factory_gpu(device)),
    ptrs_factory(std::move(ptrs_factory_))
  {
    if (!encoder_factory || !ptrs_factory) {
      invalid("pdsch_processor_factory_gpu", "invalid encoder or PT-RS factory");
    }
  }

  std::unique_ptr<pdsch_processor> create() override
  {
    return std::make_unique<pdsch_processor_impl>(
        encoder_factory->create(), modulator_factory->create(), dmrs_factory->create(), ptrs_factory->create());
  }

  std::unique_ptr<pdsch_pdu_validator> create_validator() override
  {
    return std::make_unique<pdsch_processor_validator_impl>();
  }

private:
  std::shared_ptr<pdsch_encoder_factory>        encoder_factory;
  std::shared_ptr<pdsch_modulator_factory>      modulator_factory;
  std::shared_ptr<dmrs_pdsch_processor_factory> dmrs_factory;
  std::shared_ptr<ptrs_pdsch_generator_factory> ptrs_factory;
};

// ---------------------------------------------------------------------------------------------------------------------
// Uplink processor factory
// ---------------------------------------------------------------------------------------------------------------------

/// uplink_processor_base_factory (upper_phy_factories.cpp:52-149) over GPU slot batches.
class uplink_processor_factory_gpu : public uplink_processor_factory
{
  static constexpr const char* WHO = "uplink_processor_factory_gpu";

public:
  explicit uplink_processor_factory_gpu(const uplink_processor_factory_gpu_configuration& c) : cfg(c)
  {
    if (!cfg.pucch_factory || !cfg.prach_factory || !cfg.srs_factory || !cfg.grid_factory || !cfg.pusch_factory ||
        !cfg.uci_dec_factory) {
      invalid(WHO, "invalid PUCCH, PRACH, SRS, resource grid, PUSCH or UCI decoder factory");
    }
    if (!cfg.pucch_executor || !cfg.pusch_executor || !cfg.srs_executor || !cfg.prach_executor) {
      invalid(WHO, "invalid task executors");
    }
    // The HARQ arena (and so the service that reads it) lives on the root device of a multi-GPU batch.
    root_device = cfg.batch.devices.empty() ? cfg.batch.device : cfg.batch.devices.front();
    if (cfg.service == nullptr) {
      gpu::pusch_service_configuration sc = cfg.service_config;
      sc.device                           = root_device;
      cfg.service                         = gpu::get_pusch_gpu_service(sc);
    }
  }

  std::unique_ptr<uplink_processor> create(const uplink_processor_config& config) override
  {
    return build(config, cfg.prach_factory->create(), cfg.pusch_factory->create(), cfg.pucch_factory->create(),
                 cfg.srs_factory->create());
  }

  std::unique_ptr<uplink_processor>
  create(const uplink_processor_config& config, srslog::basic_logger& logger, bool log_all_opportunities) override
  {
    return build(config, cfg.prach_factory->create(logger, log_all_opportunities), cfg.pusch_factory->create(logger),
                 cfg.pucch_factory->create(logger), cfg.srs_factory->create(logger));
  }

  std::unique_ptr<uplink_pdu_validator> create_pdu_validator() override
  {
    return std::make_unique<uplink_processor_validator_impl>(cfg.prach_factory->create_validator(),
                                                             cfg.pucch_factory->create_validator(),
                                                             cfg.pusch_factory->create_validator(),
                                                             cfg.srs_factory->create_validator());
  }

private:
  std::unique_ptr<uplink_processor> build(const uplink_processor_config&   config,
                                          std::unique_ptr<prach_detector>  prach,
                                          std::unique_ptr<pusch_processor> fallback,
                                          std::unique_ptr<pucch_processor> pucch,
                                          std::unique_ptr<srs_estimator>   srs)
  {
    if (!prach || !fallback || !pucch || !srs) {
      invalid(WHO, "a channel factory returned no processor");
    }
    std::unique_ptr<resource_grid> grid =
        cfg.grid_factory->create(config.nof_rx_ports, MAX_NSYMB_PER_SLOT, config.nof_rb * NOF_SUBCARRIERS_PER_RB);
    if (!grid) {
      invalid(WHO, "invalid resource grid");
    }
    std::shared_ptr<gpu::pusch_slot_batch> batch = gpu::create_pusch_slot_batch(
        cfg.batch, arena_for(root_device, config.rm_buffer_pool, cfg.batch.max_cb_ids), nullptr, cfg.uci_dec_factory, std::move(fallback), cfg.service);
    // The reference's processor posts each PUSCH PDU to its PUSCH executor (uplink_processor_impl.cpp:236): here the
    // batch's processor records it inline, and the wrapper hands the slot's PDUs to the real PUSCH executor as one job.
    uplink_processor_impl::task_executor_collection execs{*cfg.pucch_executor,
                                                          gpu::pusch_inline_executor(),
                                                          *cfg.srs_executor,
                                                          *cfg.prach_executor};
    auto impl = std::make_unique<uplink_processor_impl>(std::move(prach),
                                                        gpu::create_pusch_processor_batch_gpu(batch),
                                                        std::move(pucch),
                                                        std::move(srs),
                                                        std::move(grid),
                                                        execs,
                                                        config.rm_buffer_pool,
                                                        config.notifier,
                                                        config.nof_rb,
                                                        config.max_nof_layers);
    return gpu::create_uplink_processor_batch_gpu(std::move(impl), std::move(batch), *cfg.pusch_executor);
  }

  uplink_processor_factory_gpu_configuration cfg;
  int                                        root_device = 0;
};

// ---------------------------------------------------------------------------------------------------------------------
// Downlink processor factory
// ---------------------------------------------------------------------------------------------------------------------

/// The batching downlink processor together with the executor its inner processor was built on (the executor must
/// outlive the inner processor: declared first, destroyed last).
class downlink_processor_gpu_owner : public downlink_processor_base
{
public:
  downlink_processor_gpu_owner(std::unique_ptr<gpu::pdsch_batch_executor> exec_,
                               std::unique_ptr<downlink_processor_base>   proc_) :
    exec(std::move(exec_)), proc(std::move(proc_))
  {
  }
  downlink_processor_controller& get_controller() override { return proc->get_controller(); }
  void                           stop() override { proc->stop(); }

private:
  std::unique_ptr<gpu::pdsch_batch_executor> exec;
  std::unique_ptr<downlink_processor_base>   proc;
};

/// downlink_processor_single_executor_factory (upper_phy_factories.cpp:153-259) over a GPU PDSCH slot batch.
class downlink_processor_factory_gpu : public downlink_processor_factory
{
  static constexpr const char* WHO = "downlink_processor_factory_gpu";

public:
  explicit downlink_processor_factory_gpu(const downlink_processor_factory_gpu_configuration& c) : cfg(c)
  {
    if (!cfg.pdcch_factory || !cfg.pdsch_factory || !cfg.ssb_factory || !cfg.nzp_csi_rs_factory || !cfg.prs_factory ||
        !cfg.ptrs_factory) {
      invalid(WHO, "invalid PDCCH, PDSCH, SSB, NZP-CSI-RS, PRS or PT-RS factory");
    }
  }

  std::unique_ptr<downlink_processor_base> create(const downlink_processor_config& config) override
  {
    return build(config, cfg.pdcch_factory->create(), cfg.pdsch_factory->create(), cfg.ssb_factory->create(),
                 cfg.nzp_csi_rs_factory->create(), cfg.prs_factory->create(), srslog::fetch_basic_logger("PHY"));
  }

  std::unique_ptr<downlink_processor_base>
  create(const downlink_processor_config& config, srslog::basic_logger& logger, bool enable_broadcast) override
  {
    // As the reference: the PDCCH / PDSCH processors log every PDU, the others only with broadcast logging.
    return build(config,
                 cfg.pdcch_factory->create(logger, enable_broadcast),
                 cfg.pdsch_factory->create(logger, enable_broadcast),
                 enable_broadcast ? cfg.ssb_factory->create(logger) : cfg.ssb_factory->create(),
                 enable_broadcast ? cfg.nzp_csi_rs_factory->create(logger) : cfg.nzp_csi_rs_factory->create(),
                 enable_broadcast ? cfg.prs_factory->create(logger) : cfg.prs_factory->create(),
                 srslog::fetch_basic_logger("PHY"));
  }

  std::unique_ptr<downlink_pdu_validator> create_pdu_validator() override
  {
    return std::make_unique<downlink_processor_validator_impl>(cfg.ssb_factory->create_validator(),
                                                               cfg.pdcch_factory->create_validator(),
                                                               cfg.pdsch_factory->create_validator(),
                                                               cfg.nzp_csi_rs_factory->create_validator(),
                                                               cfg.prs_factory->create_validator());
  }

private:
  std::unique_ptr<downlink_processor_base> build(const downlink_processor_config&      config,
                                                 std::unique_ptr<pdcch_processor>      pdcch,
                                                 std::unique_ptr<pdsch_processor>      fallback,
                                                 std::unique_ptr<ssb_processor>        ssb,
                                                 std::unique_ptr<nzp_csi_rs_generator> nzp_csi,
                                                 std::unique_ptr<prs_generator>        prs,
                                                 srslog::basic_logger&                 logger)
  {
    if (!pdcch || !fallback || !ssb || !nzp_csi || !prs) {
      invalid(WHO, "a channel factory returned no processor");
    }
    if (config.gateway == nullptr || config.executor == nullptr) {
      invalid(WHO, "invalid resource grid gateway or executor");
    }
    std::shared_ptr<gpu::pdsch_slot_batch> batch =
        gpu::create_pdsch_slot_batch(gpu::pdsch_batch_configuration{cfg.device, cfg.devices}, cfg.ptrs_factory->create(),
                                     std::move(fallback));
    // The reference posts each PDSCH to its executor (downlink_processor_single_executor_impl.cpp:96-135): the batch
    // executor runs it inline while the wrapper's process_pdsch is in progress, so the batch records it.
    auto exec = std::make_unique<gpu::pdsch_batch_executor>(*config.executor);
    auto impl = std::make_unique<downlink_processor_single_executor_impl>(*config.gateway,
                                                                         std::move(pdcch),
                                                                         gpu::create_pdsch_processor_batch_gpu(batch),
                                                                         std::move(ssb),
                                                                         std::move(nzp_csi),
                                                                         std::move(prs),
                                                                         *exec,
                                                                         logger);
    auto proc = gpu::create_downlink_processor_batch_gpu(std::move(impl), std::move(batch), *config.executor);
    return std::make_unique<downlink_processor_gpu_owner>(std::move(exec), std::move(proc));
  }

  downlink_processor_factory_gpu_configuration cfg;
};

} // namespace

std::shared_ptr<pusch_processor_factory>
create_pusch_processor_factory_gpu(const pusch_processor_factory_gpu_configuration& config)
{
  return std::make_shared<pusch_processor_factory_gpu>(config);
}

std::shared_ptr<pdsch_processor_factory>
create_pdsch_processor_factory_gpu(int                                           device,
                                   std::shared_ptr<pdsch_encoder_factory>        encoder_factory,
                                   std::shared_ptr<ptrs_pdsch_generator_factory> ptrs_factory)
{
  return std::make_shared<pdsch_processor_factory_gpu>(device, std::move(encoder_factory), std::move(ptrs_factory));
}

std::shared_ptr<uplink_processor_factory>
create_uplink_processor_factory_gpu(const uplink_processor_factory_gpu_configuration& config)
{
  return std::make_shared<uplink_processor_factory_gpu>(config);
}

std::shared_ptr<downlink_processor_factory>
create_downlink_processor_factory_gpu(const downlink_processor_factory_gpu_configuration& config)
{
  return std::make_shared<downlink_processor_factory_gpu>(config);
}

} // namespace srsran
