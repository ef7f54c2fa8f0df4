// Reference-side bindings of the lower-PHY OFDM transforms (the file a srsRAN maintainer adds next to
// lib/phy/lower/modulation/): srsran::ofdm_slot_modulator / ofdm_slot_demodulator
// (include/srsran/phy/lower/modulation/ofdm_modulator.h:100, ofdm_demodulator.h:102) created by
// ofdm_modulator_factory / ofdm_demodulator_factory implementations (modulation_factories.h:92/:96) over the srsgpu
// C ABI. One plan per slot index within the subframe (the TS 38.211 section 5.4 phase compensation and the CP lengths
// depend on it), one port per call, as the reference's slot interface takes it: the port's 14 grid rows go up, the
// slot's samples come back (modulator); samples up, every subcarrier of every symbol of the port back into the grid
// through resource_grid_writer::put (demodulator, ofdm_demodulator_impl.cpp:128-134).
//
// Symbol objects (ofdm_symbol_modulator / _demodulator, ofdm_modulator.h:58, ofdm_demodulator.h:59): one plan per
// symbol of the subframe (one port), one synchronous launch per call. They make the reference's own
// pdxch_processor_impl / puxch_processor_impl run on the GPU unchanged; the throughput path of the lower PHY is the
// slot-granular pdxch / puxch processors of integration/lower_phy_gpu.cpp.
#include "signal_chain_gpu.h"

#include "gpu_staging.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/support/resource_grid_writer.h"

#include <map>
#include <stdexcept>
#include <string>

namespace srsran {

namespace {

/// The plans of one OFDM configuration, one per slot index within the subframe, created on first use.
class ofdm_plans
{
public:
  ofdm_plans(srsgpu_context* ctx_, const srsgpu_ofdm_config& cfg_, bool modulator_, const char* who_) :
    ctx(ctx_), cfg(cfg_), modulator(modulator_), who(who_)
  {
  }
  ofdm_plans(const ofdm_plans&)            = delete;
  ofdm_plans& operator=(const ofdm_plans&) = delete;
  ~ofdm_plans()
  {
    for (auto& e : plans) {
      srsgpu_ofdm_plan_destroy(e.second);
    }
  }

  srsgpu_ofdm_plan* get(unsigned slot_index)
  {
    auto it = plans.find(slot_index);
    if (it != plans.end()) {
      return it->second;
    }
    srsgpu_ofdm_plan* p = nullptr;
    const uint32_t    s = slot_index;
    gpu::srsgpu_check(modulator ? srsgpu_ofdm_modulator_plan_create(ctx, &cfg, 1, 1, &s, &p)
                                : srsgpu_ofdm_demodulator_plan_create(ctx, &cfg, 1, 1, &s, &p),
                      who);
    plans.emplace(slot_index, p);
    return p;
  }

  unsigned nof_symbols() const { return cfg.cp_extended ? 12 : 14; }

private:
  srsgpu_context*                        ctx;
  srsgpu_ofdm_config                     cfg;
  bool                                   modulator;
  const char*                            who;
  std::map<unsigned, srsgpu_ofdm_plan*>  plans;
};

srsgpu_ofdm_config to_srsgpu(unsigned numerology, unsigned bw_rb, unsigned dft_size, cyclic_prefix cp,
                             unsigned window_offset, float scale, double center_freq_hz)
{
  srsgpu_ofdm_config c;
  std::memset(&c, 0, sizeof(c));
  c.numerology                = numerology;
  c.bw_rb                     = bw_rb;
  c.dft_size                  = dft_size;
  c.cp_extended               = (cp == cyclic_prefix::EXTENDED) ? 1 : 0;
  c.nof_samples_window_offset = window_offset;
  c.scale                     = scale;
  c.center_freq_hz            = center_freq_hz;
  return c;
}

class ofdm_slot_modulator_gpu : public ofdm_slot_modulator
{
  static constexpr const char* WHO = "ofdm_slot_modulator_gpu";

public:
  ofdm_slot_modulator_gpu(std::shared_ptr<srsgpu_context> owner_, const ofdm_modulator_configuration& config) :
    owner(std::move(owner_)),
    stream(owner.get(), WHO),
    plans(owner.get(),
          to_srsgpu(config.numerology, config.bw_rb, config.dft_size, config.cp, 0, config.scale, config.center_freq_hz),
          true,
          WHO),
    nsc(config.bw_rb * NRE),
    grid_buf(WHO),
    out_buf(WHO)
  {
    (void)plans.get(0);  // validates the configuration now (the reference asserts in the constructor)
  }

  unsigned get_slot_size(unsigned slot_index) const override
  {
    return static_cast<unsigned>(srsgpu_ofdm_plan_nof_samples(const_cast<ofdm_plans&>(plans).get(slot_index)));
  }

  void modulate(span<cf_t> output, const resource_grid_reader& grid, unsigned port_index, unsigned slot_index) override
  {
    gpu::device_scope dev_scope(owner.get(), WHO);
    srsgpu_ofdm_plan* plan = plans.get(slot_index);
    const size_t      n    = srsgpu_ofdm_plan_nof_samples(plan);
    if (output.size() != n) {
      throw std::invalid_argument(std::string(WHO) + ": output of " + std::to_string(output.size()) +
                                  " samples for a slot of " + std::to_string(n));
    }
    // An empty port modulates to zeros (ofdm_modulator_impl.cpp:77).
    if (grid.is_empty(port_index)) {
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    const unsigned nsymb = plans.nof_symbols();
    const size_t   row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    hipStream_t    s     = stream.get();
    grid_buf.reserve(nsymb * row);
    for (unsigned l = 0; l != nsymb; ++l) {
      std::memcpy(grid_buf.host(l * row), grid.get_view(port_index, l).data(), row);
    }
    grid_buf.upload(0, nsymb * row, s);
    out_buf.reserve(n * sizeof(cf_t));
    gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_execute(plan, grid_buf.dev<uint32_t>(), out_buf.dev<float>(), s), WHO);
    out_buf.download(0, n * sizeof(cf_t), s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");
    std::memcpy(output.data(), out_buf.host(), n * sizeof(cf_t));
  }

private:
  std::shared_ptr<srsgpu_context> owner;
  gpu::owned_stream               stream;
  ofdm_plans                      plans;
  unsigned                        nsc;
  gpu::staged_buffer              grid_buf;
  gpu::staged_buffer              out_buf;
};

class ofdm_slot_demodulator_gpu : public ofdm_slot_demodulator
{
  static constexpr const char* WHO = "ofdm_slot_demodulator_gpu";

public:
  ofdm_slot_demodulator_gpu(std::shared_ptr<srsgpu_context> owner_, const ofdm_demodulator_configuration& config) :
    owner(std::move(owner_)),
    stream(owner.get(), WHO),
    plans(owner.get(),
          to_srsgpu(config.numerology,
                    config.bw_rb,
                    config.dft_size,
                    config.cp,
                    config.nof_samples_window_offset,
                    config.scale,
                    config.center_freq_hz),
          false,
          WHO),
    nsc(config.bw_rb * NRE),
    in_buf(WHO),
    grid_buf(WHO)
  {
    (void)plans.get(0);
  }

  unsigned get_slot_size(unsigned slot_index) const override
  {
    return static_cast<unsigned>(srsgpu_ofdm_plan_nof_samples(const_cast<ofdm_plans&>(plans).get(slot_index)));
  }

  void demodulate(resource_grid_writer& grid, span<const cf_t> input, unsigned port_index, unsigned slot_index) override
  {
    gpu::device_scope dev_scope(owner.get(), WHO);
    srsgpu_ofdm_plan* plan = plans.get(slot_index);
    const size_t      n    = srsgpu_ofdm_plan_nof_samples(plan);
    if (input.size() != n) {
      throw std::invalid_argument(std::string(WHO) + ": input of " + std::to_string(input.size()) +
                                  " samples for a slot of " + std::to_string(n));
    }
    const unsigned nsymb = plans.nof_symbols();
    const size_t   row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    hipStream_t    s     = stream.get();
    in_buf.reserve(n * sizeof(cf_t));
    std::memcpy(in_buf.host(), input.data(), n * sizeof(cf_t));
    in_buf.upload(0, n * sizeof(cf_t), s);
    grid_buf.reserve(nsymb * row);
    gpu::srsgpu_check(srsgpu_ofdm_demodulator_plan_execute(plan, in_buf.dev<float>(), grid_buf.dev<uint32_t>(), s), WHO);
    grid_buf.download(0, nsymb * row, s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");
    for (unsigned l = 0; l != nsymb; ++l) {
      grid.put(port_index, l, 0, 1, span<const cbf16_t>(grid_buf.host<cbf16_t>(l * row), nsc));
    }
  }

private:
  std::shared_ptr<srsgpu_context> owner;
  gpu::owned_stream               stream;
  ofdm_plans                      plans;
  unsigned                        nsc;
  gpu::staged_buffer              in_buf;
  gpu::staged_buffer              grid_buf;
};

/// The single-symbol plans (one port) of one OFDM configuration, created on first use per symbol of the subframe.
class ofdm_symbol_plans
{
public:
  ofdm_symbol_plans(srsgpu_context* ctx_, const srsgpu_ofdm_config& cfg_, bool modulator_, const char* who_) :
    ctx(ctx_), cfg(cfg_), modulator(modulator_), who(who_)
  {
  }
  ofdm_symbol_plans(const ofdm_symbol_plans&)            = delete;
  ofdm_symbol_plans& operator=(const ofdm_symbol_plans&) = delete;
  ~ofdm_symbol_plans()
  {
    for (auto& e : plans) {
      srsgpu_ofdm_plan_destroy(e.second);
    }
  }

  unsigned nof_symbols() const { return cfg.cp_extended ? 12 : 14; }

  srsgpu_ofdm_plan* get(unsigned symbol_index)
  {
    auto it = plans.find(symbol_index);
    if (it != plans.end()) {
      return it->second;
    }
    srsgpu_ofdm_plan* p    = nullptr;
    const uint32_t    slot = symbol_index / nof_symbols();
    const uint32_t    l    = symbol_index % nof_symbols();
    gpu::srsgpu_check(modulator ? srsgpu_ofdm_modulator_symbols_plan_create(ctx, &cfg, 1, slot, l, 1, &p)
                                : srsgpu_ofdm_demodulator_symbols_plan_create(ctx, &cfg, 1, slot, l, 1, &p),
                      who);
    plans.emplace(symbol_index, p);
    return p;
  }

private:
  srsgpu_context*                       ctx;
  srsgpu_ofdm_config                    cfg;
  bool                                  modulator;
  const char*                           who;
  std::map<unsigned, srsgpu_ofdm_plan*> plans;
};

class ofdm_symbol_modulator_gpu : public ofdm_symbol_modulator
{
  static constexpr const char* WHO = "ofdm_symbol_modulator_gpu";

public:
  ofdm_symbol_modulator_gpu(std::shared_ptr<srsgpu_context> owner_, const ofdm_modulator_configuration& config) :
    owner(std::move(owner_)),
    stream(owner.get(), WHO),
    plans(owner.get(),
          to_srsgpu(config.numerology, config.bw_rb, config.dft_size, config.cp, 0, config.scale, config.center_freq_hz),
          true,
          WHO),
    nsc(config.bw_rb * NRE),
    grid_buf(WHO),
    out_buf(WHO)
  {
    gpu::device_scope dev_scope(owner.get(), WHO);
    (void)plans.get(0);  // validates the configuration now (the reference asserts in the constructor)
  }

  unsigned get_symbol_size(unsigned symbol_index) const override
  {
    return static_cast<unsigned>(srsgpu_ofdm_plan_nof_samples(const_cast<ofdm_symbol_plans&>(plans).get(symbol_index)));
  }

  void modulate(span<cf_t> output, const resource_grid_reader& grid, unsigned port_index, unsigned symbol_index) override
  {
    gpu::device_scope dev_scope(owner.get(), WHO);
    srsgpu_ofdm_plan* plan = plans.get(symbol_index);
    const size_t      n    = srsgpu_ofdm_plan_nof_samples(plan);
    if (output.size() != n) {
      throw std::invalid_argument(std::string(WHO) + ": output of " + std::to_string(output.size()) +
                                  " samples for a symbol of " + std::to_string(n));
    }
    if (grid.is_empty(port_index)) {  // ofdm_modulator_impl.cpp:77
      std::fill(output.begin(), output.end(), cf_t());
      return;
    }
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
    hipStream_t  s   = stream.get();
    grid_buf.reserve(row);
    std::memcpy(grid_buf.host(), grid.get_view(port_index, symbol_index % plans.nof_symbols()).data(), row);
    grid_buf.upload(0, row, s);
    out_buf.reserve(n * sizeof(cf_t));
    gpu::srsgpu_check(srsgpu_ofdm_modulator_plan_execute(plan, grid_buf.dev<uint32_t>(), out_buf.dev<float>(), s), WHO);
    out_buf.download(0, n * sizeof(cf_t), s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");
    std::memcpy(output.data(), out_buf.host(), n * sizeof(cf_t));
  }

private:
  std::shared_ptr<srsgpu_context> owner;
  gpu::owned_stream               stream;
  ofdm_symbol_plans               plans;
  unsigned                        nsc;
  gpu::staged_buffer              grid_buf;
  gpu::staged_buffer              out_buf;
};

class ofdm_symbol_demodulator_gpu : public ofdm_symbol_demodulator
{
  static constexpr const char* WHO = "ofdm_symbol_demodulator_gpu";

public:
  ofdm_symbol_demodulator_gpu(std::shared_ptr<srsgpu_context> owner_, const ofdm_demodulator_configuration& config) :
    owner(std::move(owner_)),
    stream(owner.get(), WHO),
    plans(owner.get(),
          to_srsgpu(config.numerology,
                    config.bw_rb,
                    config.dft_size,
                    config.cp,
                    config.nof_samples_window_offset,
                    config.scale,
                    config.center_freq_hz),
          false,
          WHO),
    nsc(config.bw_rb * NRE),
    in_buf(WHO),
    grid_buf(WHO)
  {
    gpu::device_scope dev_scope(owner.get(), WHO);
    (void)plans.get(0);
  }

  unsigned get_symbol_size(unsigned symbol_index) const override
  {
    return static_cast<unsigned>(srsgpu_ofdm_plan_nof_samples(const_cast<ofdm_symbol_plans&>(plans).get(symbol_index)));
  }

  void demodulate(resource_grid_writer& grid, span<const cf_t> input, unsigned port_index, unsigned symbol_index) override
  {
    gpu::device_scope dev_scope(owner.get(), WHO);
    srsgpu_ofdm_plan* plan = plans.get(symbol_index);
    const size_t      n    = srsgpu_ofdm_plan_nof_samples(plan);
    if (input.size() != n) {
      throw std::invalid_argument(std::string(WHO) + ": input of " + std::to_string(input.size()) +
                                  " samples for a symbol of " + std::to_string(n));
    }
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
    hipStream_t  s   = stream.get();
    in_buf.reserve(n * sizeof(cf_t));
    std::memcpy(in_buf.host(), input.data(), n * sizeof(cf_t));
    in_buf.upload(0, n * sizeof(cf_t), s);
    grid_buf.reserve(row);
    gpu::srsgpu_check(srsgpu_ofdm_demodulator_plan_execute(plan, in_buf.dev<float>(), grid_buf.dev<uint32_t>(), s), WHO);
    grid_buf.download(0, row, s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");
    grid.put(port_index, symbol_index % plans.nof_symbols(), 0, 1, span<const cbf16_t>(grid_buf.host<cbf16_t>(), nsc));
  }

private:
  std::shared_ptr<srsgpu_context> owner;
  gpu::owned_stream               stream;
  ofdm_symbol_plans               plans;
  unsigned                        nsc;
  gpu::staged_buffer              in_buf;
  gpu::staged_buffer              grid_buf;
};

class ofdm_modulator_factory_gpu : public ofdm_modulator_factory
{
public:
  explicit ofdm_modulator_factory_gpu(int device) : ctx(gpu::shared_context(device)) {}
  std::unique_ptr<ofdm_symbol_modulator> create_ofdm_symbol_modulator(const ofdm_modulator_configuration& config) override
  {
    return std::make_unique<ofdm_symbol_modulator_gpu>(ctx, config);
  }
  std::unique_ptr<ofdm_slot_modulator> create_ofdm_slot_modulator(const ofdm_modulator_configuration& config) override
  {
    return std::make_unique<ofdm_slot_modulator_gpu>(ctx, config);
  }

private:
  std::shared_ptr<srsgpu_context> ctx;
};

class ofdm_demodulator_factory_gpu : public ofdm_demodulator_factory
{
public:
  explicit ofdm_demodulator_factory_gpu(int device) : ctx(gpu::shared_context(device)) {}
  std::unique_ptr<ofdm_symbol_demodulator>
  create_ofdm_symbol_demodulator(const ofdm_demodulator_configuration& config) override
  {
    return std::make_unique<ofdm_symbol_demodulator_gpu>(ctx, config);
  }
  std::unique_ptr<ofdm_slot_demodulator> create_ofdm_slot_demodulator(const ofdm_demodulator_configuration& config) override
  {
    return std::make_unique<ofdm_slot_demodulator_gpu>(ctx, config);
  }

private:
  std::shared_ptr<srsgpu_context> ctx;
};

} // namespace

std::shared_ptr<ofdm_modulator_factory> create_ofdm_modulator_factory_gpu(int device)
{
  return std::make_shared<ofdm_modulator_factory_gpu>(device);
}

std::shared_ptr<ofdm_demodulator_factory> create_ofdm_demodulator_factory_gpu(int device)
{
  return std::make_shared<ofdm_demodulator_factory_gpu>(device);
}

} // namespace srsran
