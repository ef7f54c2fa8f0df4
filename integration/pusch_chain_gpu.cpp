// Reference-side bindings of the PUSCH signal chain (the files a srsRAN maintainer adds next to
// lib/phy/upper/signal_processors/ and lib/phy/upper/channel_processors/pusch/): srsran::dmrs_pusch_estimator
// (include/srsran/phy/upper/signal_processors/dmrs_pusch_estimator.h:100) and srsran::pusch_demodulator
// (include/srsran/phy/upper/channel_processors/pusch/pusch_demodulator.h:95) over the srsgpu C ABI, created by
// dmrs_pusch_estimator_factory / pusch_demodulator_factory implementations, so that the reference's own
// pusch_processor_impl (pusch_processor_impl.cpp:217 estimate, :335 demodulate), wired by upper_phy_factories.cpp:432-609,
// runs its channel estimation and demodulation on an MI355X.
//
// Data path per call: the rows the kernel reads are staged from the caller's resource grid / channel estimate (host
// objects of the reference: resource_grid_reader::get_view, channel_estimate::get_symbol_ch_estimate) through pinned
// memory into HBM, the cached plan runs on the binding's stream, and the results come back into the reference's
// objects: the estimator writes the allocated REs of every symbol / port / layer of the channel_estimate and its
// noise variance, RSRP, EPRE, SNR, time alignment and CFO (dmrs_pusch_estimator_impl.cpp:45 resize, port_channel_
// estimator_average_impl.cpp:140-151); the demodulator feeds the codeword buffer block by block with the descrambled
// LLRs and the scrambling sequence, and notifies the per-symbol and end statistics in the reference's order
// (pusch_demodulator_impl.cpp:272-443).
#include "signal_chain_gpu.h"

#include "chain_convert.h"
#include "gpu_staging.h"
#include "srsran/phy/support/resource_grid_reader.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_codeword_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_demodulator_notifier.h"
#include "srsran/srsvec/bit.h"

#include <cmath>
#include <limits>
#include <stdexcept>
#include <string>

namespace srsran {

namespace {

using gpu::crb_alloc;

// --------------------------------------------------------------------------------------------------------------------
// DM-RS PUSCH channel estimator
// --------------------------------------------------------------------------------------------------------------------

class dmrs_pusch_estimator_gpu : public dmrs_pusch_estimator
{
  static constexpr const char* WHO = "dmrs_pusch_estimator_gpu";

public:
  dmrs_pusch_estimator_gpu(std::shared_ptr<srsgpu_context> owner_, const gpu::pusch_estimator_options& opts_) :
    owner(std::move(owner_)),
    ctx(owner.get()),
    opts(opts_),
    stream(ctx, WHO),
    plans(srsgpu_pusch_chest_plan_destroy),
    grid_buf(WHO),
    ce_buf(WHO),
    stat_buf(WHO)
  {
  }

  void estimate(channel_estimate& estimate, const resource_grid_reader& grid, const configuration& config) override
  {
    gpu::device_scope dev_scope(ctx, WHO);
    const unsigned              nsc      = grid.get_nof_subc();
    const unsigned              grid_prb = nsc / NRE;
    const gpu::pusch_chest_desc d        = gpu::make_pusch_chest_desc(config, grid_prb, opts, SRSGPU_CE_PER_SYMBOL, WHO);
    const srsgpu_pusch_chest_config& c   = d.c;
    const crb_alloc&                 a   = d.alloc;
    const unsigned                   P   = d.nof_ports;
    const unsigned                   L   = d.nof_layers;

    std::vector<uint8_t> key;
    d.append_key(key);
    gpu::key_append(key, grid_prb);
    srsgpu_pusch_chest_plan* plan = plans.get(key, [&] {
      const srsgpu_alloc_ext   ext = d.ext();
      srsgpu_pusch_chest_plan* p   = nullptr;
      gpu::srsgpu_check(srsgpu_pusch_chest_plan_create_ex(ctx, &c, &ext, 1, grid_prb, P, &p), WHO);
      return p;
    });

    // Rx grid: the DM-RS symbols of every rx port, [port][symbol][subcarrier] (the plan's grid layout).
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
    grid_buf.reserve(P * 14 * row);
    hipStream_t s = stream.get();
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = 0; l != 14; ++l) {
        if ((c.dmrs_symbol_mask >> l) & 1u) {
          span<const cbf16_t> v = grid.get_view(config.rx_ports[p], l);
          std::memcpy(grid_buf.host((p * 14 + l) * row), v.data(), row);
          grid_buf.upload((p * 14 + l) * row, row, s);
        }
      }
    }
    // Estimates [layer][port][symbol][subcarrier], noise variances [port], metrics [port][SRSGPU_CHEST_METRICS].
    const size_t ce_bytes = static_cast<size_t>(L) * P * 14 * row;
    ce_buf.reserve(static_cast<size_t>(4) * P * 14 * row);
    stat_buf.reserve(sizeof(float) * (4 + 4 * SRSGPU_CHEST_METRICS));
    gpu::srsgpu_check(srsgpu_pusch_chest_plan_execute(plan, grid_buf.dev<uint32_t>(), ce_buf.dev<uint32_t>(),
                                                      stat_buf.dev<float>(), stat_buf.dev<float>(4 * sizeof(float)),
                                                      s),
                      WHO);
    // The allocated subcarriers of every row (one 2D copy), and the statistics.
    const size_t col0 = static_cast<size_t>(a.rb_start) * NRE * sizeof(uint32_t);
    const size_t cols = static_cast<size_t>(a.span_end - a.rb_start) * NRE * sizeof(uint32_t);
    gpu::hip_check(hipMemcpy2DAsync(ce_buf.host(col0), row, ce_buf.dev(col0), row, cols, ce_bytes / row,
                                    hipMemcpyDeviceToHost, s),
                   WHO, "estimate download");
    stat_buf.download(0, sizeof(float) * (4 + 4 * SRSGPU_CHEST_METRICS), s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");

    // Into the reference's channel estimate (dimensions as dmrs_pusch_estimator_impl.cpp:45 sets them).
    estimate.resize({static_cast<unsigned>(config.rb_mask.size()), config.first_symbol + config.nof_symbols, P, L});
    const float* nv = stat_buf.host<float>();
    const float* m  = stat_buf.host<float>(4 * sizeof(float));
    for (unsigned ly = 0; ly != L; ++ly) {
      for (unsigned p = 0; p != P; ++p) {
        for (unsigned l = config.first_symbol; l != config.first_symbol + config.nof_symbols; ++l) {
          span<cbf16_t> dst   = estimate.get_symbol_ch_estimate(l, p, ly);
          const size_t  k0    = static_cast<size_t>(a.rb_start) * NRE;
          const size_t  n     = std::min<size_t>(dst.size(), static_cast<size_t>(a.span_end) * NRE) - k0;
          const auto*   src   = ce_buf.host<uint32_t>(((static_cast<size_t>(ly) * P + p) * 14 + l) * row);
          if (a.mask.empty()) {
            std::memcpy(dst.data() + k0, src + k0, n * sizeof(uint32_t));
          } else {
            for (unsigned rb = a.rb_start; rb != a.span_end; ++rb) {
              if (a.mask[rb] != 0 && (rb + 1) * NRE <= dst.size()) {
                std::memcpy(dst.data() + rb * NRE, src + rb * NRE, NRE * sizeof(uint32_t));
              }
            }
          }
        }
      }
    }
    gpu::write_chest_metrics(estimate, nv, m, P, L);
  }

private:
  std::shared_ptr<srsgpu_context>           owner;
  srsgpu_context*                           ctx;
  gpu::pusch_estimator_options              opts;
  gpu::owned_stream                         stream;
  gpu::plan_cache<srsgpu_pusch_chest_plan>  plans;
  gpu::staged_buffer                        grid_buf;
  gpu::staged_buffer                        ce_buf;
  gpu::staged_buffer                        stat_buf;
};

class dmrs_pusch_estimator_factory_gpu : public dmrs_pusch_estimator_factory
{
public:
  dmrs_pusch_estimator_factory_gpu(int device, const gpu::pusch_estimator_options& opts_) :
    ctx(gpu::shared_context(device)), opts(opts_)
  {
  }
  std::unique_ptr<dmrs_pusch_estimator> create() override
  {
    return std::make_unique<dmrs_pusch_estimator_gpu>(ctx, opts);
  }

private:
  std::shared_ptr<srsgpu_context> ctx;
  gpu::pusch_estimator_options    opts;
};

// --------------------------------------------------------------------------------------------------------------------
// PUSCH demodulator
// --------------------------------------------------------------------------------------------------------------------

class pusch_demodulator_gpu : public pusch_demodulator
{
  static constexpr const char* WHO = "pusch_demodulator_gpu";

public:
  pusch_demodulator_gpu(std::shared_ptr<srsgpu_context> owner_, const gpu::pusch_demodulator_options& opts_) :
    owner(std::move(owner_)),
    ctx(owner.get()),
    opts(opts_),
    stream(ctx, WHO),
    plans(srsgpu_pusch_demodulator_plan_destroy),
    grid_buf(WHO),
    ce_buf(WHO),
    out_buf(WHO)
  {
  }

  void demodulate(pusch_codeword_buffer&      codeword_buffer,
                  pusch_demodulator_notifier& notifier,
                  const resource_grid_reader& grid,
                  const channel_estimate&     estimates,
                  const configuration&        config) override
  {
    gpu::device_scope dev_scope(ctx, WHO);
    const unsigned              nsc      = grid.get_nof_subc();
    const unsigned              grid_prb = nsc / NRE;
    const gpu::pusch_demod_desc d        = gpu::make_pusch_demod_desc(config, grid_prb, opts, SRSGPU_CE_PER_SYMBOL, WHO);
    const srsgpu_pusch_demod_config& c   = d.c;
    const crb_alloc&                 a   = d.alloc;
    const unsigned                   P   = d.nof_ports;
    const unsigned                   L   = d.nof_layers;

    std::vector<uint8_t> key;
    d.append_key(key);
    gpu::key_append(key, grid_prb);
    srsgpu_pusch_demodulator_plan* plan = plans.get(key, [&] {
      const srsgpu_alloc_ext         ext = d.ext();
      srsgpu_pusch_demodulator_plan* p   = nullptr;
      gpu::srsgpu_check(srsgpu_pusch_demodulator_plan_create_ex(ctx, &c, &ext, 1, grid_prb, P, &p), WHO);
      return p;
    });
    const uint32_t nof_llrs = srsgpu_pusch_demodulator_plan_nof_llrs(plan, 0);

    // Rx grid rows of the allocated symbols, [port][symbol][subcarrier].
    hipStream_t    s     = stream.get();
    const size_t   row   = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const unsigned l0    = config.start_symbol_index;
    const unsigned nsym  = config.nof_symbols;
    grid_buf.reserve(P * 14 * row);
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = l0; l != l0 + nsym; ++l) {
        std::memcpy(grid_buf.host((p * 14 + l) * row), grid.get_view(config.rx_ports[p], l).data(), row);
      }
      grid_buf.upload((p * 14 + l0) * row, nsym * row, s);
    }
    // Channel estimates [layer][port][symbol][subcarrier] (channel_estimate rows are CRB-indexed like the grid) and
    // the noise variances at [4 tx + port].
    const size_t ce_slot = static_cast<size_t>(P) * 14 * row;
    ce_buf.reserve(4 * ce_slot + 4 * sizeof(float));
    for (unsigned ly = 0; ly != L; ++ly) {
      for (unsigned p = 0; p != P; ++p) {
        const size_t base = ly * ce_slot + static_cast<size_t>(p) * 14 * row;
        for (unsigned l = l0; l != l0 + nsym; ++l) {
          span<const cbf16_t> v = estimates.get_symbol_ch_estimate(l, p, ly);
          const size_t        n = std::min<size_t>(v.size(), nsc) * sizeof(uint32_t);
          std::memcpy(ce_buf.host(base + l * row), v.data(), n);
          if (n < row) {
            std::memset(ce_buf.host(base + l * row + n), 0, row - n);
          }
        }
        ce_buf.upload(base + l0 * row, nsym * row, s);
      }
    }
    float* nv = ce_buf.host<float>(4 * ce_slot);
    for (unsigned p = 0; p != 4; ++p) {
      nv[p] = p < P ? estimates.get_noise_variance(p) : 0.0F;
    }
    ce_buf.upload(4 * ce_slot, 4 * sizeof(float), s);

    // LLRs, statistics and the descrambling sequence.
    const size_t seq_words = (nof_llrs + 31) / 32;
    const size_t stats_off = (nof_llrs + 15) / 16 * 16;
    const size_t seq_off   = stats_off + SRSGPU_DEMOD_STATS * sizeof(float);
    out_buf.reserve(seq_off + seq_words * 4);
    gpu::srsgpu_check(srsgpu_pusch_demodulator_plan_execute_ex(plan, grid_buf.dev<uint32_t>(), ce_buf.dev<uint32_t>(),
                                                               ce_buf.dev<float>(4 * ce_slot), out_buf.dev<int8_t>(),
                                                               out_buf.dev<float>(stats_off), s),
                      WHO);
    gpu::srsgpu_check(srsgpu_pusch_demodulator_plan_scrambling(plan, 0, out_buf.dev<uint32_t>(seq_off), s), WHO);
    out_buf.download(0, seq_off + seq_words * 4, s);
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");

    gpu::feed_codeword(codeword_buffer, notifier, config, a.nof_rb, out_buf.host<int8_t>(),
                       out_buf.host<uint32_t>(seq_off), nof_llrs, out_buf.host<float>(stats_off), opts, seq_bytes,
                       block_seq, WHO);
  }

private:
  std::shared_ptr<srsgpu_context>                owner;
  srsgpu_context*                                ctx;
  gpu::pusch_demodulator_options                 opts;
  gpu::owned_stream                              stream;
  gpu::plan_cache<srsgpu_pusch_demodulator_plan> plans;
  gpu::staged_buffer                             grid_buf;
  gpu::staged_buffer                             ce_buf;
  gpu::staged_buffer                             out_buf;
  std::vector<uint8_t>                           seq_bytes;
  dynamic_bit_buffer                             block_seq;
};

class pusch_demodulator_factory_gpu : public pusch_demodulator_factory
{
public:
  pusch_demodulator_factory_gpu(int device, const gpu::pusch_demodulator_options& opts_) :
    ctx(gpu::shared_context(device)), opts(opts_)
  {
  }
  std::unique_ptr<pusch_demodulator> create() override { return std::make_unique<pusch_demodulator_gpu>(ctx, opts); }

private:
  std::shared_ptr<srsgpu_context> ctx;
  gpu::pusch_demodulator_options  opts;
};

} // namespace

std::shared_ptr<dmrs_pusch_estimator_factory>
create_dmrs_pusch_estimator_factory_gpu(int device, const gpu::pusch_estimator_options& opts)
{
  return std::make_shared<dmrs_pusch_estimator_factory_gpu>(device, opts);
}

std::shared_ptr<pusch_demodulator_factory> create_pusch_demodulator_factory_gpu(int                                   device,
                                                                                const gpu::pusch_demodulator_options& opts)
{
  return std::make_shared<pusch_demodulator_factory_gpu>(device, opts);
}

} // namespace srsran
