// Reference-side bindings of the PDSCH signal chain (the files a srsRAN maintainer adds next to
// lib/phy/upper/channel_processors/pdsch/ and lib/phy/upper/signal_processors/): srsran::pdsch_modulator
// (include/srsran/phy/upper/channel_processors/pdsch/pdsch_modulator.h:93) and srsran::dmrs_pdsch_processor
// (include/srsran/phy/upper/signal_processors/dmrs_pdsch_processor.h:65) over the srsgpu C ABI, so that the reference's
// own pdsch_processor_impl (pdsch_processor_impl.cpp:123 modulate, :153 DM-RS; upper_phy_factories.cpp:940-1014)
// maps its PDSCH on an MI355X.
//
// The reference's resource grid is shared by every channel of the slot and written concurrently by their processors
// (each writes its own REs), so a binding must write exactly the REs the reference would and nothing else. The kernel
// maps into a device scratch grid pre-filled with a sentinel (0xffffffff: a bf16 NaN pair, which the modulator and the
// DM-RS mapper never produce from finite inputs); after the copy back, exactly the non-sentinel REs are stored into the
// caller's grid, and every port written is marked non-empty through resource_grid_writer::put (the empty flags the
// OFDM modulator checks, ofdm_modulator_impl.cpp:77).
#include "signal_chain_gpu.h"

#include "chain_convert.h"
#include "gpu_staging.h"
#include "srsran/phy/support/resource_grid_writer.h"

#include <stdexcept>
#include <string>

namespace srsran {

namespace {

using gpu::store_written_res;

// --------------------------------------------------------------------------------------------------------------------
// PDSCH modulator
// --------------------------------------------------------------------------------------------------------------------

class pdsch_modulator_gpu : public pdsch_modulator
{
  static constexpr const char* WHO = "pdsch_modulator_gpu";

public:
  explicit pdsch_modulator_gpu(std::shared_ptr<srsgpu_context> owner_) :
    owner(std::move(owner_)),
    ctx(owner.get()),
    stream(ctx, WHO),
    plans(srsgpu_pdsch_modulator_plan_destroy),
    cw_buf(WHO),
    grid_buf(WHO)
  {
  }

  void modulate(resource_grid_writer& grid, span<const bit_buffer> codewords, const config_t& config) override
  {
    gpu::device_scope dev_scope(ctx, WHO);
    if (codewords.size() != 1) {
      throw std::invalid_argument(std::string(WHO) + ": one codeword, 1..4 layers on 1..4 ports");
    }
    const unsigned      nsc      = grid.get_nof_subc();
    const unsigned      grid_prb = nsc / NRE;
    gpu::pdsch_mod_desc d =
        gpu::make_pdsch_mod_desc(config, codewords[0].size(), grid_prb, grid.get_nof_ports(), WHO);
    const unsigned P = d.c.nof_ports;

    std::vector<uint8_t> key;
    d.append_key(key);
    gpu::key_append(key, grid_prb);
    srsgpu_pdsch_modulator_plan* plan = plans.get(key, [&] {
      const srsgpu_alloc_ext       ext = d.ext();
      srsgpu_pdsch_modulator_plan* p   = nullptr;
      gpu::srsgpu_check(srsgpu_pdsch_modulator_plan_create_ex(ctx, &d.c, &ext, 1, grid_prb, P, &p), WHO);
      return p;
    });

    // Codeword (packed MSB first, as srsran::bit_buffer stores it) padded to whole words.
    hipStream_t    s      = stream.get();
    span<const uint8_t> cw = codewords[0].get_buffer();
    const size_t   cw_len = (cw.size() + 3) / 4 * 4;
    cw_buf.reserve(cw_len);
    std::memcpy(cw_buf.host(), cw.data(), cw.size());
    std::memset(cw_buf.host(cw.size()), 0, cw_len - cw.size());
    cw_buf.upload(0, cw_len, s);
    // Sentinel scratch grid, the allocated symbols' rows of every port.
    const size_t   row  = static_cast<size_t>(nsc) * sizeof(uint32_t);
    const unsigned l0   = config.start_symbol_index;
    const unsigned nsym = config.nof_symbols;
    grid_buf.reserve(P * 14 * row);
    for (unsigned p = 0; p != P; ++p) {
      gpu::hip_check(hipMemsetAsync(grid_buf.dev((p * 14 + l0) * row), 0xff, nsym * row, s), WHO, "scratch");
    }
    gpu::srsgpu_check(srsgpu_pdsch_modulator_plan_execute(plan, cw_buf.dev(), grid_buf.dev<uint32_t>(), s), WHO);
    for (unsigned p = 0; p != P; ++p) {
      grid_buf.download((p * 14 + l0) * row, nsym * row, s);
    }
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");
    store_written_res(grid, grid_buf.host<uint32_t>(), P, nsc, l0, nsym);
  }

private:
  std::shared_ptr<srsgpu_context>              owner;
  srsgpu_context*                              ctx;
  gpu::owned_stream                            stream;
  gpu::plan_cache<srsgpu_pdsch_modulator_plan> plans;
  gpu::staged_buffer                           cw_buf;
  gpu::staged_buffer                           grid_buf;
};

class pdsch_modulator_factory_gpu : public pdsch_modulator_factory
{
public:
  explicit pdsch_modulator_factory_gpu(int device) : ctx(gpu::shared_context(device)) {}
  std::unique_ptr<pdsch_modulator> create() override { return std::make_unique<pdsch_modulator_gpu>(ctx); }

private:
  std::shared_ptr<srsgpu_context> ctx;
};

// --------------------------------------------------------------------------------------------------------------------
// PDSCH DM-RS processor
// --------------------------------------------------------------------------------------------------------------------

class dmrs_pdsch_processor_gpu : public dmrs_pdsch_processor
{
  static constexpr const char* WHO = "dmrs_pdsch_processor_gpu";

public:
  explicit dmrs_pdsch_processor_gpu(std::shared_ptr<srsgpu_context> owner_) :
    owner(std::move(owner_)), ctx(owner.get()), stream(ctx, WHO), plans(srsgpu_pdsch_dmrs_plan_destroy), grid_buf(WHO)
  {
  }

  void map(resource_grid_writer& grid, const config_t& config) override
  {
    gpu::device_scope dev_scope(ctx, WHO);
    const unsigned             nsc      = grid.get_nof_subc();
    const unsigned             grid_prb = nsc / NRE;
    const gpu::pdsch_dmrs_desc d        = gpu::make_pdsch_dmrs_desc(config, grid_prb, grid.get_nof_ports(), WHO);
    const srsgpu_pdsch_dmrs_config& c   = d.c;
    const unsigned                  P   = c.nof_ports;

    std::vector<uint8_t> key;
    d.append_key(key);
    gpu::key_append(key, grid_prb);
    srsgpu_pdsch_dmrs_plan* plan = plans.get(key, [&] {
      const srsgpu_alloc_ext  ext = d.ext();
      srsgpu_pdsch_dmrs_plan* p   = nullptr;
      gpu::srsgpu_check(srsgpu_pdsch_dmrs_plan_create_ex(ctx, &c, &ext, 1, grid_prb, P, &p), WHO);
      return p;
    });

    hipStream_t  s   = stream.get();
    const size_t row = static_cast<size_t>(nsc) * sizeof(uint32_t);
    grid_buf.reserve(P * 14 * row);
    gpu::hip_check(hipMemsetAsync(grid_buf.dev(), 0xff, P * 14 * row, s), WHO, "scratch");
    gpu::srsgpu_check(srsgpu_pdsch_dmrs_plan_execute(plan, grid_buf.dev<uint32_t>(), s), WHO);
    for (unsigned p = 0; p != P; ++p) {
      for (unsigned l = 0; l != 14; ++l) {
        if ((c.dmrs_symbol_mask >> l) & 1u) {
          grid_buf.download((p * 14 + l) * row, row, s);
        }
      }
    }
    gpu::hip_check(hipStreamSynchronize(s), WHO, "synchronise");
    for (unsigned l = 0; l != 14; ++l) {
      if ((c.dmrs_symbol_mask >> l) & 1u) {
        store_written_res(grid, grid_buf.host<uint32_t>(), P, nsc, l, 1);
      }
    }
  }

private:
  std::shared_ptr<srsgpu_context>         owner;
  srsgpu_context*                         ctx;
  gpu::owned_stream                       stream;
  gpu::plan_cache<srsgpu_pdsch_dmrs_plan> plans;
  gpu::staged_buffer                      grid_buf;
};

class dmrs_pdsch_processor_factory_gpu : public dmrs_pdsch_processor_factory
{
public:
  explicit dmrs_pdsch_processor_factory_gpu(int device) : ctx(gpu::shared_context(device)) {}
  std::unique_ptr<dmrs_pdsch_processor> create() override { return std::make_unique<dmrs_pdsch_processor_gpu>(ctx); }

private:
  std::shared_ptr<srsgpu_context> ctx;
};

} // namespace

std::shared_ptr<pdsch_modulator_factory> create_pdsch_modulator_factory_gpu(int device)
{
  return std::make_shared<pdsch_modulator_factory_gpu>(device);
}

std::shared_ptr<dmrs_pdsch_processor_factory> create_dmrs_pdsch_processor_factory_gpu(int device)
{
  return std::make_shared<dmrs_pdsch_processor_factory_gpu>(device);
}

} // namespace srsran
