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

#include "gpu_staging.h"
#include "srsran/phy/support/resource_grid_writer.h"

#include <stdexcept>
#include <string>

namespace srsran {

namespace {

constexpr uint32_t SENTINEL = 0xffffffffu;

/// Copies the non-sentinel REs of scratch rows [port][14][nsc] (symbols [l0, l0 + nsym) of ports 0..P-1) into the
/// grid; a port that received any RE is marked non-empty.
void store_written_res(resource_grid_writer& grid, const uint32_t* scratch, unsigned P, unsigned nsc, unsigned l0,
                       unsigned nsym)
{
  for (unsigned p = 0; p != P; ++p) {
    int      first_k = -1;
    unsigned first_l = 0;
    cbf16_t  first_v;
    for (unsigned l = l0; l != l0 + nsym; ++l) {
      const uint32_t* src = scratch + (static_cast<size_t>(p) * 14 + l) * nsc;
      span<cbf16_t>   dst = grid.get_view(p, l);
      for (unsigned k = 0; k != nsc; ++k) {
        if (src[k] != SENTINEL) {
          std::memcpy(&dst[k], &src[k], sizeof(uint32_t));
          if (first_k < 0) {
            first_k = static_cast<int>(k);
            first_l = l;
            first_v = dst[k];
          }
        }
      }
    }
    if (first_k >= 0) {
      // Rewrites one RE with its own value: resource_grid_writer_impl clears the port's empty flag on put().
      grid.put(p, first_l, static_cast<unsigned>(first_k), 1, span<const cbf16_t>(&first_v, 1));
    }
  }
}

/// Grid CRB mask (one byte per CRB) of a crb_bitmap.
std::vector<uint8_t> crb_bytes(const crb_bitmap& m, unsigned grid_prb)
{
  std::vector<uint8_t> out(grid_prb, 0);
  for (unsigned rb = 0; rb != std::min<unsigned>(grid_prb, m.size()); ++rb) {
    out[rb] = m.test(rb) ? 1 : 0;
  }
  return out;
}

/// Wideband precoding weights [port][layer] of PRG 0.
void wideband_weights(const precoding_configuration& pc, float (&w)[4][4][2])
{
  std::memset(w, 0, sizeof(w));
  for (unsigned p = 0; p != pc.get_nof_ports(); ++p) {
    for (unsigned ly = 0; ly != pc.get_nof_layers(); ++ly) {
      const cf_t c = pc.get_coefficient(ly, p, 0);
      w[p][ly][0]  = c.real();
      w[p][ly][1]  = c.imag();
    }
  }
}

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
    const precoding_configuration& pc = config.precoding;
    const unsigned                 L  = pc.get_nof_layers();
    const unsigned                 P  = pc.get_nof_ports();
    if (codewords.size() != 1 || L == 0 || L > 4 || P < L || P > 4 || P > grid.get_nof_ports()) {
      throw std::invalid_argument(std::string(WHO) + ": one codeword, 1..4 layers on 1..4 ports");
    }
    const unsigned       nsc      = grid.get_nof_subc();
    const unsigned       grid_prb = nsc / NRE;
    const crb_bitmap     crbs     = config.freq_allocation.get_crb_mask(config.bwp_start_rb, config.bwp_size_rb);
    std::vector<uint8_t> crb_mask = crb_bytes(crbs, grid_prb);

    srsgpu_pdsch_mod_config c;
    std::memset(&c, 0, sizeof(c));
    c.rnti                        = config.rnti;
    c.n_id                        = static_cast<uint16_t>(config.n_id);
    c.modulation_order            = static_cast<uint8_t>(get_bits_per_symbol(config.modulation1));
    c.nof_layers                  = static_cast<uint8_t>(L);
    c.nof_ports                   = static_cast<uint8_t>(P);
    c.start_symbol                = static_cast<uint8_t>(config.start_symbol_index);
    c.nof_symbols                 = static_cast<uint8_t>(config.nof_symbols);
    c.dmrs_type                   = (config.dmrs_config_type == dmrs_type::TYPE1) ? 1 : 2;
    c.nof_cdm_groups_without_data = static_cast<uint8_t>(config.nof_cdm_groups_without_data);
    for (unsigned l = 0; l != 14; ++l) {
      c.dmrs_symbol_mask |= config.dmrs_symb_pos.test(l) ? (1u << l) : 0u;
    }
    c.bwp_start_rb = static_cast<uint16_t>(config.bwp_start_rb);
    c.bwp_size_rb  = static_cast<uint16_t>(config.bwp_size_rb);
    c.rb_start     = static_cast<uint16_t>(std::max(crbs.find_lowest(), 0));
    c.nof_rb       = static_cast<uint16_t>(crbs.count());
    c.scaling      = config.scaling;
    wideband_weights(pc, c.precoding);
    c.cw_offset  = 0;
    c.nof_bits   = codewords[0].size();
    c.grid_index = 0;

    // Reserved patterns and per-PRG weights (srsgpu_alloc_ext).
    std::vector<std::vector<uint8_t>> res_crbs;
    std::vector<srsgpu_re_pattern>    res;
    for (const re_pattern& r : config.reserved.get_re_patterns()) {
      res_crbs.push_back(crb_bytes(r.crb_mask, grid_prb));
      srsgpu_re_pattern x;
      std::memset(&x, 0, sizeof(x));
      for (unsigned k = 0; k != NRE; ++k) {
        x.re_mask |= r.re_mask.test(k) ? (1u << k) : 0u;
      }
      for (unsigned l = 0; l != 14; ++l) {
        x.symbol_mask |= r.symbols.test(l) ? (1u << l) : 0u;
      }
      res.push_back(x);
    }
    for (size_t i = 0; i != res.size(); ++i) {
      res[i].crb_mask = res_crbs[i].data();
    }
    std::vector<float> prg_w;
    if (pc.get_nof_prg() > 1) {
      for (unsigned g = 0; g != pc.get_nof_prg(); ++g) {
        for (unsigned p = 0; p != P; ++p) {
          for (unsigned ly = 0; ly != L; ++ly) {
            const cf_t w = pc.get_coefficient(ly, p, g);
            prg_w.push_back(w.real());
            prg_w.push_back(w.imag());
          }
        }
      }
    }

    std::vector<uint8_t> key;
    gpu::key_append(key, c);
    gpu::key_append(key, grid_prb);
    key.insert(key.end(), crb_mask.begin(), crb_mask.end());
    for (size_t i = 0; i != res.size(); ++i) {
      gpu::key_append(key, res[i].re_mask);
      gpu::key_append(key, res[i].symbol_mask);
      key.insert(key.end(), res_crbs[i].begin(), res_crbs[i].end());
    }
    gpu::key_append(key, pc.get_prg_size());
    const auto* pw = reinterpret_cast<const uint8_t*>(prg_w.data());
    key.insert(key.end(), pw, pw + prg_w.size() * sizeof(float));
    srsgpu_pdsch_modulator_plan* plan = plans.get(key, [&] {
      srsgpu_alloc_ext ext;
      std::memset(&ext, 0, sizeof(ext));
      ext.crb_mask     = crb_mask.data();
      ext.reserved     = res.empty() ? nullptr : res.data();
      ext.nof_reserved = static_cast<uint32_t>(res.size());
      if (!prg_w.empty()) {
        ext.prg_size    = static_cast<uint16_t>(pc.get_prg_size());
        ext.nof_prg     = static_cast<uint16_t>(pc.get_nof_prg());
        ext.prg_weights = prg_w.data();
      }
      srsgpu_pdsch_modulator_plan* p = nullptr;
      gpu::srsgpu_check(srsgpu_pdsch_modulator_plan_create_ex(ctx, &c, &ext, 1, grid_prb, P, &p), WHO);
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
    const precoding_configuration& pc = config.precoding;
    const unsigned                 L  = pc.get_nof_layers();
    const unsigned                 P  = pc.get_nof_ports();
    if (L == 0 || L > 4 || P < L || P > 4 || P > grid.get_nof_ports()) {
      throw std::invalid_argument(std::string(WHO) + ": 1..4 layers on 1..4 ports");
    }
    const unsigned       nsc      = grid.get_nof_subc();
    const unsigned       grid_prb = nsc / NRE;
    std::vector<uint8_t> crb_mask = crb_bytes(config.rb_mask, grid_prb);

    srsgpu_pdsch_dmrs_config c;
    std::memset(&c, 0, sizeof(c));
    c.slot_index    = static_cast<uint16_t>(config.slot.slot_index());
    c.scrambling_id = static_cast<uint16_t>(config.scrambling_id);
    c.n_scid        = config.n_scid ? 1 : 0;
    c.dmrs_type     = (config.type == dmrs_type::TYPE1) ? 1 : 2;
    c.nof_layers    = static_cast<uint8_t>(L);
    c.nof_ports     = static_cast<uint8_t>(P);
    for (unsigned l = 0; l != 14; ++l) {
      c.dmrs_symbol_mask |= config.symbols_mask.test(l) ? (1u << l) : 0u;
    }
    c.reference_point_k_rb = static_cast<uint16_t>(config.reference_point_k_rb);
    c.rb_start             = static_cast<uint16_t>(std::max(config.rb_mask.find_lowest(), 0));
    c.nof_rb               = static_cast<uint16_t>(config.rb_mask.count());
    c.amplitude            = config.amplitude;
    wideband_weights(pc, c.precoding);
    c.grid_index = 0;

    std::vector<uint8_t> key;
    gpu::key_append(key, c);
    gpu::key_append(key, grid_prb);
    key.insert(key.end(), crb_mask.begin(), crb_mask.end());
    srsgpu_pdsch_dmrs_plan* plan = plans.get(key, [&] {
      srsgpu_alloc_ext ext;
      std::memset(&ext, 0, sizeof(ext));
      ext.crb_mask                = crb_mask.data();
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
