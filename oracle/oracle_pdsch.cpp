// =====================================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU restatement ("oracle") of the srsRAN PDSCH modulator: scrambling, modulation mapping,
// layer mapping, precoding and resource-element mapping into a bf16 resource grid.
//
// Same rules as oracle.cpp: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it, as the
// checker. Pinned bit-for-bit against the reference's own pdsch_modulator_impl (oracle/ref/ref_pdsch_mod.cpp in
// oracle/_ref/libsrsref.so) by tests/test_oracle_vs_reference.py and against tests/golden/pdsch_mod_*.npz.
//
// Reference files (under /root/reference/lib/phy/):
//   upper/channel_processors/pdsch/pdsch_modulator_impl.cpp:30  scramble, c_init = (rnti << 15) + (q << 14) + n_id
//   upper/sequence_generators/pseudo_random_generator_impl.cpp:44  Gold sequence, Nc = 1600 (TS 38.211 §5.2.1)
//   upper/channel_modulation/modulation_mapper_lut_impl.cpp:39  constellation tables (TS 38.211 §5.1), ci8 symbols,
//                                                              scaling sqrt(1 / average power)
//   upper/channel_processors/pdsch/pdsch_modulator_impl.cpp:52  allocation and DM-RS patterns, scaling *= config
//   support/resource_grid_mapper_impl.cpp:269                   RE order (symbol, then subcarrier), layer mapping
//   generic_functions/precoding/channel_precoder_generic.cpp:51  sum over layers of to_cf(x) * w, then to cbf16
//   include/srsran/adt/bf16.h:39                                 float -> bf16, round half to even
// =====================================================================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

// TS 38.211 §5.2.1 length-31 Gold sequence c(n), n = 0..len-1, for initial state c_init of x2.
std::vector<uint8_t> gold_sequence(uint32_t c_init, size_t len)
{
  const size_t         Nc = 1600;
  std::vector<uint8_t> x1(Nc + len + 31), x2(Nc + len + 31), c(len);
  for (int i = 0; i < 31; ++i) {
    x1[i] = (i == 0);
    x2[i] = (c_init >> i) & 1U;
  }
  for (size_t n = 0; n + 31 < x1.size(); ++n) {
    x1[n + 31] = x1[n + 3] ^ x1[n];
    x2[n + 31] = x2[n + 3] ^ x2[n + 2] ^ x2[n + 1] ^ x2[n];
  }
  for (size_t n = 0; n < len; ++n) {
    c[n] = x1[n + Nc] ^ x2[n + Nc];
  }
  return c;
}

// TS 38.211 §5.1 constellation point (integer grid, before normalisation) of `index` (first bit = MSB), the way
// modulation_mapper_lut_impl.cpp:39 builds its table: odd index bits (from the LSB) drive the real part, even bits the
// imaginary part, each level adding the next power of two.
void constellation_point(unsigned qm, unsigned index, int& re, int& im)
{
  float offset = -1, real = 0, imag = 0;
  for (unsigned j = 0; j < qm / 2; ++j) {
    real += offset;
    imag += offset;
    offset *= 2;
    real *= ((index >> (2 * j + 1)) & 1U) ? 1 : -1;
    imag *= ((index >> (2 * j)) & 1U) ? 1 : -1;
  }
  re = static_cast<int>(real);
  im = static_cast<int>(imag);
}

float average_power(unsigned qm)
{
  double acc = 0;
  for (unsigned i = 0; i < (1U << qm); ++i) {
    int re, im;
    constellation_point(qm, i, re, im);
    acc += re * re + im * im;
  }
  return static_cast<float>(acc / (1U << qm));
}

uint16_t to_bf16(float v)
{
  uint32_t u;
  std::memcpy(&u, &v, 4);
  u += 0x7fffU + ((u >> 16) & 1U);
  return static_cast<uint16_t>(u >> 16);
}

// DM-RS RE mask within a PRB (dmrs_mapping.h get_dmrs_prb_mask): type 1 CDM group g uses subcarriers 2k + g, type 2
// CDM group g uses 6k + 2g + {0, 1}. Bit k = subcarrier k is DM-RS (no data).
unsigned dmrs_prb_mask(int type2, int nof_cdm_groups_without_data)
{
  unsigned m = 0;
  for (int k = 0; k < 12; ++k) {
    int group = type2 ? (k % 6) / 2 : k % 2;
    if (group < nof_cdm_groups_without_data) {
      m |= 1U << k;
    }
  }
  return m;
}


// Scrambles, modulates, layer-maps and precodes the codeword onto the REs `res` (allocation order), the weights of RE
// r being w + wsel(r) * 2 * nof_ports * nof_layers (pdsch_modulator_impl.cpp:30-:105, channel_precoder_generic.cpp:51).
template <typename Sel>
int modulate_res(const std::vector<std::pair<int, int>>& res,
                 int                                     rnti,
                 int                                     n_id,
                 int                                     qm,
                 int                                     nof_layers,
                 int                                     nof_ports,
                 float                                   scaling,
                 const float*                            weights,
                 size_t                                  nof_weight_sets,
                 Sel                                     wsel,
                 const uint8_t*                          codeword_packed,
                 int                                     nof_bits,
                 int                                     grid_nof_prb,
                 uint16_t*                               grid_out)
{
  const unsigned nsc = 12 * grid_nof_prb;
  if (static_cast<long>(res.size()) * nof_layers * qm != nof_bits) {
    return -1;
  }

  // Scrambling (pdsch_modulator_impl.cpp:30, codeword q = 0).
  const uint32_t       c_init = (static_cast<uint32_t>(rnti) << 15) + static_cast<uint32_t>(n_id);
  std::vector<uint8_t> c      = gold_sequence(c_init, nof_bits);
  std::vector<uint8_t> b(nof_bits);
  for (int i = 0; i < nof_bits; ++i) {
    b[i] = ((codeword_packed[i / 8] >> (7 - i % 8)) & 1U) ^ c[i];
  }

  // Modulation scaling and the effective precoding weights (pdsch_modulator_impl.cpp:93-96).
  float amp = std::sqrt(1 / average_power(qm));
  if (std::isnormal(scaling)) {
    amp *= scaling;
  }
  std::vector<float> w(2 * nof_ports * nof_layers * nof_weight_sets);
  for (size_t i = 0; i < w.size(); ++i) {
    w[i] = weights[i] * amp;
  }

  for (size_t r = 0; r < res.size(); ++r) {
    // Layer mapping x^(l)(r) = d(L r + l) (TS 38.211 §7.3.1.3).
    int xr[4], xi[4];
    for (int l = 0; l < nof_layers; ++l) {
      unsigned idx = 0;
      for (int j = 0; j < qm; ++j) {
        idx = (idx << 1) | b[(r * nof_layers + l) * qm + j];
      }
      constellation_point(qm, idx, xr[l], xi[l]);
    }
    const float* wr_set = w.data() + wsel(res[r].second) * 2 * nof_ports * nof_layers;
    for (int p = 0; p < nof_ports; ++p) {
      float sr = 0, si = 0;
      for (int l = 0; l < nof_layers; ++l) {
        const float a = static_cast<float>(xr[l]), bb = static_cast<float>(xi[l]);
        const float wr = wr_set[2 * (p * nof_layers + l)], wi = wr_set[2 * (p * nof_layers + l) + 1];
        // Complex product (a + jb)(wr + jwi), each product rounded (no fused multiply-add), accumulated in order.
        volatile float ac = a * wr, bd = bb * wi, ad = a * wi, bc = bb * wr;
        const float    pr = ac - bd, pi = ad + bc;
        if (l == 0) {
          sr = pr;
          si = pi;
        } else {
          sr = sr + pr;
          si = si + pi;
        }
      }
      const size_t o      = 2 * ((static_cast<size_t>(p) * 14 + res[r].first) * nsc + res[r].second);
      grid_out[o]         = to_bf16(sr);
      grid_out[o + 1]     = to_bf16(si);
    }
  }
  return 0;
}

} // namespace

extern "C" {

/// Same contract as ref_pdsch_modulate (oracle/ref/ref_pdsch_mod.cpp): one codeword, VRB allocation
/// [rb_start, rb_start + nof_rb) of the BWP mapped to CRBs non-interleaved, DM-RS REs excluded, wideband precoding.
/// The grid (nof_ports x 14 x 12 * grid_nof_prb, (re, im) bf16 pairs) is written only at the PDSCH REs.
/// Returns 0, or -1 when the codeword length does not fill the allocation exactly.
int orc_pdsch_modulate(int            rnti,
                       int            n_id,
                       int            qm,
                       int            nof_layers,
                       int            nof_ports,
                       int            bwp_start_rb,
                       int            bwp_size_rb,
                       int            rb_start,
                       int            nof_rb,
                       int            start_symbol,
                       int            nof_symbols,
                       unsigned       dmrs_symbol_mask,
                       int            dmrs_type2,
                       int            nof_cdm_groups_without_data,
                       float          scaling,
                       const float*   weights,
                       const uint8_t* codeword_packed,
                       int            nof_bits,
                       int            grid_nof_prb,
                       uint16_t*      grid_out)
{
  (void)bwp_size_rb;
  const unsigned dmrs_mask = dmrs_prb_mask(dmrs_type2, nof_cdm_groups_without_data);

  // Data REs in allocation order: symbol-major, subcarrier ascending (resource_grid_mapper_impl.cpp:269).
  std::vector<std::pair<int, int>> res;
  for (int l = start_symbol; l < start_symbol + nof_symbols; ++l) {
    const bool dmrs = ((dmrs_symbol_mask >> l) & 1U) != 0;
    for (int rb = 0; rb < nof_rb; ++rb) {
      const int crb = bwp_start_rb + rb_start + rb;
      for (int k = 0; k < 12; ++k) {
        if (!dmrs || ((dmrs_mask >> k) & 1U) == 0) {
          res.emplace_back(l, crb * 12 + k);
        }
      }
    }
  }
  return modulate_res(res, rnti, n_id, qm, nof_layers, nof_ports, scaling, weights, 1, [](int) { return 0; },
                      codeword_packed, nof_bits, grid_nof_prb, grid_out);
}

/// General allocation (the srsgpu_pdsch_modulator_plan_create_ex contract): CRB mask crb_mask (one byte per grid CRB,
/// rb_allocation::get_crb_mask), the BWP's DM-RS pattern on DM-RS symbols (dmrs_mapping.h get_dmrs_pattern over
/// [bwp_start_rb, bwp_start_rb + bwp_size_rb)) and nof_reserved reserved patterns excluded (pattern i: CRBs with
/// res_crb[i * grid_nof_prb + crb] set, PRB subcarriers res_re[i], symbols res_sym[i]; re_pattern.cpp exclusion
/// masks); per-PRG precoding when prg_size > 0 (PRG of subcarrier k = k / (12 prg_size), resource_grid_mapper_impl.cpp
/// :318), prg_weights [nof_prg][port][layer] (re, im); wideband `weights` otherwise.
int orc_pdsch_modulate_ex(int             rnti,
                          int             n_id,
                          int             qm,
                          int             nof_layers,
                          int             nof_ports,
                          int             bwp_start_rb,
                          int             bwp_size_rb,
                          const uint8_t*  crb_mask,
                          int             start_symbol,
                          int             nof_symbols,
                          unsigned        dmrs_symbol_mask,
                          int             dmrs_type2,
                          int             nof_cdm_groups_without_data,
                          float           scaling,
                          const float*    weights,
                          int             nof_reserved,
                          const uint8_t*  res_crb,
                          const uint16_t* res_re,
                          const uint16_t* res_sym,
                          int             prg_size,
                          int             nof_prg,
                          const float*    prg_weights,
                          const uint8_t*  codeword_packed,
                          int             nof_bits,
                          int             grid_nof_prb,
                          uint16_t*       grid_out)
{
  const unsigned dmrs_mask = dmrs_prb_mask(dmrs_type2, nof_cdm_groups_without_data);
  std::vector<std::pair<int, int>> res;
  for (int l = start_symbol; l < start_symbol + nof_symbols; ++l) {
    const bool dmrs = ((dmrs_symbol_mask >> l) & 1U) != 0;
    for (int crb = 0; crb < grid_nof_prb; ++crb) {
      if (crb_mask[crb] == 0) {
        continue;
      }
      unsigned excl = (dmrs && crb >= bwp_start_rb && crb < bwp_start_rb + bwp_size_rb) ? dmrs_mask : 0U;
      for (int i = 0; i < nof_reserved; ++i) {
        if (((res_sym[i] >> l) & 1U) != 0 && res_crb[static_cast<size_t>(i) * grid_nof_prb + crb] != 0) {
          excl |= res_re[i];
        }
      }
      for (int k = 0; k < 12; ++k) {
        if (((excl >> k) & 1U) == 0) {
          res.emplace_back(l, crb * 12 + k);
        }
      }
    }
  }
  if (prg_size > 0) {
    const int prg_sc = 12 * prg_size;
    return modulate_res(res, rnti, n_id, qm, nof_layers, nof_ports, scaling, prg_weights, nof_prg,
                        [prg_sc](int sc) { return sc / prg_sc; }, codeword_packed, nof_bits, grid_nof_prb, grid_out);
  }
  return modulate_res(res, rnti, n_id, qm, nof_layers, nof_ports, scaling, weights, 1, [](int) { return 0; },
                      codeword_packed, nof_bits, grid_nof_prb, grid_out);
}

} // extern "C"
