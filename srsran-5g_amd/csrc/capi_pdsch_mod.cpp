// Host side of the PDSCH modulator C ABI (include/srsgpu_phy.h): validation with the reference's conditions, the
// Gold-sequence jump tables (once per context) and the per-transmission descriptors / per-chunk work items.
#include "capi_internal.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

using namespace srsgpu;

static_assert(sizeof(srsgpu_pdsch_mod_config) == 168, "srsgpu_pdsch_mod_config layout (mirrored by srsgpu.PdschModConfig)");

static_assert(sizeof(srsgpu_pdsch_dmrs_config) == 152, "srsgpu_pdsch_dmrs_config layout (mirrored by srsgpu)");

struct srsgpu_pdsch_dmrs_plan {
  srsgpu_context* ctx      = nullptr;
  dmrs_job*       d_jobs   = nullptr;
  uint32_t*       d_seq    = nullptr;  ///< DM-RS sequence words of every job (plan lifetime).
  int             nof_jobs = 0;
  int             max_pilots = 0;  ///< Largest job (workgroups per job of the launch).
};

struct srsgpu_pdsch_modulator_plan {
  srsgpu_context* ctx        = nullptr;
  mod_desc*       d_desc     = nullptr;
  uint16_t*       d_sc_map   = nullptr;  ///< RE -> grid subcarrier maps of the general allocations.
  float*          d_prg_w    = nullptr;  ///< Per-PRG weights [prg][port 4][layer 4][2] (amplitude folded in).
  mod_chunk*      d_chunks   = nullptr;
  uint32_t*       d_seq      = nullptr;  ///< Scrambling sequences of the transmissions (plan lifetime).
  int             nof_chunks = 0;
};

namespace {

/// One step of the x2 LFSR on its 31-bit window (bit k = x2(n + k)): x2(n + 31) = x2(n + 3) + x2(n + 2) + x2(n + 1) +
/// x2(n) (TS 38.211 section 5.2.1).
uint32_t x2_step(uint32_t s)
{
  const uint32_t nb = (s ^ (s >> 1) ^ (s >> 2) ^ (s >> 3)) & 1u;
  return (s >> 1) | (nb << 30);
}

uint32_t x1_step(uint32_t s)
{
  const uint32_t nb = (s ^ (s >> 3)) & 1u;
  return (s >> 1) | (nb << 30);
}

uint32_t gf2_apply(const uint32_t* cols, uint32_t v)
{
  uint32_t r = 0;
  for (int j = 0; j < 31; ++j) {
    if ((v >> j) & 1u) {
      r ^= cols[j];
    }
  }
  return r;
}

} // namespace

std::vector<uint32_t> srsgpu::gold_sequence_offsets(const std::vector<uint32_t>& nwords)
{
  std::vector<uint32_t> off(nwords.size());
  uint32_t              o = 0;
  for (size_t t = 0; t < nwords.size(); ++t) {
    off[t] = o;
    o += nwords[t] + 1u;
  }
  return off;
}

int srsgpu::build_gold_sequences(srsgpu_context*              ctx,
                                 const std::vector<uint32_t>& c_inits,
                                 const std::vector<uint32_t>& nwords,
                                 const std::vector<uint32_t>& offsets,
                                 uint32_t**                   d_seq,
                                 const std::vector<uint32_t>* wstart)
{
  *d_seq = nullptr;
  if (c_inits.empty()) {
    return SRSGPU_OK;
  }
  const size_t n     = c_inits.size();
  size_t       total = 1;
  uint32_t     maxw  = 0;
  for (size_t t = 0; t < n; ++t) {
    total = std::max(total, static_cast<size_t>(offsets[t]) + nwords[t] + 1u);
    maxw  = std::max(maxw, nwords[t]);
  }
  uint32_t* d_small = nullptr;  // c_inits | offsets | nwords | wstart
  bool      ok      = hipMalloc(reinterpret_cast<void**>(d_seq), total * 4) == hipSuccess &&
               hipMemset(*d_seq, 0, total * 4) == hipSuccess &&
               hipMalloc(reinterpret_cast<void**>(&d_small), 4 * n * 4) == hipSuccess &&
               hipMemcpy(d_small, c_inits.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(d_small + n, offsets.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(d_small + 2 * n, nwords.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess &&
               (wstart == nullptr ||
                hipMemcpy(d_small + 3 * n, wstart->data(), n * 4, hipMemcpyHostToDevice) == hipSuccess);
  if (ok) {
    launch_gold_fill(d_small, d_small + n, d_small + 2 * n, wstart != nullptr ? d_small + 3 * n : nullptr,
                     static_cast<int>(n), maxw, *d_seq, ctx->d_gold_x1, ctx->d_gold_x2_jump, ctx->d_gold_x2_lane,
                     nullptr);
    ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(nullptr) == hipSuccess;
  }
  if (d_small != nullptr) {
    (void)hipFree(d_small);
  }
  if (!ok) {
    if (*d_seq != nullptr) {
      (void)hipFree(*d_seq);
      *d_seq = nullptr;
    }
    return fail(SRSGPU_ERR_HIP, "failed to build the scrambling sequences");
  }
  return SRSGPU_OK;
}

/// Builds and uploads the scrambler's Gold-sequence tables into the context (once; caller holds ctx->mtx).
int srsgpu::ensure_gold_tables(srsgpu_context* ctx)
{
  if (ctx->d_gold_x1 != nullptr) {
    return SRSGPU_OK;
  }
  // x1 (initial state x1(0) = 1): words of x1(Nc + 32 w + k), bit k.
  std::vector<uint32_t> x1(GOLD_X1_WORDS, 0u);
  uint32_t              s = 1;
  for (uint32_t n = 0; n < GOLD_NC; ++n) {
    s = x1_step(s);
  }
  for (uint32_t w = 0; w < GOLD_X1_WORDS; ++w) {
    uint32_t word = 0;
    for (int k = 0; k < 32; ++k) {
      word |= (s & 1u) << k;
      s = x1_step(s);
    }
    x1[w] = word;
  }
  // Lane jumps M^(32 i), stored [column j][i].
  std::vector<uint32_t> lane(31 * 64);
  for (int j = 0; j < 31; ++j) {
    uint32_t v = 1u << j;
    for (int i = 0; i < 64; ++i) {
      lane[static_cast<size_t>(j) * 64 + static_cast<size_t>(i)] = v;
      for (int k = 0; k < 32; ++k) {
        v = x2_step(v);
      }
    }
  }
  // Chunk jumps M^(Nc + 2048 c): columns of M^Nc by stepping, then repeated products with M^2048.
  uint32_t m2048[31], cur[31];
  for (int j = 0; j < 31; ++j) {
    uint32_t v = 1u << j, u = 1u << j;
    for (int k = 0; k < 2048; ++k) {
      v = x2_step(v);
    }
    for (uint32_t k = 0; k < GOLD_NC; ++k) {
      u = x2_step(u);
    }
    m2048[j] = v;
    cur[j]   = u;
  }
  std::vector<uint32_t> jump(static_cast<size_t>(GOLD_X2_JUMPS) * 31);
  for (uint32_t c = 0; c < GOLD_X2_JUMPS; ++c) {
    std::memcpy(&jump[static_cast<size_t>(c) * 31], cur, sizeof(cur));
    for (int j = 0; j < 31; ++j) {
      cur[j] = gf2_apply(m2048, cur[j]);
    }
  }
  uint32_t *d_x1 = nullptr, *d_jump = nullptr, *d_lane = nullptr;
  if (hipMalloc(&d_x1, x1.size() * 4) != hipSuccess || hipMalloc(&d_jump, jump.size() * 4) != hipSuccess ||
      hipMalloc(&d_lane, lane.size() * 4) != hipSuccess ||
      hipMemcpy(d_x1, x1.data(), x1.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d_jump, jump.data(), jump.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d_lane, lane.data(), lane.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    for (uint32_t* p : {d_x1, d_jump, d_lane}) {
      if (p != nullptr) {
        (void)hipFree(p);
      }
    }
    return fail(SRSGPU_ERR_HIP, "failed to upload the Gold sequence tables");
  }
  ctx->d_gold_x1      = d_x1;
  ctx->d_gold_x2_jump = d_jump;
  ctx->d_gold_x2_lane = d_lane;
  return SRSGPU_OK;
}

namespace {

/// TS 38.211 section 5.1 constellation point (integer grid) of `index`, as modulation_mapper_lut_impl.cpp:39 builds
/// its tables; used for the average power only.
void constellation_point(unsigned qm, unsigned index, int& re, int& im)
{
  int offset = -1, real = 0, imag = 0;
  for (unsigned j = 0; j < qm / 2; ++j) {
    real += offset;
    imag += offset;
    offset *= 2;
    real *= ((index >> (2 * j + 1)) & 1U) ? 1 : -1;
    imag *= ((index >> (2 * j)) & 1U) ? 1 : -1;
  }
  re = real;
  im = imag;
}

/// Amplitude sqrt(1 / average power) of the modulation mapper's integer constellation (modulation_mapper_lut_impl.cpp
/// returns it as the scaling the modulator applies through the precoding weights, pdsch_modulator_impl.cpp:93).
float modulation_amplitude(unsigned qm)
{
  double acc = 0;
  for (unsigned i = 0; i < (1U << qm); ++i) {
    int re, im;
    constellation_point(qm, i, re, im);
    acc += re * re + im * im;
  }
  const float avg = static_cast<float>(acc / (1U << qm));
  return std::sqrt(1 / avg);
}

} // namespace

extern "C" {

int srsgpu_pdsch_modulator_plan_create(srsgpu_context*                ctx,
                                       const srsgpu_pdsch_mod_config* cfgs,
                                       uint32_t                       nof_tx,
                                       uint32_t                       grid_nof_prb,
                                       uint32_t                       grid_nof_ports,
                                       srsgpu_pdsch_modulator_plan**  plan_out)
{
  return srsgpu_pdsch_modulator_plan_create_ex(ctx, cfgs, nullptr, nof_tx, grid_nof_prb, grid_nof_ports, plan_out);
}

int srsgpu_pdsch_modulator_plan_create_ex(srsgpu_context*                ctx,
                                          const srsgpu_pdsch_mod_config* cfgs,
                                          const srsgpu_alloc_ext*        exts,
                                          uint32_t                       nof_tx,
                                          uint32_t                       grid_nof_prb,
                                          uint32_t                       grid_nof_ports,
                                          srsgpu_pdsch_modulator_plan**  plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_tx > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (grid_nof_prb == 0 || grid_nof_prb > 275 || grid_nof_ports == 0 || grid_nof_ports > 4) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid grid geometry (%u PRB, %u ports)", grid_nof_prb, grid_nof_ports);
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  int r = ensure_gold_tables(ctx);
  if (r != SRSGPU_OK) {
    return r;
  }
  const uint32_t         nsc = 12u * grid_nof_prb;
  std::vector<mod_desc>  descs(nof_tx);
  std::vector<mod_chunk> chunks;
  std::vector<uint16_t>  sc_map;  // RE -> grid subcarrier of every general allocation
  std::vector<float>     prg_w;   // per-PRG weights of every transmission with PRG precoding
  std::vector<uint16_t>  sc_tx;
  for (uint32_t t = 0; t < nof_tx; ++t) {
    const srsgpu_pdsch_mod_config& c  = cfgs[t];
    const srsgpu_alloc_ext*        x  = (exts != nullptr) ? &exts[t] : nullptr;
    const unsigned                 qm = c.modulation_order;
    if (qm != 2 && qm != 4 && qm != 6 && qm != 8) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid modulation order %u", t, qm);
    }
    if (c.nof_layers < 1 || c.nof_layers > 4 || c.nof_ports < c.nof_layers || c.nof_ports > grid_nof_ports) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid layers/ports (%u, %u)", t, c.nof_layers, c.nof_ports);
    }
    // pdsch_modulator_impl.cpp:61: the time allocation must not exceed the slot boundary.
    if (c.nof_symbols < 1 || c.start_symbol + c.nof_symbols > 14) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: time allocation [%u, %u) exceeds the slot", t, c.start_symbol,
                  c.start_symbol + c.nof_symbols);
    }
    if ((c.dmrs_type != 1 && c.dmrs_type != 2) || c.nof_cdm_groups_without_data < 1 ||
        c.nof_cdm_groups_without_data > (c.dmrs_type == 1 ? 2 : 3)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid DM-RS type %u / CDM groups without data %u", t,
                  c.dmrs_type, c.nof_cdm_groups_without_data);
    }
    // PRG precoding indexes PRGs by absolute CRB (resource_grid_mapper_impl.cpp:218), so it takes the RE map path too.
    const bool general = x != nullptr && (x->crb_mask != nullptr || x->nof_reserved > 0 || x->prg_size > 0);
    if (c.n_id > 1023 || c.bwp_size_rb < 1 || c.bwp_start_rb + c.bwp_size_rb > grid_nof_prb ||
        (!general && (c.nof_rb < 1 || c.rb_start + c.nof_rb > c.bwp_size_rb))) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: allocation outside the BWP or the grid, or n_id > 1023", t);
    }
    if (x != nullptr && ((x->nof_reserved > 0 && x->reserved == nullptr) ||
                         (x->prg_size > 0 && (x->prg_weights == nullptr || x->nof_prg == 0 ||
                                              static_cast<uint32_t>(x->prg_size) * x->nof_prg < grid_nof_prb)))) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid allocation extension (reserved patterns / PRG weights)", t);
    }
    if (c.cw_offset % 4 != 0) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: codeword offset not a multiple of 4", t);
    }
    mod_desc d{};
    // DM-RS RE pattern of a PRB (dmrs_mapping.h): type 1 CDM group g on subcarriers 2k + g, type 2 on 6k + 2g + {0, 1}.
    unsigned nd = 0;
    for (unsigned k = 0; k < 12; ++k) {
      const unsigned group = (c.dmrs_type == 2) ? (k % 6) / 2 : k % 2;
      if (group >= c.nof_cdm_groups_without_data) {
        d.dmrs_lut |= static_cast<uint64_t>(k) << (4 * nd);
        ++nd;
      }
    }
    d.nd_dmrs = static_cast<uint8_t>(nd);
    uint32_t nre = 0;
    d.sc_map     = NO_SC_MAP;
    if (general) {
      // CRB mask (a contiguous allocation when the extension has none) minus the BWP's DM-RS pattern and the
      // reserved patterns (pdsch_modulator_impl.cpp:58-:87).
      std::vector<uint8_t> crbs(grid_nof_prb, 0);
      for (unsigned rb = 0; rb < grid_nof_prb; ++rb) {
        crbs[rb] = (x->crb_mask != nullptr) ? x->crb_mask[rb]
                                            : (rb >= c.bwp_start_rb + c.rb_start &&
                                               rb < static_cast<unsigned>(c.bwp_start_rb + c.rb_start + c.nof_rb));
      }
      enumerate_data_res(grid_nof_prb, crbs.data(), c.start_symbol, c.nof_symbols, c.dmrs_symbol_mask, c.dmrs_type,
                         c.nof_cdm_groups_without_data, c.bwp_start_rb, c.bwp_start_rb + c.bwp_size_rb, x->reserved,
                         x->nof_reserved, sc_tx, d.sym_cum);
      nre      = static_cast<uint32_t>(sc_tx.size());
      d.sc_map = static_cast<uint32_t>(sc_map.size());
      sc_map.insert(sc_map.end(), sc_tx.begin(), sc_tx.end());
    } else {
      for (unsigned l = 0; l < 14; ++l) {
        d.sym_cum[l] = static_cast<uint16_t>(nre);
        if (l >= c.start_symbol && l < static_cast<unsigned>(c.start_symbol + c.nof_symbols)) {
          nre += (((c.dmrs_symbol_mask >> l) & 1u) ? nd : 12u) * c.nof_rb;
        }
      }
      d.sym_cum[14] = static_cast<uint16_t>(nre);
      d.sym_cum[15] = static_cast<uint16_t>(nre);
    }
    const uint64_t need = static_cast<uint64_t>(nre) * c.nof_layers * qm;
    if (nre == 0 || need != c.nof_bits || c.nof_bits > MOD_MAX_BITS) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: codeword of %u bits for %u data REs x %u layers x Qm %u", t,
                  c.nof_bits, nre, c.nof_layers, qm);
    }
    d.cw_word_offset = c.cw_offset / 4;
    d.nof_bits       = c.nof_bits;
    d.c_init         = (static_cast<uint32_t>(c.rnti) << 15) + c.n_id;  // pdsch_modulator_impl.cpp:35, q = 0
    d.port_stride    = 14u * nsc;
    d.nsc            = nsc;
    d.grid_base      = c.grid_index * grid_nof_ports * 14u * nsc + (general ? 0u : (c.bwp_start_rb + c.rb_start) * 12u);
    d.dmrs_mask      = c.dmrs_symbol_mask;
    d.qm             = static_cast<uint8_t>(qm);
    d.L              = c.nof_layers;
    d.P              = c.nof_ports;
    // Modulation amplitude times the power scaling, folded into the precoding weights (pdsch_modulator_impl.cpp:93).
    float amp = modulation_amplitude(qm);
    if (std::isnormal(c.scaling)) {
      amp *= c.scaling;
    }
    for (int p = 0; p < 4; ++p) {
      for (int l = 0; l < 4; ++l) {
        const bool used = p < c.nof_ports && l < c.nof_layers;
        d.w[p][l][0]    = used ? c.precoding[p][l][0] * amp : 0.f;
        d.w[p][l][1]    = used ? c.precoding[p][l][1] * amp : 0.f;
      }
    }
    d.prg_sc = 0;
    if (x != nullptr && x->prg_size > 0) {
      // Per-PRG weights, the same amplitude folding (precoding2 *= scaling, pdsch_modulator_impl.cpp:96).
      d.prg_sc = static_cast<uint16_t>(x->prg_size * 12u);
      d.prg_w  = static_cast<uint32_t>(prg_w.size());
      for (unsigned g = 0; g < x->nof_prg; ++g) {
        for (int p = 0; p < 4; ++p) {
          for (int l = 0; l < 4; ++l) {
            const bool   used = p < c.nof_ports && l < c.nof_layers;
            const float* src  = x->prg_weights + ((static_cast<size_t>(g) * c.nof_ports + p) * c.nof_layers + l) * 2;
            prg_w.push_back(used ? src[0] * amp : 0.f);
            prg_w.push_back(used ? src[1] * amp : 0.f);
          }
        }
      }
    }
    descs[t]              = d;
    const uint32_t Lq     = static_cast<uint32_t>(c.nof_layers) * qm;
    const uint32_t nwords = (c.nof_bits + 31) / 32;
    for (uint32_t w0 = 0; w0 < nwords; w0 += MOD_CHUNK_WORDS) {
      const uint32_t b0 = w0 * 32, b1 = b0 + MOD_CHUNK_WORDS * 32;
      mod_chunk      ch{};
      ch.tx       = t;
      ch.word0    = w0;
      ch.re_begin = (b0 + Lq - 1) / Lq;
      ch.re_end   = std::min(nre, (b1 + Lq - 1) / Lq);
      if (ch.re_end > ch.re_begin) {
        chunks.push_back(ch);
      }
    }
  }
  std::vector<uint32_t> c_inits(descs.size()), nwords(descs.size());
  for (size_t t = 0; t < descs.size(); ++t) {
    c_inits[t] = descs[t].c_init;
    nwords[t]  = (descs[t].nof_bits + 31u) / 32u;
  }
  const std::vector<uint32_t> seq_off = gold_sequence_offsets(nwords);
  for (size_t t = 0; t < descs.size(); ++t) {
    descs[t].seq_word_offset = seq_off[t];
  }
  auto* plan       = new srsgpu_pdsch_modulator_plan();
  plan->ctx        = ctx;
  plan->nof_chunks = static_cast<int>(chunks.size());
  bool ok          = true;
  if (!chunks.empty()) {
    if (build_gold_sequences(ctx, c_inits, nwords, seq_off, &plan->d_seq) != SRSGPU_OK) {
      srsgpu_pdsch_modulator_plan_destroy(plan);
      return SRSGPU_ERR_HIP;
    }
    ok = hipMalloc(&plan->d_desc, descs.size() * sizeof(mod_desc)) == hipSuccess &&
         hipMemcpy(plan->d_desc, descs.data(), descs.size() * sizeof(mod_desc), hipMemcpyHostToDevice) == hipSuccess &&
         hipMalloc(&plan->d_chunks, chunks.size() * sizeof(mod_chunk)) == hipSuccess &&
         hipMemcpy(plan->d_chunks, chunks.data(), chunks.size() * sizeof(mod_chunk), hipMemcpyHostToDevice) ==
             hipSuccess;
    if (ok && !sc_map.empty()) {
      ok = hipMalloc(&plan->d_sc_map, sc_map.size() * sizeof(uint16_t)) == hipSuccess &&
           hipMemcpy(plan->d_sc_map, sc_map.data(), sc_map.size() * sizeof(uint16_t), hipMemcpyHostToDevice) ==
               hipSuccess;
    }
    if (ok && !prg_w.empty()) {
      ok = hipMalloc(&plan->d_prg_w, prg_w.size() * sizeof(float)) == hipSuccess &&
           hipMemcpy(plan->d_prg_w, prg_w.data(), prg_w.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess;
    }
  }
  if (!ok) {
    srsgpu_pdsch_modulator_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload modulator descriptors");
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

int srsgpu_pdsch_modulator_plan_execute(const srsgpu_pdsch_modulator_plan* plan,
                                        const uint8_t*                     d_codewords,
                                        uint32_t*                          d_grids,
                                        void*                              stream)
{
  if (plan == nullptr || d_codewords == nullptr || d_grids == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  launch_pdsch_modulate(plan->d_desc, plan->d_sc_map, plan->d_prg_w, plan->d_chunks, plan->nof_chunks,
                        reinterpret_cast<const uint32_t*>(d_codewords), d_grids, plan->d_seq,
                        static_cast<hipStream_t>(stream));
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

void srsgpu_pdsch_modulator_plan_destroy(srsgpu_pdsch_modulator_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  for (void* p : {static_cast<void*>(plan->d_desc), static_cast<void*>(plan->d_chunks),
                  static_cast<void*>(plan->d_seq), static_cast<void*>(plan->d_sc_map),
                  static_cast<void*>(plan->d_prg_w)}) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  delete plan;
}

int srsgpu_pdsch_dmrs_plan_create(srsgpu_context*                 ctx,
                                  const srsgpu_pdsch_dmrs_config* cfgs,
                                  uint32_t                        nof_tx,
                                  uint32_t                        grid_nof_prb,
                                  uint32_t                        grid_nof_ports,
                                  srsgpu_pdsch_dmrs_plan**        plan_out)
{
  return srsgpu_pdsch_dmrs_plan_create_ex(ctx, cfgs, nullptr, nof_tx, grid_nof_prb, grid_nof_ports, plan_out);
}

int srsgpu_pdsch_dmrs_plan_create_ex(srsgpu_context*                 ctx,
                                     const srsgpu_pdsch_dmrs_config* cfgs,
                                     const srsgpu_alloc_ext*         exts,
                                     uint32_t                        nof_tx,
                                     uint32_t                        grid_nof_prb,
                                     uint32_t                        grid_nof_ports,
                                     srsgpu_pdsch_dmrs_plan**        plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_tx > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (grid_nof_prb == 0 || grid_nof_prb > 275 || grid_nof_ports == 0 || grid_nof_ports > 4) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid grid geometry (%u PRB, %u ports)", grid_nof_prb, grid_nof_ports);
  }
  const uint32_t        nsc = 12u * grid_nof_prb;
  std::vector<dmrs_job> jobs;
  for (uint32_t t = 0; t < nof_tx; ++t) {
    const srsgpu_pdsch_dmrs_config& c = cfgs[t];
    const srsgpu_alloc_ext*         x = (exts != nullptr) ? &exts[t] : nullptr;
    if (x != nullptr && (x->nof_reserved > 0 || x->prg_size > 0)) {
      // dmrs_pdsch_processor_impl.cpp:149 builds each CDM group's precoding with one PRG (more PRGs assert there).
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: PDSCH DM-RS takes a CRB mask only (no reserved REs or PRGs)", t);
    }
    // Allocated CRB intervals (dmrs_helper.cpp dmrs_sequence_generate for_each_interval over rb_mask).
    std::vector<std::pair<unsigned, unsigned>> runs;
    if (x != nullptr && x->crb_mask != nullptr) {
      for (unsigned rb = 0; rb < grid_nof_prb;) {
        if (x->crb_mask[rb] == 0) {
          ++rb;
          continue;
        }
        unsigned e = rb;
        while (e < grid_nof_prb && x->crb_mask[e] != 0) {
          ++e;
        }
        runs.emplace_back(rb, e);
        rb = e;
      }
    } else if (c.nof_rb >= 1 && c.rb_start + c.nof_rb <= grid_nof_prb) {
      runs.emplace_back(c.rb_start, c.rb_start + c.nof_rb);
    }
    if (c.nof_layers < 1 || c.nof_layers > 4 || c.nof_ports < c.nof_layers || c.nof_ports > grid_nof_ports ||
        (c.dmrs_type != 1 && c.dmrs_type != 2) || c.n_scid > 1 || runs.empty() ||
        runs.front().first < c.reference_point_k_rb || (c.dmrs_symbol_mask >> 14)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tx %u: invalid DM-RS configuration", t);
    }
    const uint32_t per_rb = c.dmrs_type == 2 ? 4 : 6;
    for (unsigned l = 0; l < 14; ++l) {
      if (((c.dmrs_symbol_mask >> l) & 1u) == 0) {
        continue;
      }
      for (const auto& run : runs) {
        // One job per symbol and CRB interval: the sequence index of CRB n is (n - k_ref) x per RB, and the cover
        // code parity of a DM-RS RE is that of its index within the PRB (per RB is even).
        dmrs_job       jb{};
        const uint64_t nid = c.scrambling_id;
        jb.grid_base   = c.grid_index * grid_nof_ports * 14u * nsc + l * nsc + run.first * 12u;
        jb.port_stride = 14u * nsc;
        jb.c_init      = static_cast<uint32_t>(
            ((14ull * c.slot_index + l + 1) * (2 * nid + 1) * (1ull << 17) + 2 * nid + c.n_scid) % (1ull << 31));
        jb.seq_offset = (run.first - c.reference_point_k_rb) * per_rb;
        jb.amp        = static_cast<float>(M_SQRT1_2) * c.amplitude;  // dmrs_pdsch_processor_impl.cpp:61
        for (int p = 0; p < 4; ++p) {
          for (int q = 0; q < 4; ++q) {
            const bool used = p < c.nof_ports && q < c.nof_layers;
            jb.w[p][q][0]   = used ? c.precoding[p][q][0] : 0.f;
            jb.w[p][q][1]   = used ? c.precoding[p][q][1] : 0.f;
          }
        }
        jb.nof_pilots = static_cast<uint16_t>((run.second - run.first) * per_rb);
        jb.type2      = c.dmrs_type == 2;
        jb.L          = c.nof_layers;
        jb.P          = c.nof_ports;
        jb.lp         = (l > 0 && ((c.dmrs_symbol_mask >> (l - 1)) & 1u)) ? 1 : 0;
        jobs.push_back(jb);
      }
    }
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  int r = ensure_gold_tables(ctx);
  if (r != SRSGPU_OK) {
    return r;
  }
  auto* plan     = new srsgpu_pdsch_dmrs_plan();
  plan->ctx      = ctx;
  plan->nof_jobs = static_cast<int>(jobs.size());
  for (const dmrs_job& j : jobs) {
    plan->max_pilots = std::max(plan->max_pilots, static_cast<int>(j.nof_pilots));
  }
  // Resident sequence words of every job, filled once.
  std::vector<uint32_t> c_inits, nwords, offsets, wstart;
  uint32_t              base = 0;
  for (dmrs_job& jb : jobs) {
    const uint32_t n0 = 2u * jb.seq_offset;
    const uint32_t nw = ((n0 & 31u) + 2u * jb.nof_pilots + 31u) >> 5;
    jb.gseq_base      = base;
    c_inits.push_back(jb.c_init);
    nwords.push_back(nw);
    offsets.push_back(base);
    wstart.push_back(n0 >> 5);
    base += nw;
  }
  if (build_gold_sequences(ctx, c_inits, nwords, offsets, &plan->d_seq, &wstart) != SRSGPU_OK) {
    srsgpu_pdsch_dmrs_plan_destroy(plan);
    return SRSGPU_ERR_HIP;
  }
  if (!jobs.empty() && (hipMalloc(&plan->d_jobs, jobs.size() * sizeof(dmrs_job)) != hipSuccess ||
                        hipMemcpy(plan->d_jobs, jobs.data(), jobs.size() * sizeof(dmrs_job), hipMemcpyHostToDevice) !=
                            hipSuccess)) {
    srsgpu_pdsch_dmrs_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload DM-RS jobs");
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

int srsgpu_pdsch_dmrs_plan_execute(const srsgpu_pdsch_dmrs_plan* plan, uint32_t* d_grids, void* stream)
{
  if (plan == nullptr || d_grids == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  launch_pdsch_dmrs(plan->d_jobs, plan->nof_jobs, plan->max_pilots, d_grids, plan->d_seq, static_cast<hipStream_t>(stream));
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

void srsgpu_pdsch_dmrs_plan_destroy(srsgpu_pdsch_dmrs_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  if (plan->d_jobs != nullptr) {
    (void)hipFree(plan->d_jobs);
  }
  if (plan->d_seq != nullptr) {
    (void)hipFree(plan->d_seq);
  }
  delete plan;
}

} // extern "C"
