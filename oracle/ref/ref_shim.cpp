// TEST INFRASTRUCTURE ONLY - never linked into the product.
//
// C-ABI shim over the srsRAN reference classes, compiled together with the reference's own source files (read in
// place from /root/reference by oracle/build_ref.sh) into oracle/_ref/libsrsref.so.  It lets the parity tests pin the
// C restatement in oracle/oracle.c against the real reference and generate the golden fixtures in tests/golden/.
//
// Classes driven here (reference file:line):
//   ldpc_decoder_generic / _avx2 / _avx512   lib/phy/upper/channel_coding/ldpc/ldpc_decoder_impl.cpp:64 (decode)
//   ldpc_encoder_generic / _avx2             lib/phy/upper/channel_coding/ldpc/ldpc_encoder_impl.cpp:42 (encode)
//   ldpc_rate_matcher_impl                   lib/phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.cpp:95
//   ldpc_rate_dematcher_impl (+avx2/avx512)  lib/phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_impl.cpp:46
//   ldpc_segmenter_tx_impl                   lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.cpp:51
//   crc_calculator_generic_impl              lib/phy/upper/channel_coding/crc_calculator_generic_impl.cpp:64
#include "crc_calculator_generic_impl.h"
#include "ldpc/ldpc_decoder_avx2.h"
#include "ldpc/ldpc_decoder_avx512.h"
#include "ldpc/ldpc_decoder_generic.h"
#include "ldpc/ldpc_encoder_avx2.h"
#include "ldpc/ldpc_encoder_generic.h"
#include "ldpc/ldpc_graph_impl.h"
#include "ldpc/ldpc_luts_impl.h"
#include "ldpc/ldpc_rate_dematcher_avx2_impl.h"
#include "ldpc/ldpc_rate_dematcher_impl.h"
#include "ldpc/ldpc_rate_matcher_impl.h"
#include "ldpc/ldpc_segmenter_tx_impl.h"
#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc_encoder_buffer.h"
#include "srsran/srsvec/bit.h"
#include <memory>
#include <vector>

using namespace srsran;

namespace {

crc_generator_poly to_poly(int p)
{
  return static_cast<crc_generator_poly>(p);
}

std::unique_ptr<ldpc_decoder> make_decoder(int impl)
{
  switch (impl) {
    case 1:
      return std::make_unique<ldpc_decoder_avx2>();
    case 2:
      return std::make_unique<ldpc_decoder_avx512>();
    default:
      return std::make_unique<ldpc_decoder_generic>();
  }
}

modulation_scheme to_mod(int qm)
{
  switch (qm) {
    case 1:
      return modulation_scheme::BPSK;
    case 2:
      return modulation_scheme::QPSK;
    case 4:
      return modulation_scheme::QAM16;
    case 6:
      return modulation_scheme::QAM64;
    default:
      return modulation_scheme::QAM256;
  }
}

ldpc_base_graph_type to_bg(int bg)
{
  return bg == 2 ? ldpc_base_graph_type::BG2 : ldpc_base_graph_type::BG1;
}

} // namespace

extern "C" {

int ref_cpu_has_avx512()
{
  return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
}

/// CRC over an unpacked bit sequence (one bit per byte).
unsigned ref_crc_bits(int poly, const uint8_t* bits, unsigned nbits)
{
  crc_calculator_generic_impl crc(to_poly(poly));
  return crc.calculate_bit(span<const uint8_t>(bits, nbits));
}

/// CRC over packed bytes.
unsigned ref_crc_bytes(int poly, const uint8_t* bytes, unsigned nbytes)
{
  crc_calculator_generic_impl crc(to_poly(poly));
  return crc.calculate_byte(span<const uint8_t>(bytes, nbytes));
}

/// Dumps the lifted parity-check matrix (shift or 0xffff) for (bg, Z) as an M x N_full row-major array, and the
/// adjacency rows (M x 20).
int ref_ldpc_graph(int bg, int Z, uint16_t* matrix, uint16_t* adjacency)
{
  auto ls = static_cast<ldpc::lifting_size_t>(Z);
  if (ldpc::get_lifting_index(ls) == ldpc::VOID_LIFTSIZE) {
    return -1;
  }
  ldpc_graph_impl g(to_bg(bg), ls);
  unsigned        M = g.get_nof_BG_check_nodes();
  unsigned        N = g.get_nof_BG_var_nodes_full();
  for (unsigned m = 0; m != M; ++m) {
    for (unsigned n = 0; n != N; ++n) {
      matrix[m * N + n] = g.get_lifted_node(m, n);
    }
    const auto& row = g.get_adjacency_row(m);
    for (unsigned e = 0; e != ldpc::MAX_BG_CHECK_EDGES; ++e) {
      adjacency[m * ldpc::MAX_BG_CHECK_EDGES + e] = row[e];
    }
  }
  return static_cast<int>(ldpc::get_lifting_index(ls));
}

/// LDPC encoding of a message (K*Z unpacked bits). Writes the full shortened codeblock (N_short*Z unpacked bits).
int ref_ldpc_encode(int impl, int bg, int Z, const uint8_t* msg, uint8_t* cb)
{
  std::unique_ptr<ldpc_encoder> enc;
  if (impl == 1) {
    enc = std::make_unique<ldpc_encoder_avx2>();
  } else {
    enc = std::make_unique<ldpc_encoder_generic>();
  }
  unsigned           K = (bg == 2) ? 10 : 22;
  unsigned           N = (bg == 2) ? 50 : 66;
  dynamic_bit_buffer in(K * Z);
  srsvec::bit_pack(in, span<const uint8_t>(msg, K * Z));
  codeblock_metadata::tb_common_metadata cfg;
  cfg.base_graph                 = to_bg(bg);
  cfg.lifting_size               = static_cast<ldpc::lifting_size_t>(Z);
  const ldpc_encoder_buffer& buf = enc->encode(in, cfg);
  buf.write_codeblock(span<uint8_t>(cb, N * Z), 0);
  return 0;
}

/// LDPC decoding. Returns the number of iterations on success (CRC early stop), -1 otherwise. `out` receives the
/// K*Z decoded bits unpacked. crc_poly < 0 disables early stopping.
int ref_ldpc_decode(int      impl,
                    int      bg,
                    int      Z,
                    int      nof_crc_bits,
                    int      nof_filler_bits,
                    int      crc_poly,
                    int      max_iter,
                    float    scaling,
                    const int8_t* llr,
                    unsigned n_llr,
                    uint8_t* out)
{
  auto                      dec = make_decoder(impl);
  unsigned                  K   = (bg == 2) ? 10 : 22;
  dynamic_bit_buffer        msg(K * Z);
  std::unique_ptr<crc_calculator> crc;
  if (crc_poly >= 0) {
    crc = std::make_unique<crc_calculator_generic_impl>(to_poly(crc_poly));
  }
  // Pre-fill with the caller's bytes so untouched outputs are observable.
  srsvec::bit_pack(msg, span<const uint8_t>(out, K * Z));
  ldpc_decoder::configuration cfg;
  cfg.block_conf.tb_common.base_graph     = to_bg(bg);
  cfg.block_conf.tb_common.lifting_size   = static_cast<ldpc::lifting_size_t>(Z);
  cfg.block_conf.cb_specific.nof_crc_bits = nof_crc_bits;
  cfg.block_conf.cb_specific.nof_filler_bits = nof_filler_bits;
  cfg.algorithm_conf.max_iterations          = max_iter;
  cfg.algorithm_conf.scaling_factor          = scaling;
  span<const log_likelihood_ratio> in(reinterpret_cast<const log_likelihood_ratio*>(llr), n_llr);
  std::optional<unsigned>          r = dec->decode(msg, in, crc.get(), cfg);
  srsvec::bit_unpack(span<uint8_t>(out, K * Z), msg);
  return r.has_value() ? static_cast<int>(*r) : -1;
}

/// Rate matching of the codeblock obtained by encoding `msg` (K*Z unpacked bits, filler bits set to 0).
/// Writes E unpacked output bits.
int ref_rate_match(int bg, int Z, int rv, int qm, unsigned Nref, unsigned nof_filler, const uint8_t* msg,
                   unsigned E, uint8_t* out)
{
  ldpc_encoder_generic enc;
  unsigned             K = (bg == 2) ? 10 : 22;
  dynamic_bit_buffer   in(K * Z);
  srsvec::bit_pack(in, span<const uint8_t>(msg, K * Z));
  codeblock_metadata cfg;
  cfg.tb_common.base_graph          = to_bg(bg);
  cfg.tb_common.lifting_size        = static_cast<ldpc::lifting_size_t>(Z);
  cfg.tb_common.rv                  = rv;
  cfg.tb_common.mod                 = to_mod(qm);
  cfg.tb_common.Nref                = Nref;
  cfg.cb_specific.nof_filler_bits   = nof_filler;
  cfg.cb_specific.rm_length         = E;
  const ldpc_encoder_buffer& buf    = enc.encode(in, cfg.tb_common);
  ldpc_rate_matcher_impl     rm;
  dynamic_bit_buffer         packed(E);
  rm.rate_match(packed, buf, cfg);
  srsvec::bit_unpack(span<uint8_t>(out, E), packed);
  return 0;
}

/// Rate dematching of E LLRs into a buffer of N_short*Z LLRs (in/out: combined when new_data == 0).
int ref_rate_dematch(int impl, int bg, int Z, int rv, int qm, unsigned Nref, unsigned nof_filler, int new_data,
                     const int8_t* llr, unsigned E, int8_t* buf)
{
  std::unique_ptr<ldpc_rate_dematcher> rdm;
  if (impl == 1) {
    rdm = std::make_unique<ldpc_rate_dematcher_avx2_impl>();
  } else {
    rdm = std::make_unique<ldpc_rate_dematcher_impl>();
  }
  unsigned           N = (bg == 2) ? 50 : 66;
  codeblock_metadata cfg;
  cfg.tb_common.base_graph        = to_bg(bg);
  cfg.tb_common.lifting_size      = static_cast<ldpc::lifting_size_t>(Z);
  cfg.tb_common.rv                = rv;
  cfg.tb_common.mod               = to_mod(qm);
  cfg.tb_common.Nref              = Nref;
  cfg.cb_specific.nof_filler_bits = nof_filler;
  cfg.cb_specific.rm_length       = E;
  rdm->rate_dematch(span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(buf), N * Z),
                    span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llr), E),
                    new_data != 0,
                    cfg);
  return 0;
}

/// Full PDSCH codeword encoding (segmentation + CRCs + LDPC + rate matching), as pdsch_encoder_impl::encode does
/// (lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp:28). Writes nof_ch_symbols*qm unpacked bits.
/// Also reports the segmentation: cb_meta[i*4 + {0,1,2,3}] = {Z, nof_filler, rm_length, cb_info_bits}.
int ref_pdsch_encode(int bg, int rv, int qm, int nof_layers, unsigned Nref, unsigned nof_ch_symbols,
                     const uint8_t* tb, unsigned tb_bytes, uint8_t* codeword, unsigned* cb_meta)
{
  ldpc_segmenter_tx_impl::sch_crc crcs{std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16),
                                       std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A),
                                       std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B)};
  ldpc_segmenter_tx_impl seg(crcs);
  segmenter_config       scfg;
  scfg.base_graph     = to_bg(bg);
  scfg.rv             = rv;
  scfg.mod            = to_mod(qm);
  scfg.Nref           = Nref;
  scfg.nof_layers     = nof_layers;
  scfg.nof_ch_symbols = nof_ch_symbols;
  span<const uint8_t>          tbs(tb, tb_bytes);
  const ldpc_segmenter_buffer& sb = seg.new_transmission(tbs, scfg);
  ldpc_encoder_generic         enc;
  ldpc_rate_matcher_impl       rm;
  dynamic_bit_buffer           cb_data(sb.get_segment_length().value());
  unsigned                     offset = 0;
  for (unsigned i = 0, n = sb.get_nof_codeblocks(); i != n; ++i) {
    codeblock_metadata md = sb.get_cb_metadata(i);
    sb.read_codeblock(cb_data, tbs, i);
    const ldpc_encoder_buffer& buf = enc.encode(cb_data, md.tb_common);
    unsigned                   E   = sb.get_rm_length(i);
    dynamic_bit_buffer         packed(E);
    rm.rate_match(packed, buf, md);
    srsvec::bit_unpack(span<uint8_t>(codeword + offset, E), packed);
    offset += E;
    if (cb_meta != nullptr) {
      cb_meta[i * 4 + 0] = static_cast<unsigned>(md.tb_common.lifting_size);
      cb_meta[i * 4 + 1] = md.cb_specific.nof_filler_bits;
      cb_meta[i * 4 + 2] = E;
      cb_meta[i * 4 + 3] = sb.get_cb_info_bits(i).value();
    }
  }
  return static_cast<int>(sb.get_nof_codeblocks());
}

} // extern "C"

#include <chrono>

extern "C" {

/// CPU baseline: decodes n codeblocks (LLRs at llr + i * stride, same configuration) with ONE reference decoder
/// instance of the given implementation and returns the wall time of the decode() calls only, in nanoseconds.
/// iters[i] receives the return value (iterations or -1).
long long ref_ldpc_decode_timed(int           impl,
                                int           bg,
                                int           Z,
                                int           nof_crc_bits,
                                int           nof_filler_bits,
                                int           crc_poly,
                                int           max_iter,
                                float         scaling,
                                const int8_t* llr,
                                unsigned      n_llr,
                                unsigned      stride,
                                unsigned      n,
                                int*          iters)
{
  auto                            dec = make_decoder(impl);
  unsigned                        K   = (bg == 2) ? 10 : 22;
  dynamic_bit_buffer              msg(K * Z);
  std::unique_ptr<crc_calculator> crc;
  if (crc_poly >= 0) {
    crc = std::make_unique<crc_calculator_generic_impl>(to_poly(crc_poly));
  }
  ldpc_decoder::configuration cfg;
  cfg.block_conf.tb_common.base_graph        = to_bg(bg);
  cfg.block_conf.tb_common.lifting_size      = static_cast<ldpc::lifting_size_t>(Z);
  cfg.block_conf.cb_specific.nof_crc_bits    = nof_crc_bits;
  cfg.block_conf.cb_specific.nof_filler_bits = nof_filler_bits;
  cfg.algorithm_conf.max_iterations          = max_iter;
  cfg.algorithm_conf.scaling_factor          = scaling;
  auto t0                                    = std::chrono::steady_clock::now();
  for (unsigned i = 0; i != n; ++i) {
    span<const log_likelihood_ratio> in(reinterpret_cast<const log_likelihood_ratio*>(llr + static_cast<size_t>(i) * stride),
                                        n_llr);
    std::optional<unsigned> r = dec->decode(msg, in, crc.get(), cfg);
    iters[i]                  = r.has_value() ? static_cast<int>(*r) : -1;
  }
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
}

} // extern "C"

#include "ldpc/ldpc_rate_dematcher_avx512_impl.h"

extern "C" {

int ref_cpu_has_avx512vbmi()
{
  return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
         __builtin_cpu_supports("avx512vbmi");
}

/// CPU baseline, DL leg: pdsch_encoder_impl::encode (pdsch_encoder_impl.cpp:28) of n transport blocks with one set
/// of reference objects (segmenter, encoder of the given implementation, rate matcher), codeword unpacked one bit per
/// byte like the reference. Returns the wall time of the encode loop in nanoseconds.
long long ref_pdsch_encode_slot_timed(int             enc_impl,
                                      unsigned        n,
                                      const int*      bg,
                                      const int*      qm,
                                      const int*      layers,
                                      const unsigned* nsym,
                                      const unsigned* tb_bytes,
                                      const uint8_t*  tbs,
                                      uint8_t*        cw_out)
{
  ldpc_segmenter_tx_impl::sch_crc crcs{std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16),
                                       std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A),
                                       std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B)};
  ldpc_segmenter_tx_impl        seg(crcs);
  std::unique_ptr<ldpc_encoder> enc;
  if (enc_impl == 1) {
    enc = std::make_unique<ldpc_encoder_avx2>();
  } else {
    enc = std::make_unique<ldpc_encoder_generic>();
  }
  ldpc_rate_matcher_impl rm;
  dynamic_bit_buffer     cb_data(8448);
  dynamic_bit_buffer     packed(22 * 384 * 35);
  auto                   t0     = std::chrono::steady_clock::now();
  size_t                 tb_off = 0, cw_off = 0;
  for (unsigned t = 0; t != n; ++t) {
    segmenter_config scfg;
    scfg.base_graph     = to_bg(bg[t]);
    scfg.rv             = 0;
    scfg.mod            = to_mod(qm[t]);
    scfg.Nref           = 0;
    scfg.nof_layers     = layers[t];
    scfg.nof_ch_symbols = nsym[t];
    span<const uint8_t>          tb(tbs + tb_off, tb_bytes[t]);
    const ldpc_segmenter_buffer& sb = seg.new_transmission(tb, scfg);
    cb_data.resize(sb.get_segment_length().value());
    for (unsigned i = 0, nc = sb.get_nof_codeblocks(); i != nc; ++i) {
      codeblock_metadata md = sb.get_cb_metadata(i);
      sb.read_codeblock(cb_data, tb, i);
      const ldpc_encoder_buffer& buf = enc->encode(cb_data, md.tb_common);
      unsigned                   E   = sb.get_rm_length(i);
      packed.resize(E);
      rm.rate_match(packed, buf, md);
      srsvec::bit_unpack(span<uint8_t>(cw_out + cw_off, E), packed);
      cw_off += E;
    }
    tb_off += tb_bytes[t];
  }
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
}

/// CPU baseline, UL leg: the codeblock task of pusch_decoder_impl (pusch_decoder_impl.cpp:283 /
/// pusch_codeblock_decoder.cpp:33) for n codeblocks: rate dematching (new data) + LDPC decoding with CRC early stop.
/// p[i*8 + {0..7}] = {bg, Z, qm, E, filler, crc_poly, nof_crc_bits, llr_offset}. dm_impl: 0 generic, 1 avx2,
/// 2 avx512; dec_impl: 0 generic, 1 avx2, 2 avx512. Returns nanoseconds; iters[i] = iterations or -1.
long long ref_pusch_decode_cbs_timed(int           dm_impl,
                                     int           dec_impl,
                                     unsigned      n,
                                     const int*    p,
                                     const int8_t* llrs,
                                     int           max_iter,
                                     int*          iters)
{
  std::unique_ptr<ldpc_rate_dematcher> rdm;
  if (dm_impl == 2) {
    rdm = std::make_unique<ldpc_rate_dematcher_avx512_impl>();
  } else if (dm_impl == 1) {
    rdm = std::make_unique<ldpc_rate_dematcher_avx2_impl>();
  } else {
    rdm = std::make_unique<ldpc_rate_dematcher_impl>();
  }
  auto                            dec = make_decoder(dec_impl);
  std::unique_ptr<crc_calculator> crc_set[6];
  for (int c = 0; c < 6; ++c) {
    crc_set[c] = std::make_unique<crc_calculator_generic_impl>(to_poly(c));
  }
  std::vector<log_likelihood_ratio> buf(66 * 384);
  dynamic_bit_buffer                msg(22 * 384);
  auto                              t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0; i != n; ++i) {
    const int* q  = p + 8 * i;
    int        bg = q[0], Z = q[1];
    unsigned   N  = (bg == 2 ? 50 : 66) * Z;
    unsigned   K  = (bg == 2 ? 10 : 22) * Z;
    codeblock_metadata md;
    md.tb_common.base_graph        = to_bg(bg);
    md.tb_common.lifting_size      = static_cast<ldpc::lifting_size_t>(Z);
    md.tb_common.rv                = 0;
    md.tb_common.mod               = to_mod(q[2]);
    md.tb_common.Nref              = 0;
    md.cb_specific.rm_length       = q[3];
    md.cb_specific.nof_filler_bits = q[4];
    md.cb_specific.nof_crc_bits    = q[6];
    md.cb_specific.full_length     = N + 2 * Z;
    span<log_likelihood_ratio> b(buf.data(), N);
    rdm->rate_dematch(b,
                      span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs + q[7]), q[3]),
                      true,
                      md);
    ldpc_decoder::configuration cfg;
    cfg.block_conf                    = md;
    cfg.algorithm_conf.max_iterations = max_iter;
    msg.resize(K);
    std::optional<unsigned> r = dec->decode(msg, b, crc_set[q[5]].get(), cfg);
    iters[i]                  = r.has_value() ? static_cast<int>(*r) : -1;
  }
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
}

} // extern "C"
