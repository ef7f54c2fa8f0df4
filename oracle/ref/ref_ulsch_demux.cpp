// TEST INFRASTRUCTURE ONLY: C entry point over the reference's own UL-SCH demultiplexer (ulsch_demultiplex_impl, UCI on
// PUSCH, TS 38.212 section 6.2.7) with the pseudo-random scrambling sequence, compiled from the reference sources by
// oracle/build_ref.sh into oracle/_ref/libsrsref.so. Pins oracle/ulsch_demux_oracle.py; never shipped.
#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_codeword_buffer.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_buffer.h"
#include "srsran/srsvec/bit.h"

#include "lib/phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.h"
#include "lib/phy/upper/sequence_generators/pseudo_random_generator_impl.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <memory>
#include <vector>

using namespace srsran;

namespace {

/// Decoder buffer collecting every soft bit it is given, in order.
class collecting_decoder_buffer : public pusch_decoder_buffer
{
public:
  span<log_likelihood_ratio> get_next_block_view(unsigned block_size) override
  {
    scratch.resize(block_size);
    return scratch;
  }
  void on_new_softbits(span<const log_likelihood_ratio> softbits) override
  {
    data.insert(data.end(), softbits.begin(), softbits.end());
  }
  void on_end_softbits() override
  {
    ended = true;
    if (on_end) {
      on_end();
    }
  }

  std::vector<log_likelihood_ratio> data, scratch;
  bool                              ended = false;
  std::function<void()>             on_end;
};

modulation_scheme mod_from_qm(int qm)
{
  switch (qm) {
    case 1: return modulation_scheme::PI_2_BPSK;
    case 2: return modulation_scheme::QPSK;
    case 4: return modulation_scheme::QAM16;
    case 6: return modulation_scheme::QAM64;
    default: return modulation_scheme::QAM256;
  }
}

int copy_out(const collecting_decoder_buffer& b, int8_t* out, int cap)
{
  const int n = std::min<int>(cap, static_cast<int>(b.data.size()));
  std::memcpy(out, b.data.data(), static_cast<size_t>(n));
  return static_cast<int>(b.data.size());
}

} // namespace

extern "C" {

int ref_ulsch_demux_ex(int qm, int nof_layers, int nof_prb, int start_symbol, int nof_symbols, unsigned dmrs_symbol_mask,
                       int dmrs_type2, int nof_cdm_groups_without_data, int nof_harq_ack_rvd, int nof_harq_ack_bits,
                       int nof_enc_harq_ack_bits, int nof_csi_part1_bits, int nof_enc_csi_part1_bits,
                       int nof_csi_part2_bits, int nof_enc_csi_part2_bits, unsigned c_init, const int8_t* llrs,
                       int nof_llrs, int block_size, int8_t* sch, int8_t* harq, int8_t* csi1, int8_t* csi2, int cap,
                       int* counts, int csi2_after_csi1);

/// Demultiplexes one PUSCH codeword of nof_llrs descrambled LLRs (c_init: its scrambling sequence) fed in blocks of
/// at most block_size soft bits. counts[4] returns the soft bits each buffer received (SCH, HARQ-ACK, CSI Part 1, CSI
/// Part 2); each output holds up to its capacity cap.
int ref_ulsch_demux(int           qm,
                    int           nof_layers,
                    int           nof_prb,
                    int           start_symbol,
                    int           nof_symbols,
                    unsigned      dmrs_symbol_mask,
                    int           dmrs_type2,
                    int           nof_cdm_groups_without_data,
                    int           nof_harq_ack_rvd,
                    int           nof_harq_ack_bits,
                    int           nof_enc_harq_ack_bits,
                    int           nof_csi_part1_bits,
                    int           nof_enc_csi_part1_bits,
                    int           nof_csi_part2_bits,
                    int           nof_enc_csi_part2_bits,
                    unsigned      c_init,
                    const int8_t* llrs,
                    int           nof_llrs,
                    int           block_size,
                    int8_t*       sch,
                    int8_t*       harq,
                    int8_t*       csi1,
                    int8_t*       csi2,
                    int           cap,
                    int*          counts)
{
  return ref_ulsch_demux_ex(qm, nof_layers, nof_prb, start_symbol, nof_symbols, dmrs_symbol_mask, dmrs_type2,
                            nof_cdm_groups_without_data, nof_harq_ack_rvd, nof_harq_ack_bits, nof_enc_harq_ack_bits,
                            nof_csi_part1_bits, nof_enc_csi_part1_bits, nof_csi_part2_bits, nof_enc_csi_part2_bits, c_init,
                            llrs, nof_llrs, block_size, sch, harq, csi1, csi2, cap, counts, 0);
}

/// As ref_ulsch_demux; csi2_after_csi1 != 0: set_csi_part2 is called when the CSI Part 1 buffer ends, as the
/// reference's PUSCH processor does once CSI Part 1 is decoded (pusch_processor_impl.cpp:72-100), instead of before the
/// first symbol.
int ref_ulsch_demux_ex(int           qm,
                       int           nof_layers,
                       int           nof_prb,
                       int           start_symbol,
                       int           nof_symbols,
                       unsigned      dmrs_symbol_mask,
                       int           dmrs_type2,
                       int           nof_cdm_groups_without_data,
                       int           nof_harq_ack_rvd,
                       int           nof_harq_ack_bits,
                       int           nof_enc_harq_ack_bits,
                       int           nof_csi_part1_bits,
                       int           nof_enc_csi_part1_bits,
                       int           nof_csi_part2_bits,
                       int           nof_enc_csi_part2_bits,
                       unsigned      c_init,
                       const int8_t* llrs,
                       int           nof_llrs,
                       int           block_size,
                       int8_t*       sch,
                       int8_t*       harq,
                       int8_t*       csi1,
                       int8_t*       csi2,
                       int           cap,
                       int*          counts,
                       int           csi2_after_csi1)
{
  ulsch_demultiplex::configuration cfg;
  cfg.modulation         = mod_from_qm(qm);
  cfg.nof_layers         = nof_layers;
  cfg.nof_prb            = nof_prb;
  cfg.start_symbol_index = start_symbol;
  cfg.nof_symbols        = nof_symbols;
  cfg.nof_harq_ack_rvd   = nof_harq_ack_rvd;
  cfg.dmrs               = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.dmrs_symbol_mask   = symbol_slot_mask(14);
  for (unsigned l = 0; l != 14; ++l) {
    cfg.dmrs_symbol_mask.set(l, ((dmrs_symbol_mask >> l) & 1U) != 0);
  }
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.nof_harq_ack_bits           = nof_harq_ack_bits;
  cfg.nof_enc_harq_ack_bits       = nof_enc_harq_ack_bits;
  cfg.nof_csi_part1_bits          = nof_csi_part1_bits;
  cfg.nof_enc_csi_part1_bits      = nof_enc_csi_part1_bits;

  collecting_decoder_buffer b_sch, b_harq, b_csi1, b_csi2;
  // Value-initialised like the factories' std::make_unique: ulsch_demultiplex_impl never initialises softbit_count
  // before its first codeword (ulsch_demultiplex_impl.h), so a stack object would start from garbage.
  auto                   demux = std::make_unique<ulsch_demultiplex_impl>();
  pusch_codeword_buffer& cw    = demux->demultiplex(b_sch, b_harq, b_csi1, cfg);
  if (nof_enc_csi_part2_bits > 0) {
    if (csi2_after_csi1 != 0) {
      b_csi1.on_end = [&] { demux->set_csi_part2(b_csi2, nof_csi_part2_bits, nof_enc_csi_part2_bits); };
    } else {
      demux->set_csi_part2(b_csi2, nof_csi_part2_bits, nof_enc_csi_part2_bits);
    }
  }

  pseudo_random_generator_impl prg;
  prg.init(c_init);
  dynamic_bit_buffer seq(nof_llrs);
  prg.generate(seq);

  int pos = 0;
  while (pos < nof_llrs) {
    span<log_likelihood_ratio> view = cw.get_next_block_view(std::min(block_size, nof_llrs - pos));
    for (size_t i = 0; i != view.size(); ++i) {
      view[i] = llrs[pos + static_cast<int>(i)];
    }
    dynamic_bit_buffer block(view.size());
    srsvec::copy_offset(block, 0, seq, pos, view.size());
    cw.on_new_block(view, block);
    pos += static_cast<int>(view.size());
  }
  cw.on_end_codeword();
  counts[0] = copy_out(b_sch, sch, cap);
  counts[1] = copy_out(b_harq, harq, cap);
  counts[2] = copy_out(b_csi1, csi1, cap);
  counts[3] = copy_out(b_csi2, csi2, cap);
  return 0;
}

} // extern "C"
