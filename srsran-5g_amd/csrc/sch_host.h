// Host-side SCH segmentation (TS 38.212 §5.2.2 / §5.4.2.1): C++ mirror of the reference's
// ldpc_segmenter_tx_impl::new_transmission (lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.cpp:58),
// ldpc::compute_lifting_size (include/srsran/phy/upper/channel_coding/ldpc/ldpc.h:166) and compute_rm_length
// (ldpc_segmenter_helpers.h:75). Same arithmetic as srsran-5g_amd/srsgpu/sch.py (pinned against the reference).
#pragma once

#include "ldpc_base_graphs.h"
#include <string>
#include <vector>

namespace srsgpu {

struct cb_segment {
  int E;           ///< Rate-matched length.
  int cw_offset;   ///< First codeword bit of the codeblock.
  int tb_offset;   ///< First TB(+TB CRC) bit carried.
  int nof_data;    ///< TB(+TB CRC for the last codeblock) bits carried.
  int used;        ///< Bits covered by the codeblock CRC (data + zero padding).
};

struct tb_segmentation {
  int                     tbs        = 0;  ///< Transport block size in bits.
  int                     bg         = 1;
  int                     C          = 1;  ///< Number of codeblocks.
  int                     Z          = 2;
  int                     K          = 0;  ///< Codeblock message length (22 Z or 10 Z).
  int                     filler     = 0;
  int                     tb_crc_len = 16;
  int                     cb_crc_len = 0;  ///< 24 if segmented, else 0.
  int                     zero_pad   = 0;
  int                     cw_length  = 0;  ///< G.
  std::vector<cb_segment> cbs;
};

inline bool sch_segment(int tbs, int bg, int qm, int nof_layers, int nof_ch_symbols, tb_segmentation& s,
                        std::string& err)
{
  if (tbs <= 0 || tbs % 8 != 0 || tbs + 24 > 1277992 + 24) {
    err = "invalid transport block size";
    return false;
  }
  if (bg != 1 && bg != 2) {
    err = "invalid base graph";
    return false;
  }
  if (nof_layers < 1 || nof_layers > 4 || nof_ch_symbols <= 0 || nof_ch_symbols % nof_layers != 0) {
    err = "the number of channel symbols must be a multiple of the number of layers";
    return false;
  }
  s.tbs            = tbs;
  s.bg             = bg;
  s.tb_crc_len     = (tbs <= 3824) ? 16 : 24;
  const int b_in   = tbs + s.tb_crc_len;
  const int maxseg = (bg == 1) ? 8448 : 3840;
  s.C              = (b_in <= maxseg) ? 1 : (b_in + (maxseg - 24) - 1) / (maxseg - 24);
  const int b_out  = b_in + (s.C > 1 ? 24 * s.C : 0);
  int       kb     = 22;
  if (bg == 2) {
    kb = (b_in > 640) ? 10 : (b_in > 560) ? 9 : (b_in > 192) ? 8 : 6;
  }
  s.Z = 0;
  for (int z : kLiftingSizes) {
    if (z * kb * s.C >= b_out) {
      s.Z = z;
      break;
    }
  }
  if (s.Z == 0) {
    err = "lifting size cannot be 0";
    return false;
  }
  s.K                 = ((bg == 1) ? 22 : 10) * s.Z;
  s.cb_crc_len        = (s.C > 1) ? 24 : 0;
  const int cb_info   = (b_out + s.C - 1) / s.C - s.cb_crc_len;
  s.zero_pad          = (cb_info + s.cb_crc_len) * s.C - b_out;
  const int sym_layer = nof_ch_symbols / nof_layers;
  const int nof_short = s.C - (sym_layer % s.C);
  s.filler            = s.K - cb_info - s.cb_crc_len;
  s.cw_length         = nof_ch_symbols * qm;
  s.cbs.clear();
  int cw = 0, tb = 0;
  for (int i = 0; i < s.C; ++i) {
    const bool last = (i == s.C - 1);
    cb_segment c{};
    c.E         = ((i < nof_short) ? sym_layer / s.C : (sym_layer + s.C - 1) / s.C) * nof_layers * qm;
    c.cw_offset = cw;
    c.tb_offset = tb;
    c.nof_data  = cb_info - (last ? s.zero_pad : 0);  // includes the TB CRC for the last codeblock
    c.used      = cb_info;
    s.cbs.push_back(c);
    tb += c.nof_data;
    cw += c.E;
  }
  if (tb != b_in || cw != s.cw_length) {
    err = "inconsistent segmentation";
    return false;
  }
  return true;
}

} // namespace srsgpu
