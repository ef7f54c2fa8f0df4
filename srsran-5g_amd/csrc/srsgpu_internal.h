// Internal (host <-> device) descriptors of the srsgpu PHY library. Not part of the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace srsgpu {

/// Number of bytes between consecutive lifted-node columns of the soft-bit image in LDS. A fixed stride (the maximum
/// lifting size) turns every column offset into an instruction immediate.
constexpr int SOFT_COL_STRIDE = 384;

/// Marks "no CRC early stop".
constexpr uint32_t NO_CRC_TABLE = 0xffffffffu;

/// Per-codeblock work item of the LDPC decoder (32 bytes, uploaded once per batch).
struct dec_desc {
  uint32_t llr_offset;   ///< First LLR of the codeblock in the batch LLR buffer.
  uint32_t nof_llr;      ///< Number of input LLRs (input.size() of ldpc_decoder::decode).
  uint32_t out_offset;   ///< Byte offset of the packed K*Z-bit output (MSB first, like srsran::bit_buffer).
  uint32_t crc_table;    ///< Element offset of the CRC contribution table, or NO_CRC_TABLE.
  uint32_t div_magic;    ///< ceil(2^32 / Z): exact i / Z for i < 2^16 via __umulhi.
  uint16_t Z;            ///< Lifting size.
  uint16_t zpos;         ///< Position of Z in the list of lifting sizes (row of the shift table).
  uint16_t nof_significant;  ///< K*Z - filler bits: length of the CRC-protected message.
  uint16_t max_iter;     ///< Maximum number of min-sum iterations.
  uint32_t sf16;         ///< Scaling factor as 16-bit fixed point (SIMD mode), 65536 for "no scaling".
  float    sf;           ///< Scaling factor (generic mode).
  uint32_t cb_index : 24;  ///< Index of the codeblock in the caller's batch (result slot).
  uint32_t flags : 8;      ///< DEC_FLAG_* bits.
};
static_assert(sizeof(dec_desc) == 40, "dec_desc layout");

/// dec_desc::flags: check the CRC after every iteration (early stop) instead of once after max_iter.
constexpr uint32_t DEC_FLAG_EARLY_STOP = 1u;

/// Per-codeblock work item of the rate dematcher (rate_dematcher.hip).
struct dm_desc {
  uint32_t llr_offset;   ///< First of the E rate-matched LLRs in the codeword LLR buffer.
  uint32_t harq_offset;  ///< First of the N LLRs of the codeblock's HARQ soft buffer.
  uint32_t E;            ///< Rate-matched length.
  uint32_t N;            ///< Full codeblock length N_short * Z.
  uint32_t Ncb;          ///< Circular buffer length (LBRM).
  uint32_t nsys;         ///< (K - 2) * Z systematic bits (with fillers).
  uint32_t v0;           ///< Index of k0 among the non-filler positions.
  uint16_t nof_filler;   ///< Filler bits.
  uint8_t  Qm;           ///< Modulation order.
  uint8_t  new_data;     ///< First transmission: copy instead of combine.
  uint32_t skip;         ///< Non-zero: leave this codeblock's buffer untouched.
};
static_assert(sizeof(dm_desc) == 36, "dm_desc layout");

/// Launches the batched rate dematcher (rate_dematcher.hip). mode 0: generic combining, 1: SIMD combining.
void launch_rate_dematch(int mode, const dm_desc* d_desc, int nof_cbs, const int8_t* d_llrs, int8_t* d_harq,
                         hipStream_t stream);

/// Launches the batched LDPC decoder (ldpc_decoder.hip).
void launch_ldpc_decode(int                bg,
                        int                mode,
                        const dec_desc*    d_desc,
                        int                nof_cbs,
                        int                block_threads,
                        const int8_t*      d_llrs,
                        uint8_t*           d_out,
                        int32_t*           d_results,
                        const uint16_t*    d_shifts,
                        const uint32_t*    d_crc_tables,
                        uint8_t*           d_cb_crc_ok,
                        hipStream_t        stream);

} // namespace srsgpu
