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
  uint32_t cb_index;     ///< Index of the codeblock in the caller's batch (result slot).
};
static_assert(sizeof(dec_desc) == 40, "dec_desc layout");

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
                        hipStream_t        stream);

} // namespace srsgpu
