// Internal (host <-> device) descriptors of the srsgpu PHY library. Not part of the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "srsgpu_phy.h"  // srsgpu_copy_span

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
/// dec_desc::flags: the decoder launch dematches the codeblock itself (a first transmission with a copy-only rate
/// dematching, see ldpc_decode_pk_kernel FUSE); d_llrs is then the codeword LLR buffer and d_dm its dm_desc.
constexpr uint32_t DEC_FLAG_FUSED_DM = 2u;

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
  uint32_t cb_index;     ///< Codeblock index (CRC flag slot).
  uint64_t r_magic;      ///< ceil(2^40 / (E / Qm)): exact n / R as (n * r_magic) >> 40 for n < 2^20.
};
static_assert(sizeof(dm_desc) == 48, "dm_desc layout");

/// CRC job of one transport block (tb_crc_kernel).
struct tb_crc_desc {
  uint32_t byte_offset;  ///< First byte of the transport block.
  uint32_t nbytes;       ///< Transport block size in bytes.
  uint32_t poly;         ///< Generator polynomial including the x^order term (e.g. 0x1864cfb).
  uint32_t order;        ///< 16 or 24.
  uint32_t table;        ///< Per-bit contribution table (CRC arena offset) or NO_CRC_TABLE: byte-table method.
};

/// How the double-diagonal core (rows 0..3, parity columns K..K+3) is solved for one (BG, Z): P^x p0 is the sum of
/// the four row syndromes, then three rows each determine one more parity node.
struct core_plan {
  int16_t x;          ///< Shift of p0 that survives the sum of the core rows.
  int8_t  unk[3];     ///< Parity node solved at each step.
  int8_t  row[3];     ///< Core row used at each step.
  int16_t sh[3][4];   ///< Shifts of the row's parity nodes at each step (-1: no edge).
  // Window offsets of the packed kernel (pdsch_encode_packed_kernel), precomputed mod Z: (Z - x) mod Z for p0; per
  // step (Z - s_u) mod Z for the row sum and (s_j - s_u) mod Z for parity node j (-1: not in the sum).
  int16_t o0;
  int16_t orow[3];
  int16_t oj[3][4];
};
static_assert(sizeof(core_plan) == 64, "core_plan layout");

/// Per-codeblock work item of the PDSCH encoder (pdsch_encode_kernel).
struct enc_desc {
  uint32_t tb_byte_offset;  ///< Transport block start (bytes).
  uint32_t tb_bit_offset;   ///< First TB(+TB CRC) bit carried by the codeblock.
  uint32_t tb_bits;         ///< TBS in bits: stream bits >= tb_bits come from the TB CRC.
  uint32_t out_bit_offset;  ///< First bit of the codeblock in the packed codeword output.
  uint32_t crc_table;       ///< CB CRC24B contribution table (NO_CRC_TABLE: single codeblock, no CB CRC).
  uint32_t div_magic;       ///< ceil(2^32 / Z).
  uint32_t E;               ///< Rate-matched length.
  uint32_t Ncb;             ///< Circular buffer length.
  uint32_t v0;              ///< Index of k0 among the non-filler positions.
  uint32_t tb_index;        ///< Transport block (TB CRC slot).
  uint16_t Z;
  uint16_t zpos;
  uint16_t nof_data;        ///< TB(+TB CRC) bits of the codeblock.
  uint16_t used;            ///< Bits covered by the CB CRC.
  uint16_t filler;
  uint8_t  tb_crc_len;
  uint8_t  Qm;
  uint8_t  n_ext;           ///< Extension parity rows needed by the rate matcher.
  uint8_t  pad[3];
  uint32_t tb_crc_table;    ///< TB CRC contribution table of the TB (inline TB CRC: no tb_crc_desc load).
  uint32_t pad2;
};
static_assert(sizeof(enc_desc) == 64, "enc_desc layout");

/// A byte range [begin, end) of transport block `tb` whose CRC contribution one tb_crc_kernel workgroup computes and
/// XORs into the TB's CRC word (zeroed before the launch): large TBs are spread over many workgroups instead of one.
struct tb_crc_slice {
  uint32_t tb;
  uint32_t begin;
  uint32_t end;
};
/// Slice-by-4 CRC tables in the context (crc_device.h block_crc_slice4): 4 x 256 words per polynomial, in the order
/// CRC24A, CRC24B, CRC16.
constexpr uint32_t CRC_SLICE_WORDS = 1024;
constexpr int      CRC_SLICE_24A   = 0;
constexpr int      CRC_SLICE_24B   = 1;
constexpr int      CRC_SLICE_16    = 2;

/// Slice length (256 lanes x 16-byte chunks); TBs without a contribution table take one slice (byte-table method).
constexpr uint32_t TB_CRC_SLICE_BYTES = 4096;
/// Largest TB whose CRC the packed encoder computes inline (one workgroup per TB); larger ones go to tb_crc_kernel.
constexpr uint32_t TB_CRC_INLINE_MAX_BYTES = 16384;

void launch_tb_crc(const tb_crc_desc*  d_desc,
                   const tb_crc_slice* d_slices,
                   int                 nof_slices,
                   const uint8_t*      d_tbs,
                   uint32_t*           d_crcs,
                   const uint32_t*     d_crc_tables,
                   hipStream_t         s);

void launch_pdsch_encode(int              bg,
                         const enc_desc*  d_desc,
                         int              nof_cbs,
                         int              block_threads,
                         const uint8_t*   d_tbs,
                         const uint32_t*  d_tb_crcs,
                         uint32_t*        d_out_words,
                         const uint16_t*  d_shifts,
                         const core_plan* d_core_plans,
                         const uint32_t*  d_crc_tables,
                         hipStream_t      s);

/// Packed-bit encoder for codeblocks with Z % 32 == 0 and byte-aligned data (pdsch_encode_packed_kernel). With
/// d_tb_inline (the plan's TB CRC descriptors, every one with a contribution table) the codeblock carrying a TB's CRC
/// computes it inline and d_tb_crcs is not read; without it the TB CRCs come from tb_crc_kernel.
void launch_pdsch_encode_packed(int              bg,
                                const enc_desc*  d_desc,
                                int              nof_cbs,
                                const uint8_t*   d_tbs,
                                const uint32_t*  d_tb_crcs,
                                const tb_crc_desc* d_tb_inline,
                                uint32_t*        d_out_words,
                                const uint16_t*  d_shifts,
                                const core_plan* d_core_plans,
                                const uint32_t*  d_crc_tables,
                                const uint32_t*  d_crc_slice,
                                hipStream_t      s);

/// Launches the batched rate dematcher (rate_dematcher.hip). mode 0: generic combining, 1: SIMD combining.
/// d_harq_cbs (optional): codeblock i's soft buffer is d_harq_cbs[dm_desc::cb_index] instead of d_harq + harq_offset.
void launch_rate_dematch(int            mode,
                         const dm_desc* d_desc,
                         int            nof_cbs,
                         const int8_t*  d_llrs,
                         int8_t*        d_harq,
                         uint8_t*       d_cb_crc_ok,
                         hipStream_t    stream,
                         int8_t* const* d_harq_cbs = nullptr);

/// TB stage of the PUSCH decoder (pusch_tb.hip): codeblock concatenation and TB CRC check.
struct tb_dec_desc {
  uint32_t first_cb;     ///< Index of the TB's first codeblock (flags, messages).
  uint32_t nof_cbs;      ///< C.
  uint32_t tbs_bits;     ///< Transport block size in bits.
  uint32_t cb_data_bits; ///< Data bits per codeblock (cb_info when C > 1).
  uint32_t data_magic;   ///< ceil(2^32 / cb_data_bits).
  uint32_t tb_offset;    ///< Output byte offset of the transport block.
  uint32_t tb_index;     ///< Result slot.
  uint32_t crc_table;    ///< CRC24A per-bit contribution table of tbs_bits (CRC arena offset) or NO_CRC_TABLE.
};

/// A byte range [begin, end) of a large segmented TB (pusch_tb_slice_kernel): begin a multiple of 16 (CRC chunks).
struct tb_slice {
  uint32_t tb;          ///< Index into the plan's tb_dec_desc array.
  uint32_t begin;
  uint32_t end;
  uint32_t nof_slices;  ///< Slices of the TB (its last finisher finalises).
};
/// TB bytes per slice workgroup (256 lanes x one 16-byte CRC chunk each).
constexpr uint32_t TB_SLICE_BYTES = 4096;

void launch_pusch_tb_sliced(const tb_dec_desc* d_desc,
                            const tb_slice*    d_slices,
                            int                nof_slices,
                            uint8_t*           d_cb_crc_ok,
                            const uint8_t*     d_cb_msgs,
                            uint8_t*           d_tbs,
                            uint8_t*           d_tb_crc_ok,
                            const uint32_t*    d_crc_tables,
                            uint32_t*          d_acc,
                            uint32_t*          d_cnt,
                            hipStream_t        stream);

/// threads: 256; 1024 for plans with TBs above TB_CRC_INLINE_MAX_BYTES (the TB CRC chain per lane shrinks 4x); 64
/// when every TB is one small codeblock.
void launch_pusch_tb(const tb_dec_desc* d_desc,
                     int                nof_tbs,
                     int                threads,
                     uint8_t*           d_cb_crc_ok,
                     const uint8_t*     d_cb_msgs,
                     uint8_t*           d_tbs,
                     uint8_t*           d_tb_crc_ok,
                     const uint32_t*    d_crc_tables,
                     hipStream_t        stream);

/// Bytes between the packed messages of consecutive codeblocks in the PUSCH decoder's message buffer.
constexpr uint32_t CB_MSG_STRIDE = 1056;  // 22 * 384 / 8

#ifdef CHEST_PROFILE
/// Copies the phase stamps of the instrumented estimator build (CHEST_PROFILE) into dst (n words).
int debug_read_chest_profile(uint64_t* dst, size_t n);
#endif
#ifdef ENC_PROFILE
/// Copies the phase stamps of the instrumented encoder build (ENC_PROFILE) into dst (n words).
int debug_read_encoder_profile(uint64_t* dst, size_t n);
#endif
#ifdef LDPC_DEC_PROFILE
constexpr int LDPC_DEC_PROF_CBS   = 4096;
constexpr int LDPC_DEC_PROF_SLOTS = 32;
/// Copies the phase stamps of the instrumented decoder build (LDPC_DEC_PROFILE) into dst (n words).
int debug_read_decoder_profile(uint64_t* dst, size_t n);
int debug_read_decoder_profile_pk(uint64_t* dst, size_t n);
#endif

/// Launches the packed two-rows-per-lane LDPC decoder (ldpc_decoder_pk.hip; even Z, block_threads >= Z / 2, or
/// >= 2 x 64 ceil(Z / 128) with split = 2) built for at most max_layers layers (8, 16 or all; every codeblock of the
/// launch must satisfy layers_bound() <= it). split = 2: each row's edges are shared by two halves of the workgroup.
void launch_ldpc_decode_pk(int             bg,
                           int             mode,
                           int             max_layers,
                           int             split,
                           const dec_desc* d_desc,
                           int             nof_cbs,
                           int             block_threads,
                           const int8_t*   d_llrs,
                           uint8_t*        d_out,
                           int32_t*        d_results,
                           const uint32_t* d_ab,
                           const uint32_t* d_crc_tables,
                           uint8_t*        d_cb_crc_ok,
                           const dm_desc*  d_dm,
                           int8_t*         d_harq,
                           hipStream_t     stream,
                           int8_t* const*  d_harq_cbs = nullptr);

/// Launches the two-codeblock packed decoder (ldpc_decode_pairs_kernel): workgroup w decodes d_desc[2 w + i] (slots
/// with nof_llr = 0 are empty; the two slots share Z, scaling, iteration limit and CRC mode), codeblock slot i on lanes
/// [i Z / 2, (i + 1) Z / 2), block_threads >= (used slots) x Z / 2. d_ab2: the interleaved image's pair constants. d_dm:
/// fused rate dematching of first transmissions (d_dm[2 w + i], d_llrs the codeword LLRs, soft buffers at d_harq +
/// harq_offset or d_llr_cbs[cb]).
void launch_ldpc_decode_pairs(int             bg,
                              int             mode,
                              int             max_layers,
                              const dec_desc* d_desc,
                              int             nof_groups,
                              int             block_threads,
                              const int8_t*   d_llrs,
                              uint8_t*        d_out,
                              int32_t*        d_results,
                              const uint32_t* d_ab2,
                              const uint32_t* d_crc_tables,
                              uint8_t*        d_cb_crc_ok,
                              hipStream_t     stream,
                              int8_t* const*  d_llr_cbs = nullptr,
                              const dm_desc*  d_dm      = nullptr,
                              int8_t*         d_harq    = nullptr);

/// Launches the batched LDPC decoder (ldpc_decoder.hip). d_llr_cbs (optional): codeblock c's input is
/// d_llr_cbs[dec_desc::cb_index] instead of d_llrs + llr_offset (the same for the packed launchers: per-codeblock HARQ
/// soft buffers in a persistent arena).
void launch_ldpc_decode(int                bg,
                        int                mode,
                        const dec_desc*    d_desc,
                        int                nof_cbs,
                        int                block_threads,
                        const int8_t*      d_llrs,
                        uint8_t*           d_out,
                        int32_t*           d_results,
                        const uint32_t*    d_shifts,
                        const uint32_t*    d_crc_tables,
                        uint8_t*           d_cb_crc_ok,
                        hipStream_t        stream,
                        int8_t* const*     d_llr_cbs = nullptr);

/// PDSCH modulator (pdsch_modulator.hip): per-transmission descriptor.
struct mod_desc {
  uint64_t dmrs_lut;        ///< Data subcarriers (4 bits each, ascending) of a PRB on DM-RS symbols.
  uint32_t cw_word_offset;  ///< First 32-bit word of the packed codeword.
  uint32_t nof_bits;        ///< Codeword length G.
  uint32_t c_init;          ///< Scrambling sequence initial state (31 bits).
  uint32_t grid_base;       ///< Element of (port 0, symbol 0, first allocated subcarrier) in the grids.
  uint32_t port_stride;     ///< Elements per port of a grid (14 * nsc).
  uint32_t nsc;             ///< Subcarriers per OFDM symbol.
  uint16_t dmrs_mask;       ///< DM-RS symbols.
  uint8_t  qm;              ///< Modulation order.
  uint8_t  L;               ///< Layers.
  uint8_t  P;               ///< Ports.
  uint8_t  nd_dmrs;         ///< Data REs per PRB on DM-RS symbols.
  uint16_t prg_sc;          ///< Per-PRG precoding: subcarriers per PRG (0: the wideband weights w).
  uint16_t sym_cum[16];     ///< Data REs in the symbols before symbol l (l = 0..14).
  float    w[4][4][2];      ///< Precoding weights [port][layer] times the modulation amplitude.
  uint32_t seq_word_offset; ///< First word of the transmission's scrambling sequence in the plan's sequence buffer.
  uint32_t sc_map;          ///< General allocation: first entry of the RE -> grid subcarrier map (NO_SC_MAP: contiguous).
  uint32_t prg_w;           ///< Per-PRG precoding: first float of [prg][port][layer][2] (amplitude folded in).
  uint32_t pad3[3];
};
static_assert(sizeof(mod_desc) == 224, "mod_desc layout");

/// mod_desc::sc_map of the contiguous fast path.
constexpr uint32_t NO_SC_MAP = 0xffffffffu;

/// PDSCH modulator / PUSCH demodulator work item: MOD_CHUNK_WORDS x 32 codeword bits of one transmission and the REs
/// starting in them.
struct mod_chunk {
  uint32_t tx;        ///< Transmission (descriptor index).
  uint32_t word0;     ///< First codeword word of the chunk.
  uint32_t re_begin;  ///< First RE whose bits start in the chunk.
  uint32_t re_end;    ///< One past the last.
};

/// Codeword words per modulator chunk (one workgroup): 1024 keeps a few-PRB 4-layer transmission (~23k bits) in one
/// workgroup of ~3 REs per lane instead of three workgroups of one RE per lane (DM-RS + modulator stage 59.5 -> 52.6 us
/// per step, headline +0.5 %; 512 splits such a transmission unevenly and was slower; profiles/r4_mod_chunk_ab.txt).
constexpr uint32_t MOD_CHUNK_WORDS = 1024;
/// PUSCH demodulator chunk (codeword words per workgroup, pusch_demodulator.hip). A lane that issued its next RE's
/// loads while equalising the current one was slower (r4: 4x the loads in flight, 98 -> 106 VGPRs, 28.3 -> 30.2 us).
constexpr uint32_t DEMOD_CHUNK_WORDS = 256;
constexpr uint32_t MOD_MAX_BITS    = 1u << 21;
/// Gold sequence tables (TS 38.211 section 5.2.1): x1 bits x1(1600 + n) as LSB-first words; x2 chunk jumps
/// M^(1600 + 2048 c) (c < MOD_MAX_BITS / 2048, 31 column words each); x2 lane jumps M^(32 i) (i < 64) as [column][i].
constexpr uint32_t GOLD_NC           = 1600;
constexpr uint32_t GOLD_X1_WORDS     = MOD_MAX_BITS / 32;
constexpr uint32_t GOLD_X2_JUMPS     = MOD_MAX_BITS / 2048;

void launch_pdsch_modulate(const mod_desc*  d_desc,
                           const uint16_t*  d_sc_map,
                           const float*     d_prg_w,
                           const mod_chunk* d_chunks,
                           int              nof_chunks,
                           const uint32_t*  d_codewords,
                           uint32_t*        d_grids,
                           const uint32_t*  d_seq,
                           hipStream_t      stream);

/// Fills a plan's (de)scrambling sequence buffer once, at plan creation: for entry t, words
/// seq[offsets[t] + i] = c(32 w) .. c(32 w + 31) (MSB first), w = wstart[t] + i (wstart null: 0), of the Gold sequence
/// with initial state c_inits[t], i < nwords[t] (pdsch_modulator.hip: gold_fill_kernel).
void launch_gold_fill(const uint32_t* d_c_inits,
                      const uint32_t* d_offsets,
                      const uint32_t* d_nwords,
                      const uint32_t* d_wstart,
                      int             nof_tx,
                      uint32_t        max_nwords,
                      uint32_t*       d_seq,
                      const uint32_t* d_x1,
                      const uint32_t* d_x2_jump,
                      const uint32_t* d_x2_lane,
                      hipStream_t     stream);

/// OFDM (de)modulator job: one OFDM symbol of one port of one grid (ofdm.hip).
struct ofdm_job {
  uint32_t grid_offset;    ///< Element of (grid, port, symbol, subcarrier 0).
  uint32_t sample_offset;  ///< Complex sample where the symbol's cyclic prefix starts.
  uint32_t cp_len;         ///< Cyclic prefix length in samples.
  uint32_t pad;
  float    coef_re;        ///< Phase compensation times scale.
  float    coef_im;
};

/// Largest DFT size and the twiddle table exp(-j 2 pi m / OFDM_MAX_DFT), m < OFDM_MAX_DFT, every size strides through.
constexpr uint32_t OFDM_MAX_DFT = 8192;

/// Split factor of the two-kernel transform of a DFT size above one workgroup's LDS (the generic DFT's 9216 ..
/// 98304): N = ofdm_split_factor(N) x M with M a power of two <= OFDM_MAX_DFT; 0 for the one-kernel sizes.
constexpr uint32_t ofdm_split_factor(uint32_t n)
{
  return n == 9216 ? 9 : n == 12288 ? 3 : n == 18432 ? 9 : n == 24576 ? 3 : n == 36864 ? 9 : n == 49152 ? 6
         : n == 98304 ? 12 : 0;
}

/// dft_size: a power of two 128..8192, 3 x 2^m 384..6144, 4608 (9 x 512), or a split size (ofdm_split_factor != 0),
/// which needs d_scratch: nof_jobs x dft_size complex floats.
void launch_ofdm(bool            inverse,
                 uint32_t        dft_size,
                 const ofdm_job* d_jobs,
                 int             nof_jobs,
                 uint32_t        nsc,
                 uint32_t        window_offset,
                 const float*    d_twiddles,
                 const uint32_t* d_grid_in,
                 uint32_t*       d_grid_out,
                 const float*    d_samples_in,
                 float*          d_samples_out,
                 float*          d_scratch,
                 hipStream_t     stream,
                 const uint32_t* d_twin = nullptr);  ///< modulation: HBM twin of d_grid_in (not for split sizes)
/// Direct-address job list (srsgpu_ofdm_jobs_execute_direct); false for a split DFT size (nothing launched).
bool launch_ofdm_direct(bool                          inverse,
                        uint32_t                      dft_size,
                        const srsgpu_ofdm_direct_job* d_jobs,
                        int                           nof_jobs,
                        uint32_t                      nsc,
                        uint32_t                      window_offset,
                        const float*                  d_twiddles,
                        hipStream_t                   stream);

/// PUSCH demodulator (pusch_demodulator.hip): per-transmission descriptor. Work items are mod_chunk (8192 LLRs each).
struct demod_desc {
  uint64_t dmrs_lut;        ///< Data subcarriers (4 bits each, ascending) of a PRB on DM-RS symbols.
  uint32_t grid_base;       ///< Element of (port 0, symbol 0, first allocated subcarrier) in the rx grids.
  uint32_t port_stride;     ///< Elements per port of a grid (14 * nsc).
  uint32_t nsc;             ///< Subcarriers per OFDM symbol.
  uint32_t ce_base;         ///< Element of (layer 0, port 0, symbol 0, first allocated subcarrier) in the estimates.
  uint32_t ce_layer_stride; ///< Elements per layer of a slot's estimates (grid_nof_ports * 14 * nsc).
  uint32_t llr_offset;      ///< First codeword LLR.
  uint32_t nof_llrs;        ///< Codeword length.
  uint32_t c_init;          ///< Descrambling sequence initial state.
  uint32_t tx;              ///< Transmission index (noise variances at 4 * tx).
  uint16_t dmrs_mask;       ///< DM-RS symbols.
  uint8_t  qm, L, P;        ///< Modulation order, layers, rx ports.
  uint8_t  nd_dmrs;         ///< Data REs per PRB on DM-RS symbols.
  uint8_t  eq;              ///< Equalizer kind (DEMOD_EQ_*).
  uint8_t  ce_compact;      ///< Estimates in the compact layout: every symbol reads the row at ce_base.
  uint16_t sym_cum[16];     ///< Data REs in the symbols before symbol l (l = 0..14).
  uint32_t seq_word_offset; ///< First word of the transmission's descrambling sequence in the plan's sequence buffer.
  uint32_t ce_cfo;          ///< Compact layout with CFO compensation: rotate each symbol's estimates (CFO word at
                            ///< ce_base + nsc of every (layer, port)).
  float    epochs[14];      ///< Symbol start epochs (symbol durations) for the rotation.
  uint32_t crb_list;        ///< CRB-mask allocation: first entry of the transmission's allocated CRBs (ascending) in the
                            ///< plan's CRB list, grid_base / ce_base then exclude the first subcarrier; DEMOD_CONTIGUOUS
                            ///< for the contiguous allocation.
  uint16_t transform_precoding;  ///< Transform-precoded: the demodulate_tp kernel handles the transmission.
  uint16_t cfo_sc;               ///< Subcarrier of the compact row's CFO word relative to ce_base (the first
                                 ///< allocated one: 0 for contiguous allocations, 12 x first CRB for CRB masks).
};
static_assert(sizeof(demod_desc) == 160, "demod_desc layout");
constexpr uint32_t DEMOD_CONTIGUOUS = 0xffffffffu;

/// Transform-precoded PUSCH work item: one OFDM symbol of one transmission (M data REs, the inverse DFT length).
struct demod_tp_job {
  uint32_t tx;
  uint32_t symbol;
};
/// Post-equalization statistics accumulators per transmission and OFDM symbol: (sum of finite noise variances, their
/// count, sum of squared EVM errors, equalized symbols).
constexpr int DEMOD_ACC_PER_TX = 14 * 4;
/// Statistics floats per transmission (SRSGPU_DEMOD_STATS of the C ABI): 15 rows x (SINR dB, EVM).
constexpr int DEMOD_STATS_PER_TX = 30;

/// demod_desc::eq: the reference's ZF paths (1 layer: 1 x N with port reduction; 2 layers: 2 x N) or linear MMSE.
constexpr uint8_t DEMOD_EQ_ZF   = 0;
constexpr uint8_t DEMOD_EQ_MMSE = 1;

/// Max-log interval tables of the 64QAM / 256QAM demapper: per bit pair k (stream bits 2k, 2k + 1) the reciprocal
/// interval width (the SIMD paths scale by it, avx2_helpers.h:178), a count and (slope, intercept) per interval
/// (interleaved: one 8-byte LDS read per lookup). Index 0..2: 64QAM, 3..6: 256QAM.
struct demap_pair_table {
  float    inv_width;
  uint32_t count;
  float    piece[16][2];
};
constexpr int DEMAP_TABLES = 7;

/// PDSCH DM-RS job (pdsch_modulator.hip): one DM-RS OFDM symbol of one transmission.
struct dmrs_job {
  uint32_t grid_base;    ///< Element of (port 0, DM-RS symbol, first allocated subcarrier) in the grids.
  uint32_t port_stride;  ///< Elements per port of a grid.
  uint32_t c_init;       ///< Sequence initial state of the symbol.
  uint32_t seq_offset;   ///< Sequence index of the first allocated RB's first DM-RS ((rb_start - k_ref) x per RB).
  float    amp;          ///< sqrt(1/2) x amplitude.
  float    w[4][4][2];   ///< Precoding weights [port][layer].
  uint16_t nof_pilots;   ///< DM-RS REs per CDM group in the symbol (nof_rb x per RB).
  uint8_t  type2;        ///< DM-RS type 2.
  uint8_t  L, P;         ///< Layers (DM-RS ports 0..L-1), antenna ports.
  uint8_t  lp;           ///< l' (1 when the previous symbol also carries DM-RS): selects w_t.
  uint8_t  pad[2];
  uint32_t gseq_base;    ///< The job's sequence words (from word seq_offset / 16) in the plan's buffer.
};

/// max_pilots: the largest nof_pilots of the jobs (sets the workgroups per job).
void launch_pdsch_dmrs(const dmrs_job* d_jobs,
                       int             nof_jobs,
                       int             max_pilots,
                       uint32_t*       d_grids,
                       const uint32_t* d_seq,
                       hipStream_t     stream);

/// PUSCH channel estimator job (pusch_chest.hip): one (transmission, rx port, DM-RS CDM group).
struct chest_job {
  double   ta_fs;            ///< Sampling rate of the time-alignment correlation (DFT size x SCS x pilot stride), Hz.
  uint32_t grid_base;        ///< Element of (port, symbol 0, first allocated subcarrier) in the rx grids.
  uint32_t ce_base;          ///< Element of (first layer of the group, port, symbol 0, first allocated subcarrier).
  uint32_t ce_layer_stride;  ///< Elements per layer of a slot's estimates.
  uint32_t nsc;              ///< Subcarriers per OFDM symbol.
  uint32_t seq_offset;       ///< DM-RS sequence index of the first pilot (rb_start x pilots per RB; point A = 0).
  uint32_t c_init[14];       ///< DM-RS sequence initial state of each DM-RS symbol (order of dmrs_symbols).
  uint32_t pattern;          ///< Pilot subcarriers within a PRB (4 bits each, ascending).
  uint32_t noise_slot;       ///< 4 * tx + port: noise variance / metrics slot.
  float    beta;             ///< DM-RS to data amplitude scaling.
  float    taps[32];         ///< Normalised smoothing filter taps (CHEST_FD_FILTER).
  float    epochs[14];       ///< Symbol start epochs in symbol durations (initialize_symbol_start_epochs).
  float    td_w[14];         ///< "interpolate": weight of plane td_q1 for symbol l (plane td_q0 gets 1 - w).
  float    scs_hz;           ///< Subcarrier spacing (CFO in Hz).
  uint16_t nof_pilots;       ///< Pilots per DM-RS symbol.
  uint16_t nof_rb;           ///< Allocated RBs (contiguous).
  uint16_t ta_dft;           ///< Time-alignment DFT size M (power of two, 128..4096).
  uint16_t ta_max;           ///< Correlation taps searched on each side (half cyclic prefix in samples).
  uint8_t  dmrs_symbols[14]; ///< OFDM symbols carrying DM-RS.
  int8_t   td_q0[14];        ///< "interpolate": planes interpolated for symbol l.
  int8_t   td_q1[14];
  uint8_t  nof_dmrs;         ///< Number of DM-RS symbols.
  uint8_t  group_layers;     ///< Layers of this CDM group (1 or 2).
  uint8_t  group;            ///< CDM group (0: ports 1000/1001, 1: ports 1002/1003).
  uint8_t  pilots_per_rb;    ///< 6 (type 1) or 4 (type 2).
  uint8_t  fd;               ///< CHEST_FD_* smoothing strategy.
  uint8_t  ntaps;            ///< Filter length (odd).
  uint8_t  nof_v_pilots;     ///< Virtual pilots on each side.
  uint8_t  interp_offset;    ///< Interpolator offset (first pilot subcarrier of a PRB).
  uint8_t  interp_stride;    ///< Interpolator stride.
  uint8_t  first_symbol;     ///< First allocated OFDM symbol.
  uint8_t  nof_symbols;      ///< Allocated OFDM symbols.
  uint8_t  nof_out_symbols;  ///< Rows written: nof_symbols, or 1 in the compact layout.
  uint8_t  td_interp;        ///< Time-domain strategy: 0 average (one plane), 1 interpolate (one plane per DM-RS symbol).
  uint8_t  compensate_cfo;   ///< Derotate the DM-RS symbols by the estimated CFO and rotate the estimates.
  uint8_t  compact_cfo;      ///< Compact layout with CFO compensation: store the CFO next to the estimate row.
  uint8_t  ta_log2;          ///< log2(ta_dft).
  uint8_t  ta_positions;     ///< 1: pilots at their subcarrier offset (mask path), 0: in the first bins (stride 2).
  uint8_t  pad[1];
  uint32_t gseq_base;        ///< The job's DM-RS sequence words in the plan's buffer: [DM-RS symbol][staged word].
  uint32_t crb_list;         ///< CRB-mask allocation: the allocated CRBs relative to the first one in the plan's CRB
                             ///< list (pilots and estimates follow them); CHEST_CONTIGUOUS otherwise.
  uint16_t span_pilots;      ///< DM-RS sequence positions from the first to the last allocated CRB (staged words).
  uint16_t pad2;
  uint32_t lp_base;          ///< Low-PAPR DM-RS (transform precoding): first pilot value of the job's sequence in the
                             ///< plan's table (one complex float per pilot, every DM-RS symbol); CHEST_CONTIGUOUS: the
                             ///< pseudo-random sequence words.
};
constexpr uint32_t CHEST_CONTIGUOUS = 0xffffffffu;

constexpr uint8_t CHEST_FD_NONE   = 0;
constexpr uint8_t CHEST_FD_MEAN   = 1;
constexpr uint8_t CHEST_FD_FILTER = 2;

/// Floats per (transmission, port) of the estimator's metrics output (RSRP, EPRE, noise variance, SNR, TA, CFO).
constexpr int CHEST_METRICS = 8;

/// Plan-wide maxima that size the estimator's dynamic LDS.
struct chest_geom {
  int max_pilots;  ///< Pilots per DM-RS symbol.
  int max_dmrs;    ///< DM-RS symbols.
  int max_words;   ///< Staged sequence words per DM-RS symbol.
  int max_planes;  ///< LSE planes (1 with "average", the DM-RS symbols with "interpolate").
  int max_gl;      ///< Layers per CDM group.
  int max_dft;     ///< Time-alignment DFT size.
};

/// Dynamic LDS of the channel-estimator kernel for the plan's largest job.
size_t pusch_chest_lds_bytes(const chest_geom& g);

void launch_pusch_chest(const float2*   d_lp,
                        const uint16_t* d_crbs,
                        const chest_job* d_jobs,
                        int              nof_jobs,
                        const chest_geom& geom,
                        const uint32_t*  d_grids,
                        uint32_t*        d_ce,
                        float*           d_noise_var,
                        float*           d_metrics,
                        const uint32_t*  d_seq,
                        hipStream_t      stream,
                        const srsgpu_copy_span* d_spans    = nullptr,
                        int              nof_spans  = 0,
                        uint64_t         span_bytes = 0);  ///< the largest span

/// UL-SCH demultiplexer (ulsch_demux.hip): per-transmission descriptor and per-RE routing.
struct ulsch_demux_desc {
  uint32_t llr_offset, sch_offset, uci_offset[3];  ///< Input codeword and output stream offsets (LLRs).
  uint32_t route;                                  ///< First routing entry (one per RE) in the plan's table.
  uint32_t seq_word_offset;                        ///< Scrambling sequence words (placeholders) in the plan's buffer.
  uint32_t nof_llrs;                               ///< Codeword LLRs.
  uint8_t  qm, lq;                                 ///< Modulation order, LLRs per RE (layers x Qm).
  uint8_t  placeholder[3];                         ///< Per UCI field: 0 none, 1 / 2: the 1- / 2-bit placeholders.
  uint8_t  pad[3];
};
/// Routing of one RE: sch = RE index in the UL-SCH stream or DEMUX_NONE; uci = kind (bits 30-31: 0 none, 1 HARQ-ACK,
/// 2 CSI Part 1, 3 CSI Part 2) | RE index in that stream (bits 0-29); csi2 = RE index in the CSI Part 2 stream of a
/// HARQ-ACK RE (<= 2 bits, on the reserved REs) that CSI Part 2 was also mapped to, else DEMUX_NONE. HARQ-ACK of <= 2
/// bits punctures: the UL-SCH and CSI Part 2 receive zeros on its REs (ulsch_demultiplex_impl.cpp:468).
struct ulsch_demux_route {
  uint32_t sch;
  uint32_t uci;
  uint32_t csi2;
};
constexpr uint32_t DEMUX_NONE = 0xffffffffu;

void launch_ulsch_demux(const ulsch_demux_desc*  d_desc,
                        const ulsch_demux_route* d_routes,
                        const mod_chunk*         d_chunks,
                        int                      nof_chunks,
                        const int8_t*            d_llrs,
                        int8_t*                  d_sch,
                        int8_t*                  d_harq,
                        int8_t*                  d_csi1,
                        int8_t*                  d_csi2,
                        const uint32_t*          d_seq,
                        hipStream_t              stream);

void launch_pusch_demodulate_tp(const demod_desc*       d_desc,
                                const demod_tp_job*      d_jobs,
                                int                      nof_jobs,
                                const demap_pair_table*  d_tables,
                                const uint32_t*          d_grids,
                                const uint32_t*          d_ch_est,
                                const float*             d_noise_var,
                                int8_t*                  d_llrs,
                                const uint32_t*          d_seq,
                                const uint16_t*          d_crbs,
                                float*                   d_acc,
                                hipStream_t              stream);
void launch_pusch_demod_stats(float* d_acc, float* d_stats, int nof_tx, hipStream_t stream);
void launch_pusch_demodulate(const demod_desc*        d_desc,
                             const mod_chunk*         d_chunks,
                             int                      nof_chunks,
                             int                      threads,
                             const demap_pair_table*  d_tables,
                             const uint32_t*          d_grids,
                             const uint32_t*          d_ch_est,
                             const float*             d_noise_var,
                             int8_t*                  d_llrs,
                             const uint32_t*          d_seq,
                             const uint16_t*          d_crbs,
                             float*                   d_acc,
                             hipStream_t              stream);

} // namespace srsgpu
