/*
 * srsgpu_phy.h — C ABI of the MI355X (gfx950) 5G NR PHY acceleration library (libsrsgpu_phy.so).
 *
 * Drop-in boundary for the srsRAN upper-PHY channel-coding hot path. Every entry point names the reference interface
 * it replaces (paths relative to the srsRAN tree, include/ or lib/). Plain C: pointers, sizes, POD structs; no C++ or
 * torch types. Device pointers are HIP device (HBM) addresses; `stream` is a hipStream_t (NULL = default stream).
 *
 * Error convention: functions return SRSGPU_OK (0) or a negative SRSGPU_ERR_* code; srsgpu_last_error() returns a
 * thread-local description of the last failure. Invalid configurations are rejected with the same conditions the
 * reference asserts on (e.g. ldpc_decoder_impl.cpp:48-:56, :73-:88).
 */
#ifndef SRSGPU_PHY_H
#define SRSGPU_PHY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRSGPU_OK 0
#define SRSGPU_ERR_INVALID_ARG (-1)
#define SRSGPU_ERR_HIP (-2)
#define SRSGPU_ERR_NO_MEMORY (-3)

/* CRC generator polynomials, same numbering as srsran::crc_generator_poly
 * (include/srsran/phy/upper/channel_coding/crc_calculator.h:33). */
#define SRSGPU_CRC24A 0
#define SRSGPU_CRC24B 1
#define SRSGPU_CRC24C 2
#define SRSGPU_CRC16 3
#define SRSGPU_CRC11 4
#define SRSGPU_CRC6 5
#define SRSGPU_CRC_NONE 255 /* no CRC early stop: the decoder runs max_iterations (crc == nullptr) */

/* LDPC decoder arithmetic variants of the reference (lib/phy/upper/channel_coding/channel_coding_factories.cpp,
 * create_ldpc_decoder_factory_sw): "generic" rounds the normalised min-sum magnitudes (ldpc_decoder_generic.cpp:70);
 * "avx2"/"avx512"/"neon" truncate a 16-bit fixed-point product (avx2_support.h:71). Results are bit-exact with the
 * selected variant. */
#define SRSGPU_LDPC_IMPL_GENERIC 0
#define SRSGPU_LDPC_IMPL_SIMD 1

typedef struct srsgpu_context srsgpu_context;

/** Library version (major * 10000 + minor * 100 + patch). */
int srsgpu_version(void);

/** Thread-local description of the last error. */
const char* srsgpu_last_error(void);

/** Creates a context on HIP device `device` (one process per GPU). Uploads the lifted base-graph tables. */
int srsgpu_context_create(int device, srsgpu_context** ctx);

/** Destroys a context and frees its device memory. */
void srsgpu_context_destroy(srsgpu_context* ctx);

/** HIP device index of a context (-1 for NULL): the device a binding allocates its own buffers and streams on. */
int srsgpu_context_device(const srsgpu_context* ctx);

/** Kernel-selection options of a context, read when a plan is created (not from the process environment: what a plan
 *  runs depends only on its context and configuration). Every default is the measured-fastest choice; the others are
 *  alternative kernels with identical results, kept for the parity tests that pin them. */
typedef enum {
  /** Packed LDPC decoder, even Z: -1 (default) the edge-split kernel when a launch gives under ~3 waves per SIMD,
   *  else the one-row-pair kernel; 0 always the one-row-pair kernel; 1 always the edge-split kernel. */
  SRSGPU_OPTION_DECODER_SPLIT = 1,
  /** 0 (default) / 1: codeblocks of Z = 144..192 two per workgroup (three waves for two codeblocks). */
  SRSGPU_OPTION_DECODER_PAIRS = 2,
  /** 1 (default) / 0: the PUSCH decoder dematches plain first transmissions itself (0: every codeblock through the
   *  separate rate dematcher kernel). */
  SRSGPU_OPTION_DECODER_FUSED_DEMATCH = 3,
  /** 0 (default) / 1: the PDSCH encoder's one-bit-per-byte kernel for every codeblock (0: the packed-word kernel where
   *  Z % 32 == 0 and the message is byte aligned). */
  SRSGPU_OPTION_ENCODER_BYTE_KERNEL = 4,
  /** 0 (default) / 1: the PDSCH encoder clears its codeword output before every execution (0: only when its
   *  codeblocks do not each store whole words that tile the output). */
  SRSGPU_OPTION_ENCODER_ZERO_OUTPUT = 5
} srsgpu_option;

/** Sets option `option` (srsgpu_option) of a context for the plans created afterwards. */
int srsgpu_context_set_option(srsgpu_context* ctx, int option, int value);

/** Reads option `option` of a context. */
int srsgpu_context_get_option(const srsgpu_context* ctx, int option, int* value);

/* ------------------------------------------------------------------------------------------------------------------
 * LDPC decoder — replaces srsran::ldpc_decoder::decode(bit_buffer& output, span<const log_likelihood_ratio> input,
 * crc_calculator* crc, const configuration& cfg)   (include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:72,
 * lib/phy/upper/channel_coding/ldpc/ldpc_decoder_impl.cpp:60), batched over codeblocks.
 * ------------------------------------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t  base_graph;      /* 1 or 2 (codeblock_metadata::tb_common.base_graph) */
  uint8_t  crc_poly;        /* SRSGPU_CRC* used for early stopping, or SRSGPU_CRC_NONE (crc == nullptr) */
  uint16_t lifting_size;    /* Z (tb_common.lifting_size) */
  uint16_t nof_filler_bits; /* cb_specific.nof_filler_bits */
  uint8_t  nof_crc_bits;    /* cb_specific.nof_crc_bits: 16 or 24 */
  uint8_t  max_iterations;  /* algorithm_conf.max_iterations (> 0) */
  float    scaling_factor;  /* algorithm_conf.scaling_factor, in (0, 1) */
  uint32_t llr_offset;      /* index of the codeblock's first LLR in the batch LLR buffer */
  uint32_t nof_llrs;        /* input.size(): (K + 2) * Z <= nof_llrs <= N_short * Z */
  uint32_t out_offset;      /* byte offset of the codeblock's K*Z output bits, packed MSB first (bit_buffer) */
} srsgpu_ldpc_decoder_config;

/** Pre-validated, device-resident batch of decoder work (reusable across calls and capturable in a hipGraph). */
typedef struct srsgpu_ldpc_decoder_plan srsgpu_ldpc_decoder_plan;

/** Validates `nof_cbs` configurations, builds the CRC early-stop tables they need and uploads the work descriptors.
 *  Blocking (host <-> device copies); call it outside the timed / captured region. */
int srsgpu_ldpc_decoder_plan_create(srsgpu_context*                   ctx,
                                    int                               impl,
                                    const srsgpu_ldpc_decoder_config* cfgs,
                                    uint32_t                          nof_cbs,
                                    srsgpu_ldpc_decoder_plan**        plan);

/** Decodes the planned codeblocks: reads int8 LLRs from d_llrs, writes packed bits to d_out and, per codeblock, the
 *  number of iterations on CRC success or -1 (std::nullopt) to d_nof_iterations[i]. Asynchronous on `stream`; no host
 *  synchronisation, no allocation (hipGraph-capturable). */
int srsgpu_ldpc_decoder_plan_execute(const srsgpu_ldpc_decoder_plan* plan,
                                     const int8_t*                   d_llrs,
                                     uint8_t*                        d_out,
                                     int32_t*                        d_nof_iterations,
                                     void*                           stream);

void srsgpu_ldpc_decoder_plan_destroy(srsgpu_ldpc_decoder_plan* plan);

/** One-shot convenience: plan_create + plan_execute + stream synchronisation + plan_destroy. */
int srsgpu_ldpc_decode(srsgpu_context*                   ctx,
                       int                               impl,
                       const srsgpu_ldpc_decoder_config* cfgs,
                       uint32_t                          nof_cbs,
                       const int8_t*                     d_llrs,
                       uint8_t*                          d_out,
                       int32_t*                          d_nof_iterations,
                       void*                             stream);

/* ------------------------------------------------------------------------------------------------------------------
 * PUSCH codeblock decoding — the operation behind hal::hw_accelerator_pusch_dec
 * (include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h:88-:112: configure_operation,
 * enqueue_operation, dequeue_operation, read_operation_outputs) and pusch_codeblock_decoder::decode
 * (lib/phy/upper/channel_processors/pusch/pusch_codeblock_decoder.cpp:33): rate dematching with HARQ soft combining
 * into a device-resident soft buffer (ldpc_rate_dematcher_impl.cpp:46), LDPC decoding and the codeblock CRC check,
 * batched over every codeblock of a slot.
 * ------------------------------------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t  base_graph;       /* 1 or 2 */
  uint8_t  rv;               /* redundancy version 0..3 */
  uint8_t  modulation_order; /* Qm: 1, 2, 4, 6, 8 */
  uint8_t  crc_poly;         /* codeblock CRC: CRC24B (segmented TB), CRC24A or CRC16 (single codeblock) */
  uint16_t lifting_size;     /* Z */
  uint16_t nof_filler_bits;  /* F */
  uint8_t  nof_crc_bits;     /* 16 or 24 */
  uint8_t  max_iterations;   /* > 0 */
  uint8_t  new_data;         /* 1: first transmission (copy), 0: combine with the HARQ buffer */
  uint8_t  use_early_stop;   /* 1: CRC after every iteration; 0: max_iterations then one CRC check */
  float    scaling_factor;   /* normalised min-sum factor in (0, 1) */
  uint32_t Nref;             /* limited-buffer rate matching N_ref, 0 = none */
  uint32_t rm_length;        /* E: rate-matched length (multiple of Qm) */
  uint32_t llr_offset;       /* first of the E LLRs in the codeword LLR buffer */
  uint32_t harq_offset;      /* first of the N_short * Z LLRs of the codeblock's HARQ soft buffer */
  uint32_t out_offset;       /* byte offset of the packed K*Z decoded message bits */
} srsgpu_pusch_cb_config;

typedef struct srsgpu_pusch_cb_plan srsgpu_pusch_cb_plan;

/** Validates the codeblock configurations (reference assertions of ldpc_rate_dematcher_impl.cpp:54-:99 and the
 *  decoder's) and uploads the work descriptors. Blocking; outside the timed / captured region. */
int srsgpu_pusch_cb_plan_create(srsgpu_context*               ctx,
                                int                           impl,
                                const srsgpu_pusch_cb_config* cfgs,
                                uint32_t                      nof_cbs,
                                srsgpu_pusch_cb_plan**        plan);

/** Rate-dematches d_llrs into the HARQ buffers d_harq (in place), then decodes every codeblock whose entry in
 *  d_cb_crc_ok (persistent per-codeblock HARQ flags, may be NULL) is 0: writes the packed message to d_out, the number
 *  of iterations (or -1; 0 for codeblocks skipped because their CRC had already passed) to d_nof_iterations, and sets
 *  d_cb_crc_ok on success. Asynchronous on `stream`, hipGraph-capturable. */
int srsgpu_pusch_cb_plan_execute(const srsgpu_pusch_cb_plan* plan,
                                 const int8_t*               d_llrs,
                                 int8_t*                     d_harq,
                                 uint8_t*                    d_out,
                                 int32_t*                    d_nof_iterations,
                                 uint8_t*                    d_cb_crc_ok,
                                 void*                       stream);

void srsgpu_pusch_cb_plan_destroy(srsgpu_pusch_cb_plan* plan);

/* ------------------------------------------------------------------------------------------------------------------
 * PDSCH encoder — replaces srsran::pdsch_encoder::encode(span<uint8_t> codeword, span<const uint8_t> transport_block,
 * const configuration& cfg) (include/srsran/phy/upper/channel_processors/pdsch/pdsch_encoder.h,
 * lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp:28) and hal::hw_accelerator_pdsch_enc in TB mode
 * (hw_accelerator_pdsch_enc.h): TB CRC, segmentation, CB CRC24B, LDPC encoding and rate matching of every transport
 * block of a slot. The codeword is written packed MSB first (G = nof_ch_symbols * Qm bits per TB).
 * ------------------------------------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t  base_graph;       /* 1 or 2 */
  uint8_t  rv;               /* 0..3 */
  uint8_t  modulation_order; /* Qm: 1, 2, 4, 6, 8 */
  uint8_t  nof_layers;       /* 1..4 */
  uint32_t tbs_bytes;        /* transport block size in bytes */
  uint32_t nof_ch_symbols;   /* number of channel symbols (multiple of nof_layers) */
  uint32_t Nref;             /* limited-buffer rate matching N_ref, 0 = none */
  uint32_t tb_offset;        /* byte offset of the transport block in the TB buffer */
  uint32_t cw_offset;        /* byte offset of the codeword in the output buffer (multiple of 4) */
} srsgpu_pdsch_tb_config;

typedef struct srsgpu_pdsch_encoder_plan srsgpu_pdsch_encoder_plan;

/** Segments every transport block (ldpc_segmenter_tx_impl.cpp:58), validates and uploads the work. Blocking. */
int srsgpu_pdsch_encoder_plan_create(srsgpu_context*               ctx,
                                     const srsgpu_pdsch_tb_config* cfgs,
                                     uint32_t                      nof_tbs,
                                     srsgpu_pdsch_encoder_plan**   plan);

/** Number of codeblocks the plan encodes (all transport blocks). */
uint32_t srsgpu_pdsch_encoder_plan_nof_codeblocks(const srsgpu_pdsch_encoder_plan* plan);

/** Encodes the planned transport blocks from d_tbs into d_codewords. The plan owns (zeroes, then fills) the output
 *  byte range [min cw_offset, max(cw_offset + ceil(G/32)*4)). Asynchronous on `stream`, hipGraph-capturable. */
int srsgpu_pdsch_encoder_plan_execute(const srsgpu_pdsch_encoder_plan* plan,
                                      const uint8_t*                   d_tbs,
                                      uint8_t*                         d_codewords,
                                      void*                            stream);

void srsgpu_pdsch_encoder_plan_destroy(srsgpu_pdsch_encoder_plan* plan);

/** Stage timing (see srsgpu_pusch_decoder_plan_enable_timing): stages 0: output clear + TB CRC, 1: codeblock
 *  encoding and rate matching (ms[2]). */
int srsgpu_pdsch_encoder_plan_enable_timing(srsgpu_pdsch_encoder_plan* plan, int enable);
int srsgpu_pdsch_encoder_plan_stage_times(srsgpu_pdsch_encoder_plan* plan, float* ms, uint32_t* nof_executes);

/* ------------------------------------------------------------------------------------------------------------------
 * PDSCH modulator — replaces srsran::pdsch_modulator::modulate(resource_grid_writer& grid, span<const bit_buffer>
 * codewords, const config_t& config) (include/srsran/phy/upper/channel_processors/pdsch/pdsch_modulator.h:93,
 * lib/phy/upper/channel_processors/pdsch/pdsch_modulator_impl.cpp:107): scrambling with the TS 38.211 §5.2.1 Gold
 * sequence (c_init = rnti * 2^15 + n_id, codeword q = 0, :30), modulation mapping (modulation_mapper_lut_impl.cpp:39,
 * amplitude sqrt(1 / average power) times `scaling`), layer mapping, wideband precoding (channel_precoder_generic.cpp:51)
 * and resource-element mapping (resource_grid_mapper_impl.cpp:269) into bf16 resource grids, for every PDSCH
 * transmission of a batch of slots. Codewords come packed MSB first (the PDSCH encoder's output format).
 * A resource grid holds `grid_nof_ports` x 14 symbols x 12 * `grid_nof_prb` subcarriers of complex bf16 (re, im)
 * pairs (srsran::cbf16_t), port-major then symbol-major; grid g starts g * grid_nof_ports * 14 * 12 * grid_nof_prb
 * elements into d_grids. Only the PDSCH REs are written (the DM-RS REs belong to the DM-RS processor).
 * ------------------------------------------------------------------------------------------------------------------ */
typedef struct {
  uint16_t rnti;                        /* n_RNTI */
  uint16_t n_id;                        /* n_ID, 0..1023 */
  uint8_t  modulation_order;            /* Qm of modulation1: 2 (QPSK), 4, 6, 8 (256QAM) */
  uint8_t  nof_layers;                  /* 1..4 */
  uint8_t  nof_ports;                   /* precoding ports, nof_layers..4 (<= grid_nof_ports) */
  uint8_t  start_symbol;                /* start_symbol_index */
  uint8_t  nof_symbols;                 /* start_symbol + nof_symbols <= 14 */
  uint8_t  dmrs_type;                   /* dmrs_config_type: 1 or 2 */
  uint8_t  nof_cdm_groups_without_data; /* 1..2 (type 1), 1..3 (type 2) */
  uint8_t  reserved;
  uint16_t dmrs_symbol_mask;            /* dmrs_symb_pos: bit l = OFDM symbol l carries DM-RS */
  uint16_t bwp_start_rb;                /* BWP start (CRB) */
  uint16_t bwp_size_rb;                 /* BWP size */
  uint16_t rb_start;                    /* contiguous non-interleaved VRB allocation [rb_start, rb_start + nof_rb) */
  uint16_t nof_rb;
  uint16_t pad;
  float    scaling;                     /* config.scaling (applied when std::isnormal) */
  float    precoding[4][4][2];          /* wideband precoding weight [port][layer] = (re, im) */
  uint32_t cw_offset;                   /* byte offset of the packed codeword (multiple of 4) */
  uint32_t nof_bits;                    /* codeword length: data REs x nof_layers x Qm */
  uint32_t grid_index;                  /* resource grid (slot) the transmission is mapped into */
} srsgpu_pdsch_mod_config;

/* Generalised frequency allocation, reserved resource elements and per-PRG precoding of one transmission (the
 * *_plan_create_ex entry points; a NULL extension array, or NULL members, keep the contiguous / no reserved REs /
 * wideband defaults of the plain configuration).
 *
 * srsgpu_re_pattern mirrors srsran::re_pattern (include/srsran/phy/support/re_pattern.h): the REs of re_mask (bit k =
 * subcarrier k of a PRB) in every CRB of crb_mask and every OFDM symbol of symbol_mask. */
typedef struct {
  const uint8_t* crb_mask;    /* one byte per grid CRB (nonzero = included); NULL = every CRB */
  uint16_t       re_mask;     /* 12 bits */
  uint16_t       symbol_mask; /* 14 bits */
} srsgpu_re_pattern;

typedef struct {
  const uint8_t*           crb_mask;     /* allocated CRBs, one byte per grid CRB: rb_allocation::get_crb_mask of any
                                            type-0 bitmap or interleaved VRB-to-PRB mapping (pdsch_modulator_impl.cpp:58,
                                            pusch_demodulator.h:55 rb_mask); NULL = the contiguous allocation of the
                                            plain configuration */
  const srsgpu_re_pattern* reserved;     /* reserved REs besides the DM-RS (pdsch_modulator::config_t::reserved: SSB,
                                            CSI-RS, ZP-CSI-RS, PT-RS ...); PDSCH modulator only */
  uint32_t                 nof_reserved;
  uint16_t                 prg_size;     /* precoding resource block group size in PRBs (precoding_configuration);
                                            0 = the wideband weights of the plain configuration */
  uint16_t                 nof_prg;      /* PRGs in prg_weights: PRG i covers CRBs [i prg_size, (i + 1) prg_size) */
  const float*             prg_weights;  /* [nof_prg][port][layer] (re, im), ports x layers of the configuration */
} srsgpu_alloc_ext;

typedef struct srsgpu_pdsch_modulator_plan srsgpu_pdsch_modulator_plan;

/** Validates the transmissions (the reference's assertions: time allocation inside the slot, allocation inside the
 *  BWP and the grid, codeword length equal to the allocation's data REs x layers x Qm) and uploads the work. */
int srsgpu_pdsch_modulator_plan_create(srsgpu_context*                ctx,
                                       const srsgpu_pdsch_mod_config* cfgs,
                                       uint32_t                       nof_tx,
                                       uint32_t                       grid_nof_prb,
                                       uint32_t                       grid_nof_ports,
                                       srsgpu_pdsch_modulator_plan**  plan);

/** As srsgpu_pdsch_modulator_plan_create with an optional allocation extension per transmission (exts may be NULL):
 *  CRB-mask allocations, reserved RE patterns and per-PRG precoding. The data REs are the allocated CRBs' REs of the
 *  allocated symbols minus the BWP's DM-RS pattern on DM-RS symbols and the reserved patterns, in symbol-major,
 *  ascending-subcarrier order (resource_grid_mapper_impl.cpp:269). */
int srsgpu_pdsch_modulator_plan_create_ex(srsgpu_context*                ctx,
                                          const srsgpu_pdsch_mod_config* cfgs,
                                          const srsgpu_alloc_ext*        exts,
                                          uint32_t                       nof_tx,
                                          uint32_t                       grid_nof_prb,
                                          uint32_t                       grid_nof_ports,
                                          srsgpu_pdsch_modulator_plan**  plan);

/** Modulates and maps every planned transmission from d_codewords into d_grids (uint32 per RE: re | im << 16).
 *  Asynchronous on `stream`, hipGraph-capturable. */
int srsgpu_pdsch_modulator_plan_execute(const srsgpu_pdsch_modulator_plan* plan,
                                        const uint8_t*                     d_codewords,
                                        uint32_t*                          d_grids,
                                        void*                              stream);

void srsgpu_pdsch_modulator_plan_destroy(srsgpu_pdsch_modulator_plan* plan);

/* ------------------------------------------------------------------------------------------------------------------
 * PDSCH DM-RS — replaces srsran::dmrs_pdsch_processor::map(resource_grid_writer& grid, const config_t& config)
 * (include/srsran/phy/upper/signal_processors/dmrs_pdsch_processor.h:65, lib/phy/upper/signal_processors/
 * dmrs_pdsch_processor_impl.cpp:117) for every PDSCH transmission of a batch of slots: DM-RS sequence per symbol
 * (c_init = ((14 n_slot + l + 1)(2 N_ID + 1) 2^17 + 2 N_ID + n_SCID) mod 2^31), CDM cover codes of DM-RS ports
 * 0..nof_layers-1, per-CDM-group wideband precoding and mapping (bf16, same grid layout as the PDSCH modulator).
 * ------------------------------------------------------------------------------------------------------------------ */
typedef struct {
  uint16_t slot_index;           /* n_slot within the frame */
  uint16_t scrambling_id;        /* N_ID^{n_SCID} */
  uint8_t  n_scid;               /* 0 or 1 */
  uint8_t  dmrs_type;            /* 1 or 2 */
  uint8_t  nof_layers;           /* DM-RS ports 0..nof_layers-1 (1..4) */
  uint8_t  nof_ports;            /* antenna ports (precoding), nof_layers..grid_nof_ports */
  uint16_t dmrs_symbol_mask;     /* symbols_mask */
  uint16_t reference_point_k_rb; /* sequence reference RB (0: point A) */
  uint16_t rb_start;             /* contiguous CRB allocation (rb_mask), rb_start >= reference_point_k_rb */
  uint16_t nof_rb;
  float    amplitude;            /* DM-RS amplitude (beta) */
  float    precoding[4][4][2];   /* [port][layer] (re, im) */
  uint32_t grid_index;
} srsgpu_pdsch_dmrs_config;

typedef struct srsgpu_pdsch_dmrs_plan srsgpu_pdsch_dmrs_plan;

int srsgpu_pdsch_dmrs_plan_create(srsgpu_context*                 ctx,
                                  const srsgpu_pdsch_dmrs_config* cfgs,
                                  uint32_t                        nof_tx,
                                  uint32_t                        grid_nof_prb,
                                  uint32_t                        grid_nof_ports,
                                  srsgpu_pdsch_dmrs_plan**        plan);

/** As srsgpu_pdsch_dmrs_plan_create, with an optional extension per transmission (NULL array or NULL crb_mask: the
 *  contiguous rb_start / nof_rb allocation): crb_mask is dmrs_pdsch_processor::config_t::rb_mask (one byte per grid
 *  CRB, any pattern; the sequence skips the unallocated CRBs, dmrs_helper.cpp dmrs_sequence_generate). Reserved
 *  patterns and PRGs are rejected: the reference's DM-RS precoding has one PRG (dmrs_pdsch_processor_impl.cpp:149). */
int srsgpu_pdsch_dmrs_plan_create_ex(srsgpu_context*                 ctx,
                                     const srsgpu_pdsch_dmrs_config* cfgs,
                                     const srsgpu_alloc_ext*         exts,
                                     uint32_t                        nof_tx,
                                     uint32_t                        grid_nof_prb,
                                     uint32_t                        grid_nof_ports,
                                     srsgpu_pdsch_dmrs_plan**        plan);

/** Writes the DM-RS REs of every planned transmission into d_grids. Asynchronous on `stream`. */
int srsgpu_pdsch_dmrs_plan_execute(const srsgpu_pdsch_dmrs_plan* plan, uint32_t* d_grids, void* stream);

void srsgpu_pdsch_dmrs_plan_destroy(srsgpu_pdsch_dmrs_plan* plan);

/* ------------------------------------------------------------------------------------------------------------------
 * OFDM slot modulator / demodulator — replace srsran::ofdm_slot_modulator::modulate(span<cf_t> output,
 * const resource_grid_reader& grid, unsigned port_index, unsigned slot_index)
 * (include/srsran/phy/lower/modulation/ofdm_modulator.h:100, lib/phy/lower/modulation/ofdm_modulator_impl.cpp:115,
 * per symbol :56) and ofdm_slot_demodulator::demodulate(resource_grid_writer& grid, span<const cf_t> input,
 * unsigned port_index, unsigned slot_index) (ofdm_demodulator.h:102, ofdm_demodulator_impl.cpp:154, per symbol :94),
 * batched over every (grid, port, symbol) of a set of slots.
 * Modulator, per symbol: grid subcarriers [0, rg/2) -> DFT bins [N - rg/2, N), [rg/2, rg) -> bins [0, rg/2), inverse
 * DFT (unnormalised), times the TS 38.211 section 5.4 phase compensation (phase_compensation_lut.h) and `scale`, CP =
 * copy of the last cp_len samples. Demodulator: N samples from cp_len - window_offset, direct DFT, the same
 * compensation (receive sign) and the DFT-window phase ramp, bins back to the grid as bf16.
 * Grids: nof_ports x nsymb (14, or 12 with extended CP) x 12 * bw_rb uint32 (re | im << 16, bf16), grid g at
 * g * nof_ports * nsymb * 12 * bw_rb. Time samples: complex float (re, im) interleaved, one slot of (grid g, port p)
 * at srsgpu_ofdm_plan_sample_offset(plan, g, p) (grids, then ports, consecutively).
 * ------------------------------------------------------------------------------------------------------------------ */
typedef struct {
  uint32_t numerology;                /* subcarrier spacing 15 kHz x 2^numerology, 0..4 */
  uint32_t bw_rb;                     /* resource grid bandwidth in RB: 12 * bw_rb < dft_size */
  uint32_t dft_size;                  /* 2^n 128..8192, 3 x 2^m 384..6144, 4608 (generic DFT sizes) */
  uint32_t cp_extended;               /* 0: normal cyclic prefix (14 symbols), 1: extended (12 symbols) */
  uint32_t nof_samples_window_offset; /* demodulator DFT window advance, < 144 * dft_size / 2048 (0: none) */
  float    scale;                     /* scaling factor at the DFT output (std::isnormal) */
  double   center_freq_hz;            /* carrier centre frequency for the phase compensation */
} srsgpu_ofdm_config;

typedef struct srsgpu_ofdm_plan srsgpu_ofdm_plan;

/** Plans the modulation of nof_grids slots (grid g is slot slot_index[g] within its subframe) of nof_ports ports. */
int srsgpu_ofdm_modulator_plan_create(srsgpu_context*           ctx,
                                      const srsgpu_ofdm_config* cfg,
                                      uint32_t                  nof_grids,
                                      uint32_t                  nof_ports,
                                      const uint32_t*           slot_index,
                                      srsgpu_ofdm_plan**        plan);

/** Plans the demodulation of nof_grids slots of nof_ports ports (same layouts). */
int srsgpu_ofdm_demodulator_plan_create(srsgpu_context*           ctx,
                                        const srsgpu_ofdm_config* cfg,
                                        uint32_t                  nof_grids,
                                        uint32_t                  nof_ports,
                                        const uint32_t*           slot_index,
                                        srsgpu_ofdm_plan**        plan);

/** Symbol-granularity plans — replace srsran::ofdm_symbol_modulator::modulate(output, grid, port, symbol_index) and
 *  ofdm_symbol_demodulator::demodulate(grid, input, port, symbol_index) (include/srsran/phy/lower/modulation/
 *  ofdm_modulator.h:58, ofdm_demodulator.h:59), batched over ports and a run of consecutive symbols: symbols
 *  [first_symbol, first_symbol + nof_symbols) of slot `slot_index` of the subframe (the symbol index within the
 *  subframe the reference passes is slot_index * symbols_per_slot + first_symbol). Layouts: grid rows
 *  [port][symbol - first_symbol][subcarrier]; samples [port][CP + N of each symbol, consecutive]
 *  (srsgpu_ofdm_plan_sample_offset(plan, 0, port)). Executed with srsgpu_ofdm_(de)modulator_plan_execute. */
int srsgpu_ofdm_modulator_symbols_plan_create(srsgpu_context*           ctx,
                                              const srsgpu_ofdm_config* cfg,
                                              uint32_t                  nof_ports,
                                              uint32_t                  slot_index,
                                              uint32_t                  first_symbol,
                                              uint32_t                  nof_symbols,
                                              srsgpu_ofdm_plan**        plan);

int srsgpu_ofdm_demodulator_symbols_plan_create(srsgpu_context*           ctx,
                                                const srsgpu_ofdm_config* cfg,
                                                uint32_t                  nof_ports,
                                                uint32_t                  slot_index,
                                                uint32_t                  first_symbol,
                                                uint32_t                  nof_symbols,
                                                srsgpu_ofdm_plan**        plan);

/** Sector groups — one launch for the same symbol (or slot) of several sectors sharing a GPU, where the reference runs
 *  one lower-PHY sector per cell, each with its own OFDM objects (lib/ru/generic/ru_factory_generic_impl.cpp:75-90,
 *  lib/phy/lower/lower_phy_factory.cpp:70/:84). Concatenates the jobs of `members` (the sectors' plans, each keeping
 *  its own carrier frequency, scaling and slot/symbol positions) into one plan: member i's grids follow member i-1's
 *  (srsgpu_ofdm_plan_nof_grid_words words each) and its time samples follow member i-1's; the plan's grid g runs over
 *  the members' grids in order (srsgpu_ofdm_plan_sample_offset). The members must share direction, DFT size, bandwidth,
 *  DFT window offset and number of ports (one kernel runs every job). The members stay owned by the caller. */
int srsgpu_ofdm_plan_concat(srsgpu_context*                ctx,
                            const srsgpu_ofdm_plan* const* members,
                            uint32_t                       nof_members,
                            srsgpu_ofdm_plan**             plan);

/** One (grid, port, symbol) transform of an OFDM launch: the grid row at grid_offset (uint32 words), the symbol's
 *  cyclic prefix at sample_offset (complex samples), its length, and the phase compensation times the scaling. */
typedef struct {
  uint32_t grid_offset;
  uint32_t sample_offset;
  uint32_t cp_len;
  uint32_t reserved;
  float    coef_re;
  float    coef_im;
} srsgpu_ofdm_job;

/** The plan's jobs (one per grid, port and symbol, offsets relative to the plan's own buffers), as its launch runs
 *  them: capacity entries at most, *nof_jobs = how many the plan has. */
int srsgpu_ofdm_plan_get_jobs(const srsgpu_ofdm_plan* plan, srsgpu_ofdm_job* jobs, uint32_t capacity,
                              uint32_t* nof_jobs);

/** Runs a caller-assembled job list — the jobs of several plans (sectors, slots, symbols) at offsets of the caller's
 *  choosing within d_in / d_out — with the launch parameters of `plan` (direction, DFT size, bandwidth, DFT window
 *  offset); the jobs' plans must share them. d_jobs, d_in and d_out are device-accessible (HBM, or mapped host memory
 *  the kernel reads / writes in place). Not for the split DFT sizes (9216 .. 98304 points: their scratch is per plan).
 *  Asynchronous on `stream`. */
int srsgpu_ofdm_jobs_execute(const srsgpu_ofdm_plan* plan,
                             const srsgpu_ofdm_job*  d_jobs,
                             uint32_t                nof_jobs,
                             const void*             d_in,
                             void*                   d_out,
                             void*                   stream);

/** An OFDM job with absolute device addresses: the grid row (12 * bw_rb uint32 bf16 pairs) and the first sample of
 *  the symbol's cyclic prefix, each anywhere device-accessible — HBM, or host memory mapped for the device — so the
 *  caller's own buffers (a resource grid's rows, a radio buffer) are read or written in place. grid_copy (demodulation
 *  only, 0: none): a second row the same subcarriers are written to — the HBM copy of a mapped uplink grid that the
 *  PUSCH slot batch on the same GPU reads instead of fetching the host grid back over PCIe. */
typedef struct {
  uint64_t grid;
  uint64_t samples;
  uint32_t cp_len;
  float    coef_re;
  float    coef_im;
  uint32_t reserved;
  uint64_t grid_copy;
} srsgpu_ofdm_direct_job;

/** srsgpu_ofdm_jobs_execute over direct-address jobs (same launch parameters, same restrictions): the lower PHY's
 *  sector group demodulates straight into the rows of an uplink grid that its owner has mapped, instead of into a
 *  staging entry copied into the grid afterwards (puxch_processor_impl.cpp:78, the grid write per symbol). */
int srsgpu_ofdm_jobs_execute_direct(const srsgpu_ofdm_plan*       plan,
                                    const srsgpu_ofdm_direct_job* d_jobs,
                                    uint32_t                      nof_jobs,
                                    void*                         stream);

/** uint32 words of the plan's grids (grids x ports x symbols x 12 * bw_rb). */
uint64_t srsgpu_ofdm_plan_nof_grid_words(const srsgpu_ofdm_plan* plan);

/** Total number of complex samples of the plan's time buffer (all grids and ports). */
uint64_t srsgpu_ofdm_plan_nof_samples(const srsgpu_ofdm_plan* plan);

/** First complex sample of (grid, port) in the time buffer. */
uint64_t srsgpu_ofdm_plan_sample_offset(const srsgpu_ofdm_plan* plan, uint32_t grid, uint32_t port);

/** Modulates d_grids into d_samples. Asynchronous on `stream`, hipGraph-capturable.
 *  Concurrency: plans of the split DFT sizes (9216..98304 points) own a mutable HBM scratch row per (grid, port,
 *  symbol) job, so one such plan must not execute on two streams at the same time (order the executes, or create one
 *  plan per stream). Plans of the other sizes hold read-only state only and may run concurrently. Same for the
 *  demodulator below. */
int srsgpu_ofdm_modulator_plan_execute(const srsgpu_ofdm_plan* plan,
                                       const uint32_t*         d_grids,
                                       float*                  d_samples,
                                       void*                   stream);

/** As srsgpu_ofdm_modulator_plan_execute, every RE taken from d_twin (same layout as d_grids, e.g. the PDSCH slot
 *  batch's HBM grid) unless it holds 0xffffffff, then from d_grids (the REs the host channels wrote): the modulation
 *  of a grid whose PDSCH REs never left the GPU (lower_phy_gpu's PDxCH, downlink_processor_single_executor_impl.cpp:268
 *  send_resource_grid -> pdxch_processor_impl handle_request). Not for the split DFT sizes. */
int srsgpu_ofdm_modulator_plan_execute_twin(const srsgpu_ofdm_plan* plan,
                                            const uint32_t*         d_grids,
                                            const uint32_t*         d_twin,
                                            float*                  d_samples,
                                            void*                   stream);

/** Demodulates d_samples into d_grids (every subcarrier of every symbol is written). Asynchronous. */
int srsgpu_ofdm_demodulator_plan_execute(const srsgpu_ofdm_plan* plan,
                                         const float*            d_samples,
                                         uint32_t*               d_grids,
                                         void*                   stream);

void srsgpu_ofdm_plan_destroy(srsgpu_ofdm_plan* plan);

/* ------------------------------------------------------------------------------------------------------------------
 * PUSCH demodulator — replaces srsran::pusch_demodulator::demodulate(pusch_codeword_buffer& codeword_buffer,
 * pusch_demodulator_notifier& notifier, const resource_grid_reader& grid, const channel_estimate& estimates,
 * const configuration& config) (include/srsran/phy/upper/channel_processors/pusch/pusch_demodulator.h:95,
 * lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.cpp:272) for every PUSCH transmission of a batch of
 * slots: per data RE, channel equalization (channel_equalizer_generic_impl.cpp: ZF 1 x N, ZF 2 x N; MMSE with one
 * layer == ZF), soft demapping (demodulation_mapper_impl.cpp, the SIMD arithmetic) and descrambling
 * (c_init = rnti * 2^15 + n_id), LLRs written to the codeword buffer in the reference's order (RE, layer, bit).
 * SRSGPU_EQ_MMSE with 2..4 layers and ZF with 3..4 layers are extensions the open-source reference does not implement
 * (its equalize_mmse_* / equalize_zf_3x4 / _4x4 assert): unbiased linear MMSE.
 * Inputs: rx grids as in the OFDM demodulator (grid_nof_ports x 14 x 12 * grid_nof_prb uint32 bf16 pairs per slot);
 * channel estimates per slot [layer 0..3][port][symbol][subcarrier] bf16 pairs (srsran::channel_estimate's path-major
 * layout, channel_estimation.h:310); noise variances d_noise_var[4 * tx + port] (channel_estimate::get_noise_variance).
 * ------------------------------------------------------------------------------------------------------------------ */
/* ------------------------------------------------------------------------------------------------------------------
 * PUSCH DM-RS channel estimator — replaces srsran::dmrs_pusch_estimator::estimate(channel_estimate& estimate,
 * const resource_grid_reader& grid, const configuration& config)
 * (include/srsran/phy/upper/signal_processors/dmrs_pusch_estimator.h, lib/phy/upper/signal_processors/
 * dmrs_pusch_estimator_impl.cpp:28, port_channel_estimator_average_impl.cpp:77) for every PUSCH transmission of a
 * batch of slots, pseudo-random DM-RS sequence, the "average" (default) and "interpolate" time-domain strategies
 * (port_channel_estimator_td_interpolation_strategy), the none / mean / filter (default) frequency-domain smoothing,
 * and the estimator's CFO estimation with optional compensation (compensate_cfo, du_low's default:
 * du_low_config.h:69; port_channel_estimator_average_impl.cpp:128, :322, :475). Outputs per transmission and rx port:
 * the channel estimate of every RE of the allocation in the layout the demodulator reads, the noise variance
 * (d_noise_var[4 * tx + port]) and, when d_metrics is not NULL, SRSGPU_CHEST_METRICS floats at
 * d_metrics[SRSGPU_CHEST_METRICS * (4 * tx + port)]: RSRP, EPRE, noise variance, SNR, time alignment (seconds,
 * channel_estimate::get_time_alignment, DFT estimator time_alignment_estimator_dft_impl.cpp:178), CFO (Hz, NaN with one
 * DM-RS symbol: channel_estimate::get_cfo_Hz), 0, 0. One layer is the reference's scope
 * (port_channel_estimator_average_impl.cpp:83 asserts it); 2..4 layers (ports 1000..1003) are an extension: the w_f
 * cover code is removed over adjacent pilot pairs. Frequency hopping: the reference's PUSCH estimator never sets
 * hopping_symbol_index / rb_mask2 (dmrs_pusch_estimator_impl.cpp:107-172; only the PUCCH estimators do), so the PUSCH
 * path has no hopping to replace.
 * ------------------------------------------------------------------------------------------------------------------ */
#define SRSGPU_CHEST_FD_NONE 0
#define SRSGPU_CHEST_FD_MEAN 1
#define SRSGPU_CHEST_FD_FILTER 2
#define SRSGPU_CHEST_TD_AVERAGE 0
#define SRSGPU_CHEST_TD_INTERPOLATE 1
#define SRSGPU_CHEST_METRICS 8

/* Channel-estimate layouts (estimate_layout of the estimator and demodulator configurations). PER_SYMBOL is the
 * reference's channel_estimate: every allocated symbol holds its estimate. COMPACT stores, with the "average" time
 * strategy (one estimate for all the symbols of the allocation), only the row of start_symbol, and the demodulator
 * reads that row for every symbol: identical LLRs with 1/nof_symbols of the estimate traffic. With CFO compensation
 * (compensate_cfo and >= 2 DM-RS symbols) the row holds the unrotated estimate and the first allocated element of the
 * next row the normalised CFO (float32 bits); the demodulator (cfo_compensated = 1) applies each symbol's rotation
 * in bf16 exactly as the estimator would have written it. The "interpolate" strategy needs PER_SYMBOL. */
#define SRSGPU_CE_PER_SYMBOL 0
#define SRSGPU_CE_COMPACT 1

typedef struct {
  uint16_t scrambling_id;    /* N_ID^{n_SCID}, 0..65535 */
  uint8_t  n_scid;           /* 0 or 1 */
  uint8_t  dmrs_type;        /* 1 or 2 */
  uint8_t  nof_tx_layers;    /* 1..4 */
  uint8_t  nof_rx_ports;     /* ports 0..n-1 of the grid */
  uint8_t  start_symbol;     /* first_symbol */
  uint8_t  nof_symbols;      /* start_symbol + nof_symbols <= 14 */
  uint16_t dmrs_symbol_mask; /* symbols_mask: DM-RS symbols, inside [start_symbol, start_symbol + nof_symbols) */
  uint16_t rb_start;         /* contiguous CRB allocation (rb_mask) */
  uint16_t nof_rb;
  uint16_t slot_index;       /* n_slot within the frame (DM-RS c_init) */
  uint8_t  fd_smoothing;     /* SRSGPU_CHEST_FD_* */
  uint8_t  estimate_layout;  /* SRSGPU_CE_PER_SYMBOL or SRSGPU_CE_COMPACT */
  uint8_t  td_strategy;      /* SRSGPU_CHEST_TD_AVERAGE or SRSGPU_CHEST_TD_INTERPOLATE */
  uint8_t  compensate_cfo;   /* 1: compensate the estimated CFO (needs >= 2 DM-RS symbols to act) */
  float    scaling;          /* beta_PUSCH^DMRS (DM-RS amplitude relative to data), > 0 */
  uint32_t grid_index;       /* slot of the rx grid and of the estimate buffer */
  uint8_t  numerology;       /* subcarrier spacing 15 kHz x 2^numerology (0..4), normal cyclic prefix */
  uint8_t  dmrs_sequence;    /* SRSGPU_DMRS_PSEUDO_RANDOM (scrambling_id, n_scid) or SRSGPU_DMRS_LOW_PAPR (transform
                                precoding: scrambling_id = n_RS_ID 0..1007, the group n_RS_ID mod 30 sequence on every
                                DM-RS symbol, dmrs_pusch_estimator_impl.cpp:77; one layer, type 1) */
  uint8_t  pad[2];
} srsgpu_pusch_chest_config;
#define SRSGPU_DMRS_PSEUDO_RANDOM 0
#define SRSGPU_DMRS_LOW_PAPR 1

typedef struct srsgpu_pusch_chest_plan srsgpu_pusch_chest_plan;

int srsgpu_pusch_chest_plan_create(srsgpu_context*                  ctx,
                                   const srsgpu_pusch_chest_config* cfgs,
                                   uint32_t                         nof_tx,
                                   uint32_t                         grid_nof_prb,
                                   uint32_t                         grid_nof_ports,
                                   srsgpu_pusch_chest_plan**        plan);

/** As srsgpu_pusch_chest_plan_create with an optional allocation extension per transmission (exts may be NULL):
 *  srsgpu_alloc_ext::crb_mask is configuration::rb_mask. The pilots of the allocated CRBs (the sequence skipping the
 *  unallocated ones, dmrs_helper.cpp:64) are smoothed and interpolated as one band, the time alignment takes the RE-mask
 *  path (port_channel_estimator_helpers.cpp:285), and PRB i of the band is written at the i-th allocated CRB. (The
 *  reference writes every PRB of a non-contiguous mask at the lowest CRB instead, port_channel_estimator_average_impl.cpp:
 *  297: DESIGN.md.) Reserved patterns and PRGs are rejected. */
int srsgpu_pusch_chest_plan_create_ex(srsgpu_context*                  ctx,
                                      const srsgpu_pusch_chest_config* cfgs,
                                      const srsgpu_alloc_ext*          exts,
                                      uint32_t                         nof_tx,
                                      uint32_t                         grid_nof_prb,
                                      uint32_t                         grid_nof_ports,
                                      srsgpu_pusch_chest_plan**        plan);

/** Estimates every planned transmission: reads d_grids, writes d_ch_estimates (slot layout [layer 0..3][port]
 *  [symbol][subcarrier], only the allocated REs), d_noise_var and optionally d_metrics (SRSGPU_CHEST_METRICS floats
 *  per transmission and port). Asynchronous on `stream`. */
int srsgpu_pusch_chest_plan_execute(const srsgpu_pusch_chest_plan* plan,
                                    const uint32_t*                d_grids,
                                    uint32_t*                      d_ch_estimates,
                                    float*                         d_noise_var,
                                    float*                         d_metrics,
                                    void*                          stream);

void srsgpu_pusch_chest_plan_destroy(srsgpu_pusch_chest_plan* plan);

#define SRSGPU_EQ_ZF 0
#define SRSGPU_EQ_MMSE 1

typedef struct {
  uint16_t rnti;                        /* n_RNTI */
  uint16_t n_id;                        /* n_ID, 0..1023 */
  uint8_t  modulation_order;            /* Qm: 2, 4, 6, 8 */
  uint8_t  nof_tx_layers;               /* 1..4 */
  uint8_t  nof_rx_ports;                /* 1..grid_nof_ports (ports 0..n-1) */
  uint8_t  start_symbol;
  uint8_t  nof_symbols;                 /* start_symbol + nof_symbols <= 14 */
  uint8_t  dmrs_type;                   /* 1 or 2 */
  uint8_t  nof_cdm_groups_without_data; /* 1..2 (type 1), 1..3 (type 2) */
  uint8_t  equalizer;                   /* SRSGPU_EQ_ZF or SRSGPU_EQ_MMSE */
  uint16_t dmrs_symbol_mask;            /* bit l = OFDM symbol l carries DM-RS */
  uint16_t rb_start;                    /* contiguous CRB allocation [rb_start, rb_start + nof_rb) (rb_mask) */
  uint16_t nof_rb;
  uint8_t  estimate_layout;             /* SRSGPU_CE_PER_SYMBOL or SRSGPU_CE_COMPACT (as the estimator wrote it) */
  uint8_t  cfo_compensated;             /* COMPACT only: the estimator compensated the CFO (its compensate_cfo) */
  uint32_t grid_index;                  /* slot (rx grid and channel estimate) of the transmission */
  uint32_t llr_offset;                  /* first codeword LLR in the output buffer */
  uint8_t  numerology;                  /* COMPACT + cfo_compensated: subcarrier spacing of the symbol epochs */
  uint8_t  transform_precoding;         /* 1: transform precoding (DFT-s-OFDM; one layer, every data symbol's REs a
                                           multiple of 12 with 2^a 3^b 5^c PRBs, TS 38.211 section 6.3.1.4):
                                           configuration::enable_transform_precoding, pusch_demodulator_impl.cpp:346 */
  uint8_t  pad2[2];
} srsgpu_pusch_demod_config;

typedef struct srsgpu_pusch_demodulator_plan srsgpu_pusch_demodulator_plan;

/** Validates the transmissions (supported layer / port / modulation combinations, allocation inside the grid) and
 *  uploads the work. */
int srsgpu_pusch_demodulator_plan_create(srsgpu_context*                  ctx,
                                         const srsgpu_pusch_demod_config* cfgs,
                                         uint32_t                         nof_tx,
                                         uint32_t                         grid_nof_prb,
                                         uint32_t                         grid_nof_ports,
                                         srsgpu_pusch_demodulator_plan**  plan);

/** Number of codeword LLRs of transmission `tx` (data REs x layers x Qm). */
uint32_t srsgpu_pusch_demodulator_plan_nof_llrs(const srsgpu_pusch_demodulator_plan* plan, uint32_t tx);

/** Demodulates every planned transmission into d_llrs. Asynchronous on `stream`, hipGraph-capturable. */
int srsgpu_pusch_demodulator_plan_execute(const srsgpu_pusch_demodulator_plan* plan,
                                          const uint32_t*                      d_grids,
                                          const uint32_t*                      d_ch_estimates,
                                          const float*                         d_noise_var,
                                          int8_t*                              d_llrs,
                                          void*                                stream);

void srsgpu_pusch_demodulator_plan_destroy(srsgpu_pusch_demodulator_plan* plan);

/** As srsgpu_pusch_demodulator_plan_create with an optional allocation extension per transmission (exts may be NULL):
 *  srsgpu_alloc_ext::crb_mask is configuration::rb_mask (any CRB pattern; data REs in symbol-major, ascending-subcarrier
 *  order, pusch_demodulator_impl.cpp:290); reserved patterns and PRGs are rejected (the demodulator has neither). */
int srsgpu_pusch_demodulator_plan_create_ex(srsgpu_context*                  ctx,
                                            const srsgpu_pusch_demod_config* cfgs,
                                            const srsgpu_alloc_ext*          exts,
                                            uint32_t                         nof_tx,
                                            uint32_t                         grid_nof_prb,
                                            uint32_t                         grid_nof_ports,
                                            srsgpu_pusch_demodulator_plan**  plan);

/** Copies the descrambling sequence of transmission tx (TS 38.211 section 5.2.1, c_init = rnti 2^15 + n_id: the
 *  sequence pusch_demodulator_impl.cpp:277 generates and passes to pusch_codeword_buffer::on_new_block) into d_words:
 *  ceil(nof_llrs / 32) 32-bit words, bit 31 of word w = c(32 w) (the plan keeps it resident). Asynchronous. */
int srsgpu_pusch_demodulator_plan_scrambling(const srsgpu_pusch_demodulator_plan* plan,
                                             uint32_t                             tx,
                                             uint32_t*                            d_words,
                                             void*                                stream);

/* Post-equalization statistics (pusch_demodulator_notifier::demodulation_stats, pusch_demodulator_impl.cpp:355-443):
 * SRSGPU_DEMOD_STATS floats per transmission, rows 0..13 = OFDM symbol l (on_provisional_stats) and row 14 = the whole
 * transmission (on_end_stats), each (SINR dB, EVM): SINR = -10 log10(mean of the finite equalizer noise variances,
 * after transform deprecoding) or +inf, EVM = sqrt(mean |modulate(hard decisions) - equalized symbol|^2) per symbol
 * (evm_calculator_generic_impl.cpp), the total EVM weighting each symbol's by its size. NaN rows: no data REs. */
#define SRSGPU_DEMOD_STATS 30

/** As srsgpu_pusch_demodulator_plan_execute, and when d_stats is not NULL also writes the statistics of every
 *  transmission (d_stats[SRSGPU_DEMOD_STATS * tx + 2 * row + {0: SINR dB, 1: EVM}]). Asynchronous, hipGraph-capturable
 *  (the plan's accumulators are reset by the same execute). */
int srsgpu_pusch_demodulator_plan_execute_ex(const srsgpu_pusch_demodulator_plan* plan,
                                             const uint32_t*                      d_grids,
                                             const uint32_t*                      d_ch_estimates,
                                             const float*                         d_noise_var,
                                             int8_t*                              d_llrs,
                                             float*                               d_stats,
                                             void*                                stream);

/* ------------------------------------------------------------------------------------------------------------------
 * UL-SCH demultiplexer (UCI on PUSCH, TS 38.212 section 6.2.7) — replaces srsran::ulsch_demultiplex::demultiplex /
 * set_csi_part2 (include/srsran/phy/upper/channel_processors/pusch/ulsch_demultiplex.h:64,
 * lib/phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.cpp:199) for every transmission of a batch: routes the
 * demodulated, descrambled codeword LLRs (the PUSCH demodulator's output, RE by RE) to the UL-SCH data stream (the PUSCH
 * decoder's input; REs carrying HARQ-ACK of <= 2 bits stay in it as zeros), HARQ-ACK, CSI Part 1 and CSI Part 2 LLR
 * streams, with the reference's 1- / 2-bit UCI placeholder handling (the scrambling sequence c_init = rnti 2^15 + n_id
 * re-applied to the "y" and "x" placeholder bits, :91 / :131). The RE sets per OFDM symbol (reserved HARQ-ACK REs,
 * HARQ-ACK, CSI Part 1, CSI Part 2, :316) are fixed at plan creation; CSI Part 2 is placed from csi2_first_symbol on
 * (0: as if set_csi_part2 were called before the first symbol). Input and output offsets are in LLRs.
 * ------------------------------------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t  modulation_order;            /* Qm: 2, 4, 6, 8 */
  uint8_t  nof_layers;                  /* 1..4 */
  uint16_t nof_prb;                     /* allocated PRBs (count) */
  uint8_t  start_symbol;                /* start_symbol_index */
  uint8_t  nof_symbols;
  uint16_t dmrs_symbol_mask;            /* DM-RS symbols */
  uint8_t  dmrs_type;                   /* 1 or 2 */
  uint8_t  nof_cdm_groups_without_data; /* 1..2 (type 1), 1..3 (type 2) */
  uint16_t rnti;                        /* scrambling c_init = rnti 2^15 + n_id (placeholders) */
  uint16_t n_id;
  uint16_t csi2_first_symbol;           /* CSI Part 2 REs only in OFDM symbols >= this one: the symbol whose
                                           demultiplexing completes CSI Part 1, where the reference's processor calls
                                           set_csi_part2 (pusch_processor_impl.cpp:72-100, ulsch_demultiplex_impl.cpp:241)
                                           0: from the first symbol, as if set before it */
  uint32_t nof_harq_ack_rvd;            /* G^HARQ-ACK_rvd */
  uint32_t nof_harq_ack_bits;           /* O^HARQ-ACK */
  uint32_t nof_enc_harq_ack_bits;       /* G^HARQ-ACK */
  uint32_t nof_csi_part1_bits;          /* O^CSI-1 */
  uint32_t nof_enc_csi_part1_bits;      /* G^CSI-1 */
  uint32_t nof_csi_part2_bits;          /* O^CSI-2 */
  uint32_t nof_enc_csi_part2_bits;      /* G^CSI-2 (0: none) */
  uint32_t llr_offset;                  /* first codeword LLR in the input */
  uint32_t sch_offset;                  /* first UL-SCH LLR in d_sch */
  uint32_t harq_offset;                 /* first HARQ-ACK LLR in d_harq */
  uint32_t csi1_offset;                 /* first CSI Part 1 LLR in d_csi1 */
  uint32_t csi2_offset;                 /* first CSI Part 2 LLR in d_csi2 */
} srsgpu_ulsch_demux_config;

typedef struct srsgpu_ulsch_demux_plan srsgpu_ulsch_demux_plan;

/** Validates the transmissions (every UCI field must fit the allocation, as the reference asserts at the end of the
 *  codeword) and uploads the RE routing. */
int srsgpu_ulsch_demux_plan_create(srsgpu_context*                  ctx,
                                   const srsgpu_ulsch_demux_config* cfgs,
                                   uint32_t                         nof_tx,
                                   srsgpu_ulsch_demux_plan**        plan);

/** LLRs of transmission tx: stream 0 = codeword (input), 1 = UL-SCH, 2 = HARQ-ACK, 3 = CSI Part 1, 4 = CSI Part 2. */
uint32_t srsgpu_ulsch_demux_plan_nof_llrs(const srsgpu_ulsch_demux_plan* plan, uint32_t tx, uint32_t stream);

/** LLRs of `stream` (as above) that transmission tx's OFDM symbol l (0..13, slot numbering) carries: counts[l]. The
 *  reference's demultiplexer hands a UCI field's LLRs to its decoder buffer while it demultiplexes the symbol that holds
 *  them and ends the field in the symbol that completes it (ulsch_demultiplex_impl.cpp:474-576); a host that replays
 *  the GPU's streams into the reference's UCI decoders feeds them symbol by symbol with these counts. */
int srsgpu_ulsch_demux_plan_symbol_llrs(const srsgpu_ulsch_demux_plan* plan, uint32_t tx, uint32_t stream,
                                        uint32_t counts[14]);

/** Demultiplexes every planned transmission. Asynchronous on `stream`, hipGraph-capturable. Output pointers of streams
 *  no transmission uses may be NULL. */
int srsgpu_ulsch_demux_plan_execute(const srsgpu_ulsch_demux_plan* plan,
                                    const int8_t*                  d_llrs,
                                    int8_t*                        d_sch,
                                    int8_t*                        d_harq,
                                    int8_t*                        d_csi1,
                                    int8_t*                        d_csi2,
                                    void*                          stream);

void srsgpu_ulsch_demux_plan_destroy(srsgpu_ulsch_demux_plan* plan);

/* ------------------------------------------------------------------------------------------------------------------
 * PUSCH decoder (transport-block level) — replaces srsran::pusch_decoder (include/srsran/phy/upper/channel_processors/
 * pusch/pusch_decoder.h; lib/phy/upper/channel_processors/pusch/pusch_decoder_impl.cpp: new_data :98, segmentation
 * :190, codeblock tasks :283, join_and_notify :386): segmentation, per-codeblock rate dematching + HARQ combining +
 * LDPC decoding + CB CRC, codeblock concatenation and TB CRC24A check, for every transport block of a slot.
 * The HARQ context lives in device memory owned by the caller: d_harq (C * N_short * Z LLRs per TB), d_cb_crc_ok (one
 * flag per codeblock) and d_cb_msgs (SRSGPU_CB_MSG_STRIDE bytes of decoded message per codeblock).
 * ------------------------------------------------------------------------------------------------------------------ */
#define SRSGPU_CB_MSG_STRIDE 1056u /* bytes per codeblock message slot (22 * 384 bits) */

typedef struct {
  uint8_t  base_graph;       /* 1 or 2 */
  uint8_t  rv;               /* 0..3 */
  uint8_t  modulation_order; /* Qm */
  uint8_t  nof_layers;       /* 1..4 */
  uint8_t  new_data;         /* 1: new transmission (resets the TB's CB CRC flags) */
  uint8_t  use_early_stop;   /* LDPC early stop with the codeblock CRC */
  uint8_t  max_iterations;   /* nof_ldpc_iterations (> 0) */
  uint8_t  reserved;
  float    scaling_factor;   /* normalised min-sum factor in (0, 1) */
  uint32_t tbs_bytes;        /* transport block size in bytes */
  uint32_t nof_ch_symbols;   /* G / Qm */
  uint32_t Nref;             /* limited-buffer rate matching N_ref, 0 = none */
  uint32_t llr_offset;       /* first of the G codeword LLRs */
  uint32_t harq_offset;      /* first LLR of the TB's HARQ soft buffer */
  uint32_t cb_offset;        /* index of the TB's first codeblock (CRC flags, messages, iteration counts) */
  uint32_t tb_offset;        /* byte offset of the decoded transport block */
} srsgpu_pusch_tb_config;

typedef struct srsgpu_pusch_decoder_plan srsgpu_pusch_decoder_plan;

int srsgpu_pusch_decoder_plan_create(srsgpu_context*               ctx,
                                     int                           impl,
                                     const srsgpu_pusch_tb_config* cfgs,
                                     uint32_t                      nof_tbs,
                                     srsgpu_pusch_decoder_plan**   plan);

uint32_t srsgpu_pusch_decoder_plan_nof_codeblocks(const srsgpu_pusch_decoder_plan* plan);

/** Number of LLR bytes the LDPC decoder stage moves per execute: every codeblock's span of the HARQ buffer, trimmed to
 *  the rate dematcher's zero tail for new transmissions (what decode() would trim to, ldpc_decoder_impl.cpp:94); for
 *  a codeblock whose rate dematching the decoder performs itself (first transmissions that are a plain copy), the E
 *  codeword LLRs it reads plus the N HARQ bytes it writes. For traffic accounting. */
uint64_t srsgpu_pusch_decoder_plan_decoder_input_llrs(const srsgpu_pusch_decoder_plan* plan);

/** Decodes the planned transport blocks. d_tb_crc_ok[t] = 1 when the TB CRC passed (pusch_decoder_result
 *  tb_crc_ok); d_cb_nof_iterations[c] as in srsgpu_pusch_cb_plan_execute. Asynchronous, hipGraph-capturable.
 *  A plan of at most 8 large segmented TBs runs its TB stage over slices whose CRC sums live in the plan (reset by
 *  every execute): executes (and assembles) of one plan must be ordered, e.g. on one stream, never concurrent. */
int srsgpu_pusch_decoder_plan_execute(const srsgpu_pusch_decoder_plan* plan,
                                      const int8_t*                    d_llrs,
                                      int8_t*                          d_harq,
                                      uint8_t*                         d_cb_crc_ok,
                                      uint8_t*                         d_cb_msgs,
                                      int32_t*                         d_cb_nof_iterations,
                                      uint8_t*                         d_tbs,
                                      uint8_t*                         d_tb_crc_ok,
                                      void*                            stream);

/** As srsgpu_pusch_decoder_plan_execute, with codeblock c's HARQ soft buffer (N bytes, the rate dematcher's output and
 *  the decoder's input) at d_harq_cbs[c], c = srsgpu_pusch_tb_config::cb_offset + the codeblock's index in its TB (the
 *  index of its CRC flag and message) - a device array covering every such index of the plan, e.g. the slots of
 *  a persistent rx-buffer arena (the reference's rx_buffer.h:72 get_codeblock_soft_bits for the codeblock's absolute
 *  identifier, :65) - instead of at d_harq + srsgpu_pusch_tb_config::harq_offset. The soft bits stay in the arena: no
 *  copy into a batch buffer before the decode and back after it (srsgpu_harq_copy_arenas). Asynchronous,
 *  hipGraph-capturable (the pointer array may change between replays). */
int srsgpu_pusch_decoder_plan_execute_arena(const srsgpu_pusch_decoder_plan* plan,
                                            const int8_t*                    d_llrs,
                                            int8_t* const*                   d_harq_cbs,
                                            uint8_t*                         d_cb_crc_ok,
                                            uint8_t*                         d_cb_msgs,
                                            int32_t*                         d_cb_nof_iterations,
                                            uint8_t*                         d_tbs,
                                            uint8_t*                         d_tb_crc_ok,
                                            void*                            stream);

/** The transport-block stage alone (pusch_decoder_impl.cpp:386 join_and_notify, :438 concatenate_codeblocks): TB
 *  assembly from the codeblock messages and flags already in d_cb_msgs / d_cb_crc_ok (the plan's codeblock layout,
 *  SRSGPU_CB_MSG_STRIDE bytes per codeblock) and the TB CRC24A check; a TB CRC mismatch clears the TB's codeblock
 *  flags, as execute does. For codeblocks decoded elsewhere: codeblock-sharded decoding, where every rank runs the
 *  srsgpu_pusch_cb_plan of its codeblock range and the FAPI rank gathers the messages and flags (srsgpu/dist.py
 *  CodeblockShard). Asynchronous, hipGraph-capturable. */
int srsgpu_pusch_decoder_plan_assemble(const srsgpu_pusch_decoder_plan* plan,
                                       uint8_t*                         d_cb_crc_ok,
                                       const uint8_t*                   d_cb_msgs,
                                       uint8_t*                         d_tbs,
                                       uint8_t*                         d_tb_crc_ok,
                                       void*                            stream);

void srsgpu_pusch_decoder_plan_destroy(srsgpu_pusch_decoder_plan* plan);

/** HARQ soft buffers kept across slots in a persistent arena, one slot of arena_stride bytes per absolute codeblock
 *  identifier (the reference's rx buffer pool: rx_buffer.h:65 get_absolute_codeblock_id, :72 get_codeblock_soft_bits),
 *  moved to / from a slot batch's contiguous HARQ buffer (srsgpu_pusch_tb_config::harq_offset layout) around a
 *  srsgpu_pusch_decoder_plan_execute. d_jobs: device array of nof_jobs entries. Asynchronous on `stream`. */
#define SRSGPU_HARQ_TO_BATCH 0
#define SRSGPU_HARQ_TO_ARENA 1
typedef struct {
  uint32_t slot;         /* arena slot (absolute codeblock identifier) */
  uint32_t batch_offset; /* first byte of the codeblock's soft bits in the batch HARQ buffer */
  uint32_t bytes;        /* soft bits to move (N of the codeblock) */
  uint32_t arena;        /* srsgpu_harq_copy_arenas: index into the arena table (0 for srsgpu_harq_copy) */
} srsgpu_harq_copy_job;

int srsgpu_harq_copy(srsgpu_context*             ctx,
                     int                         direction,
                     int8_t*                     d_arena,
                     uint32_t                    arena_stride,
                     int8_t*                     d_batch,
                     const srsgpu_harq_copy_job* d_jobs,
                     uint32_t                    nof_jobs,
                     void*                       stream);

/** As srsgpu_harq_copy over several arenas in one launch (the rx buffer pools of several sectors, whose slots one
 *  GPU service batch gathers): job j moves between arena d_arenas[j.arena] (a device array of arena base pointers)
 *  and the batch buffer. */
int srsgpu_harq_copy_arenas(srsgpu_context*             ctx,
                            int                         direction,
                            int8_t* const*              d_arenas,
                            uint32_t                    arena_stride,
                            int8_t*                     d_batch,
                            const srsgpu_harq_copy_job* d_jobs,
                            uint32_t                    nof_jobs,
                            void*                       stream);

/** A list of copies as one launch: span i copies bytes bytes (a multiple of 16, 16-byte aligned addresses) from src to
 *  dst; src / dst device-accessible (HBM, or mapped host memory the kernel reads or writes in place). d_spans itself is
 *  device-accessible; max_bytes = the largest span. Replaces the per-slot rx-grid upload of a slot batch (one
 *  hipMemcpyAsync per slot: the DMA engines manage ~29 GB/s for 0.5–1 MB copies where a kernel reading mapped memory
 *  reaches 37–50 GB/s, profiles/r5_pcie_probe.txt). Asynchronous on `stream`. */
typedef struct {
  const void* src;
  void*       dst;
  uint64_t    bytes;
} srsgpu_copy_span;

int srsgpu_copy_spans(const srsgpu_copy_span* d_spans, uint32_t nof_spans, uint64_t max_bytes, void* stream);

/** As srsgpu_copy_spans, but each 32-bit word of a source replaces the destination's only when it is not `sentinel`:
 *  the gather of a multi-device PDSCH slot batch, whose shards map their UEs' REs into sentinel-filled grids and merge
 *  their bands into the root device's grid (peer reads over xGMI) before its one download
 *  (downlink_processor_single_executor_impl.cpp:268-274 sends one grid per slot). */
int srsgpu_merge_spans(const srsgpu_copy_span* d_spans,
                       uint32_t                nof_spans,
                       uint64_t                max_bytes,
                       uint32_t                sentinel,
                       void*                   stream);

/** As srsgpu_pusch_chest_plan_execute, with the span copies d_spans[0, nof_spans) (each as in srsgpu_copy_spans,
 *  max_bytes the largest) done in the same launch by extra workgroups while the estimator's run: for a slot batch whose rx
 *  grids are read from mapped host memory, the data-symbol rows, which the estimator does not read, arrive while it
 *  works on the DM-RS rows copied before (pusch_processor_impl.cpp:165-213 estimates from the DM-RS symbols only). */
int srsgpu_pusch_chest_plan_execute_copy(const srsgpu_pusch_chest_plan* plan,
                                         const uint32_t*                d_grids,
                                         uint32_t*                      d_ch_estimates,
                                         float*                         d_noise_var,
                                         float*                         d_metrics,
                                         const srsgpu_copy_span*        d_spans,
                                         uint32_t                       nof_spans,
                                         uint64_t                       max_bytes,
                                         void*                          stream);

/** Stage timing: with enable = 1 every execute records HIP events on its stream around the three kernel stages
 *  (0: rate dematching, 1: LDPC decoding, 2: TB assembly + CRC); with enable = 2 only around the decoding stage (two
 *  events: the least perturbation of a timed run); 0 disables. stage_times synchronises on them and returns the
 *  accumulated milliseconds per stage (ms[3], stages not timed read 0) and the number of executes since the previous
 *  call. */
int srsgpu_pusch_decoder_plan_enable_timing(srsgpu_pusch_decoder_plan* plan, int enable);
int srsgpu_pusch_decoder_plan_stage_times(srsgpu_pusch_decoder_plan* plan, float* ms, uint32_t* nof_executes);

#ifdef __cplusplus
}
#endif

#endif /* SRSGPU_PHY_H */
