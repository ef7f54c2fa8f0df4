// Host-side internals shared by the C-ABI translation units (capi*.cpp): error reporting, the device context and the
// per-stage event timer. Not part of the public C ABI.
#pragma once

#include "srsgpu_phy.h"
#include "srsgpu_internal.h"
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <map>
#include <tuple>
#include <mutex>
#include <string>
#include <vector>

namespace srsgpu {

/// Stores the thread-local message returned by srsgpu_last_error().
void set_last_error(const char* msg);

inline int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char* fmt, ...)
{
  char    buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  set_last_error(buf);
  return code;
}

#define HIP_TRY(expr)                                                                                                  \
  do {                                                                                                                 \
    hipError_t err_ = (expr);                                                                                          \
    if (err_ != hipSuccess) {                                                                                          \
      return fail(SRSGPU_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(err_));                                    \
    }                                                                                                                  \
  } while (0)

constexpr size_t CRC_ARENA_WORDS = 16u << 20;  // 64 MiB of contribution tables
/// Optional (fast-path) tables are only placed while at least this many arena words stay free for required ones.
constexpr size_t CRC_ARENA_RESERVE = CRC_ARENA_WORDS / 4;


using crc_key = std::tuple<int, int, int>;  ///< (polynomial, message length, zero words after the entries)

/// One contribution table in the arena: referenced by live plans (refs) or cached for reuse (refs == 0, evictable
/// least recently used first when an allocation does not fit).
struct crc_entry {
  size_t   offset   = 0;
  size_t   words    = 0;
  int      refs     = 0;
  uint64_t last_use = 0;
};

} // namespace srsgpu

struct srsgpu_context {
  int                                  device      = 0;
  uint16_t*                            d_shifts[2] = {nullptr, nullptr};
  uint32_t*                            d_shifts32[2] = {nullptr, nullptr};  ///< Same, one dword per shift (decoder).
  /// Packed decoder address constants A | B << 16 per (Z position, edge), see ldpc_decoder_pk.hip (even Z only).
  uint32_t*                            d_pair_ab[2] = {nullptr, nullptr};
  uint32_t*                            d_pair_ab2[2] = {nullptr, nullptr};  ///< Same for the two-codeblock image.
  srsgpu::core_plan*                   d_core[2]   = {nullptr, nullptr};
  std::vector<srsgpu::core_plan>       core[2];
  uint32_t*                            d_crc_arena = nullptr;
  /// Slice-by-4 byte tables (srsgpu::CRC_SLICE_WORDS per polynomial: CRC24A, CRC24B, CRC16), T_k[v] = v x^(order + 8 k)
  /// mod g, k = 0..3.
  uint32_t*                            d_crc_slice = nullptr;
  std::map<srsgpu::crc_key, srsgpu::crc_entry> crc_tables;
  std::map<size_t, size_t>             crc_free = {{0, srsgpu::CRC_ARENA_WORDS}};  ///< Free blocks: offset -> words.
  uint64_t                             crc_clock = 0;
  /// Gold-sequence jump tables of the scrambler (built on first use, see srsgpu::gold_tables): x1 words, x2 chunk
  /// jumps M^(Nc + 2048 c) and x2 lane jumps M^(32 i), each matrix as 31 column words.
  uint32_t*                            d_gold_x1      = nullptr;
  uint32_t*                            d_gold_x2_jump = nullptr;
  uint32_t*                            d_gold_x2_lane = nullptr;
  /// OFDM DFT twiddles exp(-j 2 pi m / OFDM_MAX_DFT) as (re, im) floats (built on first use).
  float*                               d_ofdm_twiddles = nullptr;
  /// srsgpu_option values (srsgpu_context_set_option), read at plan creation.
  int opt_decoder_split         = -1;
  int opt_decoder_pairs         = 0;
  int opt_decoder_fused_dematch = 1;
  int opt_encoder_byte_kernel   = 0;
  int opt_encoder_zero_output   = 0;
  std::mutex                           mtx;
};

namespace srsgpu {
/// Drops a plan's references on CRC contribution tables (caller holds ctx->mtx); the tables stay cached.
inline void crc_release_locked(srsgpu_context* ctx, std::vector<crc_key>& refs)
{
  for (const crc_key& k : refs) {
    auto it = ctx->crc_tables.find(k);
    if (it != ctx->crc_tables.end() && it->second.refs > 0) {
      --it->second.refs;
    }
  }
  refs.clear();
}

/// Releases the references taken during a plan creation unless they are committed to the plan (caller holds the lock
/// for the guard's whole life).
struct crc_ref_guard {
  srsgpu_context*      ctx;
  std::vector<crc_key> refs;
  explicit crc_ref_guard(srsgpu_context* c) : ctx(c) {}
  crc_ref_guard(const crc_ref_guard&)            = delete;
  crc_ref_guard& operator=(const crc_ref_guard&) = delete;
  void commit(std::vector<crc_key>& dst) { dst.swap(refs); refs.clear(); }
  ~crc_ref_guard() { crc_release_locked(ctx, refs); }
};

/// Builds and uploads the Gold-sequence jump tables into the context once (caller holds ctx->mtx); capi_pdsch_mod.cpp.
int ensure_gold_tables(srsgpu_context* ctx);

/// A plan's (de)scrambling sequences, resident in HBM for the plan's lifetime: word offsets of every transmission
/// (offsets[t], filled here from nwords) and the buffer, filled once on the device (launch_gold_fill) and synchronised.
/// Caller holds ctx->mtx and has called ensure_gold_tables.
int build_gold_sequences(srsgpu_context*              ctx,
                         const std::vector<uint32_t>& c_inits,
                         const std::vector<uint32_t>& nwords,
                         const std::vector<uint32_t>& offsets,
                         uint32_t**                   d_seq,
                         const std::vector<uint32_t>* wstart = nullptr);

/// Word offsets of the transmissions' sequences in a plan's sequence buffer (each padded by one word).
std::vector<uint32_t> gold_sequence_offsets(const std::vector<uint32_t>& nwords);
} // namespace srsgpu

/// Per-stage device time accounting: HIP events recorded around every kernel stage on the execution stream.
struct stage_timer {
  bool                                  enabled = false;
  int                                   stages  = 0;
  std::vector<std::vector<hipEvent_t>>  pending;  ///< One event set (stages + 1) per timed execute.
  std::vector<std::vector<hipEvent_t>>  pool;
  std::vector<double>                   acc_ms;
  uint32_t                              count = 0;

  ~stage_timer()
  {
    for (auto* v : {&pending, &pool}) {
      for (auto& set : *v) {
        for (hipEvent_t e : set) {
          (void)hipEventDestroy(e);
        }
      }
    }
  }
  /// Returns the event set for this execute (nullptr when disabled).
  std::vector<hipEvent_t>* begin()
  {
    if (!enabled) {
      return nullptr;
    }
    if (pool.empty()) {
      std::vector<hipEvent_t> set(static_cast<size_t>(stages) + 1);
      for (auto& e : set) {
        if (hipEventCreate(&e) != hipSuccess) {
          return nullptr;
        }
      }
      pool.push_back(std::move(set));
    }
    pending.push_back(std::move(pool.back()));
    pool.pop_back();
    return &pending.back();
  }
  static void mark(std::vector<hipEvent_t>* set, int i, hipStream_t s)
  {
    if (set != nullptr) {
      (void)hipEventRecord((*set)[static_cast<size_t>(i)], s);
    }
  }
  /// Synchronises on the pending events and accumulates the stage durations.
  int collect(float* out_ms, uint32_t* nof_executes)
  {
    acc_ms.resize(static_cast<size_t>(stages), 0.0);
    for (auto& set : pending) {
      if (hipEventSynchronize(set.back()) != hipSuccess) {
        return -1;
      }
      for (int i = 0; i < stages; ++i) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, set[static_cast<size_t>(i)], set[static_cast<size_t>(i) + 1]) != hipSuccess) {
          return -1;
        }
        acc_ms[static_cast<size_t>(i)] += ms;
      }
      ++count;
      pool.push_back(std::move(set));
    }
    pending.clear();
    for (int i = 0; i < stages; ++i) {
      out_ms[i] = static_cast<float>(acc_ms[static_cast<size_t>(i)]);
    }
    *nof_executes = count;
    std::fill(acc_ms.begin(), acc_ms.end(), 0.0);
    count = 0;
    return 0;
  }
};


namespace srsgpu {

constexpr double T_C = 1.0 / (480000.0 * 4096.0);  // phy_time_unit::T_C

/// initialize_symbol_start_epochs (port_channel_estimator_average_impl.cpp:496), normal CP, with the reference's
/// float / double mix: each CP duration in seconds (double) times the SCS, accumulated into float. The +16 kappa CP
/// (cyclic_prefix::get_length, cyclic_prefix.h:93) applies to symbols 0 and 7 * 2^mu of the slot.
inline void symbol_start_epochs(unsigned mu, float* ep)
{
  const double khz = 15u << mu;
  for (unsigned i = 0; i < 14; ++i) {
    const unsigned kappa = (144u >> mu) + ((i == 0 || i == (7u << mu)) ? 16u : 0u);
    const double   cp_s  = static_cast<double>(kappa * 64u) * T_C;
    ep[i] = (i == 0) ? static_cast<float>(cp_s * khz * 1000) : static_cast<float>(ep[i - 1] + cp_s * khz * 1000 + 1.0F);
  }
}

} // namespace srsgpu

namespace srsgpu {

/// Data resource elements of a transmission in mapping order (resource_grid_mapper_impl.cpp:269: symbol-major,
/// ascending grid subcarrier): the REs of the allocated CRBs (crb_mask, one byte per grid CRB) in symbols
/// [start_symbol, start_symbol + nof_symbols), minus the DM-RS RE pattern of the CDM groups without data over the
/// CRBs [dmrs_crb_begin, dmrs_crb_end) on DM-RS symbols (dmrs_mapping.h get_dmrs_pattern) and minus the reserved
/// patterns. Fills sc[] with each RE's grid subcarrier and sym_cum[l] with the REs before symbol l (l = 0..15).
inline void enumerate_data_res(unsigned                 grid_nof_prb,
                               const uint8_t*           crb_mask,
                               unsigned                 start_symbol,
                               unsigned                 nof_symbols,
                               unsigned                 dmrs_symbol_mask,
                               unsigned                 dmrs_type,
                               unsigned                 nof_cdm_groups_without_data,
                               unsigned                 dmrs_crb_begin,
                               unsigned                 dmrs_crb_end,
                               const srsgpu_re_pattern* reserved,
                               unsigned                 nof_reserved,
                               std::vector<uint16_t>&   sc,
                               uint16_t*                sym_cum)
{
  unsigned dmrs_re = 0;  // DM-RS REs of a PRB: type 1 CDM group g on 2k + g, type 2 on 6k + 2g + {0, 1}
  for (unsigned k = 0; k < 12; ++k) {
    const unsigned group = (dmrs_type == 2) ? (k % 6) / 2 : k % 2;
    if (group < nof_cdm_groups_without_data) {
      dmrs_re |= 1u << k;
    }
  }
  sc.clear();
  for (unsigned l = 0; l < 16; ++l) {
    if (l < 14) {
      sym_cum[l] = static_cast<uint16_t>(sc.size());
    }
    if (l >= 14 || l < start_symbol || l >= start_symbol + nof_symbols) {
      if (l >= 14) {
        sym_cum[l] = static_cast<uint16_t>(sc.size());
      }
      continue;
    }
    const bool dmrs_sym = ((dmrs_symbol_mask >> l) & 1u) != 0;
    for (unsigned crb = 0; crb < grid_nof_prb; ++crb) {
      if (crb_mask[crb] == 0) {
        continue;
      }
      unsigned excl = (dmrs_sym && crb >= dmrs_crb_begin && crb < dmrs_crb_end) ? dmrs_re : 0u;
      for (unsigned i = 0; i < nof_reserved; ++i) {
        const srsgpu_re_pattern& r = reserved[i];
        if (((r.symbol_mask >> l) & 1u) != 0 && (r.crb_mask == nullptr || r.crb_mask[crb] != 0)) {
          excl |= r.re_mask & 0xfffu;
        }
      }
      for (unsigned k = 0; k < 12; ++k) {
        if (((excl >> k) & 1u) == 0) {
          sc.push_back(static_cast<uint16_t>(crb * 12 + k));
        }
      }
    }
  }
}

} // namespace srsgpu
