// Host side of the srsgpu C ABI (include/srsgpu_phy.h): contexts, validation mirroring the reference's assertions,
// CRC early-stop tables and work-descriptor plans. No compute happens on the host: every codeblock is processed by the
// HIP kernels; a missing/unsupported device makes every call fail loudly (there is no CPU fallback).
#include "srsgpu_phy.h"
#include "ldpc_base_graphs.h"
#include "sch_host.h"
#include "srsgpu_internal.h"
#include "capi_internal.h"
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <tuple>
#include <map>
#include <mutex>
#include <string>
#include <vector>

using namespace srsgpu;

namespace srsgpu {
thread_local std::string g_last_error = "";
void set_last_error(const char* msg)
{
  g_last_error = msg;
}
} // namespace srsgpu

namespace {

int lifting_position(int Z)
{
  for (int i = 0; i < 51; ++i) {
    if (kLiftingSizes[i] == Z) {
      return i;
    }
  }
  return -1;
}

bool crc_params(int poly, unsigned& order, uint64_t& g)
{
  // channel_coding/crc_calculator_generic_impl.cpp:30
  switch (poly) {
    case SRSGPU_CRC24A: order = 24; g = 0x1864cfb; return true;
    case SRSGPU_CRC24B: order = 24; g = 0x1800063; return true;
    case SRSGPU_CRC24C: order = 24; g = 0x1b2b117; return true;
    case SRSGPU_CRC16: order = 16; g = 0x11021; return true;
    case SRSGPU_CRC11: order = 11; g = 0xe21; return true;
    case SRSGPU_CRC6: order = 6; g = 0x61; return true;
    default: return false;
  }
}


} // namespace

struct srsgpu_pusch_cb_plan {
  std::vector<crc_key>      crc_refs;  ///< CRC tables referenced (top-level plans only).
  srsgpu_context*           ctx     = nullptr;
  int                       impl    = SRSGPU_LDPC_IMPL_SIMD;
  dm_desc*                  d_dm    = nullptr;
  int                       nof_cbs = 0;
  srsgpu_ldpc_decoder_plan* dec     = nullptr;
};

struct srsgpu_pdsch_encoder_plan {
  std::vector<crc_key> crc_refs;  ///< CRC tables referenced.
  mutable stage_timer timer;
  srsgpu_context* ctx        = nullptr;
  tb_crc_desc*    d_tb       = nullptr;
  uint32_t*       d_tb_crc   = nullptr;
  tb_crc_slice*   d_slices   = nullptr;  ///< tb_crc_kernel work (TBs split into TB_CRC_SLICE_BYTES ranges).
  int             nof_slices = 0;
  int             nof_tbs    = 0;
  enc_desc*       d_enc[2]   = {nullptr, nullptr};  ///< Per base graph: byte-kernel codeblocks, then packed ones.
  int             count[2]   = {0, 0};
  int             count_pk[2] = {0, 0};
  bool            inline_tb_crc = false;  ///< Every codeblock packed, every TB CRC table cached, every TB at most
                                          ///< TB_CRC_INLINE_MAX_BYTES: no tb_crc_kernel.
  int             threads[2] = {64, 64};
  size_t          out_begin  = 0;
  size_t          out_end    = 0;
  /// The encoders OR a codeblock's partial edge words into the output, so [out_begin, out_end) is zeroed first, unless
  /// every codeblock covers whole 32-bit words and the TB codewords tile the range without gaps: then every word is
  /// stored exactly once (no memset node in the DL graph). SRSGPU_ENCODER_ZERO=1 keeps the memset (A/B).
  bool            zero_output = true;
};

struct srsgpu_pusch_decoder_plan {
  std::vector<crc_key>  crc_refs;   ///< CRC tables referenced.
  mutable stage_timer   timer;      ///< Three stages (enable_timing 1).
  mutable stage_timer   timer_dec;  ///< The decoding stage only (enable_timing 2): two events per execute.
  srsgpu_context*       ctx     = nullptr;
  srsgpu_pusch_cb_plan* cbs     = nullptr;
  tb_dec_desc*          d_tb    = nullptr;
  int                   nof_tbs = 0;
  int                   tb_threads = 256;  ///< pusch_tb_kernel workgroup size (1024 for large TBs).
  tb_slice*             d_slices   = nullptr;  ///< Sliced TB stage (large segmented TBs): pusch_tb_slice_kernel.
  uint32_t*             d_tb_acc   = nullptr;  ///< Per-TB CRC sums and slice counters (zero between executes).
  int                   nof_slices = 0;
};

struct srsgpu_ldpc_decoder_plan {
  std::vector<crc_key> crc_refs;  ///< CRC tables referenced (top-level plans only).
  /// One kernel launch per (base graph, kernel, layer bound): even lifting sizes go to the packed two-rows-per-lane
  /// kernel (64 * ceil(Z / 128) lanes) built for at most max_layers layers, odd ones to the one-row-per-lane kernel
  /// (64 * ceil(Z / 64) lanes).
  struct group {
    int       bg      = 1;
    bool      packed  = false;
    int       max_layers = 0;
    int       split   = 1;   ///< 2: edge-split kernel (each row's edges over two wave halves), see upload_decoder_plan
    int       pack    = 1;   ///< 2: two-codeblock workgroups (count = workgroups), see pair_layout_for
    int       threads = 64;
    int       count   = 0;
    dec_desc* d_desc  = nullptr;
    dm_desc*  d_dm    = nullptr;  ///< Fused rate dematching (DEC_FLAG_FUSED_DM): one dm_desc per codeblock, in order.
  };
  srsgpu_context*    ctx  = nullptr;
  int                impl = SRSGPU_LDPC_IMPL_SIMD;
  std::vector<group> groups;
  uint64_t           input_llrs = 0;  ///< LLR bytes the decoder moves per execute: dec_desc::nof_llr per codeblock,
                                      ///< E + N for fused ones (codeword LLRs read, HARQ buffer written).
};

namespace {

/// Returns an arena block to the free list, merged with its free neighbours.
void crc_free_block(srsgpu_context* ctx, size_t off, size_t len)
{
  auto next = ctx->crc_free.lower_bound(off);
  if (next != ctx->crc_free.end() && next->first == off + len) {
    len += next->second;
    next = ctx->crc_free.erase(next);
  }
  if (next != ctx->crc_free.begin()) {
    auto prev = std::prev(next);
    if (prev->first + prev->second == off) {
      off = prev->first;
      len += prev->second;
      ctx->crc_free.erase(prev);
    }
  }
  ctx->crc_free.emplace(off, len);
}

/// First-fit allocation of `words` arena words; evicts unreferenced cached tables (least recently used first) when
/// nothing fits and `evict` is set. Returns false when the arena cannot hold them (or, for optional tables, when
/// placing them would leave less than `keep_free` words).
bool crc_alloc(srsgpu_context* ctx, size_t words, size_t keep_free, bool evict, size_t& offset)
{
  auto free_words = [ctx]() {
    size_t n = 0;
    for (const auto& b : ctx->crc_free) {
      n += b.second;
    }
    return n;
  };
  for (;;) {
    if (free_words() >= words + keep_free) {
      for (auto it = ctx->crc_free.begin(); it != ctx->crc_free.end(); ++it) {
        if (it->second >= words) {
          offset                = it->first;
          const size_t rest     = it->second - words;
          ctx->crc_free.erase(it);
          if (rest > 0) {
            ctx->crc_free.emplace(offset + words, rest);
          }
          return true;
        }
      }
    }
    if (!evict) {
      return false;
    }
    auto victim = ctx->crc_tables.end();
    for (auto it = ctx->crc_tables.begin(); it != ctx->crc_tables.end(); ++it) {
      if (it->second.refs == 0 && (victim == ctx->crc_tables.end() || it->second.last_use < victim->second.last_use)) {
        victim = it;
      }
    }
    if (victim == ctx->crc_tables.end()) {
      return false;
    }
    const size_t off = victim->second.offset, len = victim->second.words;
    ctx->crc_tables.erase(victim);
    crc_free_block(ctx, off, len);
  }
}

/// Contribution table of every message bit to the CRC remainder: P[i] = x^(order + L - 1 - i) mod g(x), so that
/// CRC(m) = XOR of P[i] over the set bits m_i (the calculate() of crc_calculator_generic_impl.cpp:136 is linear),
/// followed by `tail` zero entries (the packed decoders read entry i for every systematic position i < K Z of a
/// codeblock without clamping to its message length K Z - fillers: tail = fillers).
/// The caller's plan takes a reference (refs) released with the plan. Optional tables (fast paths with a fallback)
/// never evict and leave CRC_ARENA_RESERVE words for required ones, so a long-running cell with link adaptation keeps
/// finding room for its codeblock tables (unreferenced tables are evicted for them).
int get_crc_table(srsgpu_context* ctx, int poly, int L, uint32_t& offset, std::vector<crc_key>& refs,
                  bool optional = false, int tail = 0)
{
  const crc_key key(poly, L, tail);
  auto          it = ctx->crc_tables.find(key);
  if (it != ctx->crc_tables.end()) {
    ++it->second.refs;
    it->second.last_use = ++ctx->crc_clock;
    refs.push_back(key);
    offset = static_cast<uint32_t>(it->second.offset);
    return SRSGPU_OK;
  }
  unsigned order;
  uint64_t g;
  if (!crc_params(poly, order, g)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid CRC polynomial %d", poly);
  }
  // Tables start 16-byte aligned and are padded to whole 16-byte vectors (the decoder copies them with 16-B loads):
  // every block is a multiple of 4 words, so every offset is too.
  const size_t words = (static_cast<size_t>(L) + static_cast<size_t>(tail) + 3u) & ~static_cast<size_t>(3u);
  size_t       off   = 0;
  if (!crc_alloc(ctx, words, optional ? CRC_ARENA_RESERVE : 0, !optional, off)) {
    return optional ? SRSGPU_ERR_NO_MEMORY : fail(SRSGPU_ERR_NO_MEMORY, "CRC table arena exhausted");
  }
  std::vector<uint32_t> tab(words, 0u);
  const uint64_t        high = 1ULL << order;
  uint64_t              r    = 1;
  for (unsigned k = 0; k < order; ++k) {
    r <<= 1;
    if (r & high) {
      r ^= g;
    }
  }
  for (int i = L - 1; i >= 0; --i) {
    tab[static_cast<size_t>(i)] = static_cast<uint32_t>(r);
    r <<= 1;
    if (r & high) {
      r ^= g;
    }
  }
  if (hipMemcpy(ctx->d_crc_arena + off, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice) !=
      hipSuccess) {
    crc_free_block(ctx, off, words);
    return fail(SRSGPU_ERR_HIP, "CRC table upload failed");
  }
  crc_entry e;
  e.offset   = off;
  e.words    = words;
  e.refs     = 1;
  e.last_use = ++ctx->crc_clock;
  ctx->crc_tables.emplace(key, e);
  refs.push_back(key);
  offset = static_cast<uint32_t>(off);
  return SRSGPU_OK;
}

/// Contribution table for an optional fast path: its arena offset, or NO_CRC_TABLE (no error) when it would eat into
/// the reserve kept for required tables.
uint32_t try_crc_table(srsgpu_context* ctx, int poly, int L, std::vector<crc_key>& refs)
{
  uint32_t off = NO_CRC_TABLE;
  return get_crc_table(ctx, poly, L, off, refs, true) == SRSGPU_OK ? off : NO_CRC_TABLE;
}

/// Solves the core of the lifted base graph (rows 0..3 x parity columns K..K+3) once per (BG, Z), like
/// ldpc_encoder_generic.cpp:226-:328 special-cases it per lifting set: P^x p0 = sum of the core syndromes, then every
/// row with a single unknown parity node yields it.
bool build_core_plan(int bg, int Z, core_plan& cp)
{
  const int             K   = (bg == 1) ? kBG1_K : kBG2_K;
  const uint16_t*       rs  = (bg == 1) ? kBG1_ROW_START : kBG2_ROW_START;
  const uint8_t*        col = (bg == 1) ? kBG1_COL : kBG2_COL;
  const int             ils = kLiftingSetIndex[Z];
  const uint16_t*       V   = (bg == 1) ? kBG1_V[ils] : kBG2_V[ils];
  int                   sh[4][4];
  for (int m = 0; m < 4; ++m) {
    for (int j = 0; j < 4; ++j) {
      sh[m][j] = -1;
    }
    for (int e = rs[m]; e < rs[m + 1]; ++e) {
      if (col[e] >= K && col[e] < K + 4) {
        sh[m][col[e] - K] = V[e] % Z;
      }
    }
  }
  std::vector<int> cnt(static_cast<size_t>(Z), 0);
  for (int m = 0; m < 4; ++m) {
    if (sh[m][0] >= 0) {
      cnt[static_cast<size_t>(sh[m][0])] ^= 1;
    }
  }
  int x = -1, nsurv = 0;
  for (int s = 0; s < Z; ++s) {
    if (cnt[static_cast<size_t>(s)]) {
      x = s;
      ++nsurv;
    }
  }
  if (nsurv != 1) {
    return false;
  }
  cp.x       = static_cast<int16_t>(x);
  cp.o0      = static_cast<int16_t>((Z - x) % Z);
  bool known[4] = {true, false, false, false};
  int  step     = 0;
  for (int round = 0; round < 4 && step < 3; ++round) {
    for (int m = 0; m < 4 && step < 3; ++m) {
      int u = -1, nunk = 0;
      for (int j = 0; j < 4; ++j) {
        if (sh[m][j] >= 0 && !known[j]) {
          u = j;
          ++nunk;
        }
      }
      if (nunk != 1) {
        continue;
      }
      cp.unk[step] = static_cast<int8_t>(u);
      cp.row[step] = static_cast<int8_t>(m);
      const int su  = sh[m][u];
      cp.orow[step] = static_cast<int16_t>((Z - su) % Z);
      for (int j = 0; j < 4; ++j) {
        cp.sh[step][j] = static_cast<int16_t>(sh[m][j]);
        cp.oj[step][j] = static_cast<int16_t>((j != u && sh[m][j] >= 0) ? (sh[m][j] - su + Z) % Z : -1);
      }
      known[u] = true;
      ++step;
    }
  }
  return step == 3;
}

} // namespace

extern "C" {

int srsgpu_version(void)
{
  return 100;
}

const char* srsgpu_last_error(void)
{
  return g_last_error.c_str();
}

int srsgpu_context_create(int device, srsgpu_context** out)
{
  if (out == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null output pointer");
  }
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    return fail(SRSGPU_ERR_INVALID_ARG, "device %d not present (%d HIP devices)", device, ndev);
  }
  HIP_TRY(hipSetDevice(device));
  auto* ctx   = new srsgpu_context();
  ctx->device = device;
  // Lifted shift tables: shifts[bg][position of Z][edge] = V(i_LS(Z), edge) mod Z (ldpc_luts_impl.cpp:4522).
  for (int bg = 1; bg <= 2; ++bg) {
    const int             ne = (bg == 1) ? kBG1_NUM_EDGES : kBG2_NUM_EDGES;
    std::vector<uint16_t> tab(static_cast<size_t>(51) * ne);
    for (int p = 0; p < 51; ++p) {
      const int Z   = kLiftingSizes[p];
      const int ils = kLiftingSetIndex[Z];
      for (int e = 0; e < ne; ++e) {
        const int v = (bg == 1) ? kBG1_V[ils][e] : kBG2_V[ils][e];
        tab[static_cast<size_t>(p) * ne + e] = static_cast<uint16_t>(v % Z);
      }
    }
    // The decoder reads its shifts through scalar loads, which are dword-granular: it gets a 32-bit copy.
    std::vector<uint32_t> tab32(tab.begin(), tab.end());
    // Packed decoder: rows z and z + H of a lane read the pair at min(2z + A, 2z + B) (row z) and its partner byte.
    // Two-codeblock workgroups (ldpc_decoder_pk.hip): pairs are 4 bytes apart in the interleaved image, the lane
    // constant is 4 z + 2 slot: A = 4 s' + hi, B = 4 (s' - H) + 1 - hi.
    std::vector<uint32_t> ab(static_cast<size_t>(51) * ne, 0u), ab2(static_cast<size_t>(51) * ne, 0u);
    for (int p = 0; p < 51; ++p) {
      const int Z = kLiftingSizes[p];
      if (Z % 2 != 0) {
        continue;
      }
      const int H = Z / 2;
      for (int e = 0; e < ne; ++e) {
        const int sft = tab[static_cast<size_t>(p) * ne + e];
        const int hi  = sft >= H ? 1 : 0;
        const int sm  = sft - hi * H;
        const int A   = 2 * sm + hi;
        const int B   = 2 * sm - 2 * H + 1 - hi;
        // One dword per edge: A in the low half, B (negative: wraps) in the high half.
        ab[static_cast<size_t>(p) * ne + e] = static_cast<uint32_t>(A) | (static_cast<uint32_t>(B & 0xffff) << 16);
        const int A2 = 4 * sm + hi;  // two-codeblock workgroups (PKN = 2)
        const int B2 = 4 * (sm - H) + 1 - hi;
        ab2[static_cast<size_t>(p) * ne + e] =
            static_cast<uint32_t>(A2) | (static_cast<uint32_t>(B2 & 0xffff) << 16);
      }
    }
    if (hipMalloc(&ctx->d_pair_ab[bg - 1], ab.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMemcpy(ctx->d_pair_ab[bg - 1], ab.data(), ab.size() * sizeof(uint32_t), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMalloc(&ctx->d_pair_ab2[bg - 1], ab2.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMemcpy(ctx->d_pair_ab2[bg - 1], ab2.data(), ab2.size() * sizeof(uint32_t), hipMemcpyHostToDevice) !=
            hipSuccess) {
      srsgpu_context_destroy(ctx);
      return fail(SRSGPU_ERR_HIP, "failed to upload LDPC pair address tables");
    }
    if (hipMalloc(&ctx->d_shifts[bg - 1], tab.size() * sizeof(uint16_t)) != hipSuccess ||
        hipMemcpy(ctx->d_shifts[bg - 1], tab.data(), tab.size() * sizeof(uint16_t), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMalloc(&ctx->d_shifts32[bg - 1], tab32.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMemcpy(ctx->d_shifts32[bg - 1], tab32.data(), tab32.size() * sizeof(uint32_t), hipMemcpyHostToDevice) !=
            hipSuccess) {
      srsgpu_context_destroy(ctx);
      return fail(SRSGPU_ERR_HIP, "failed to upload LDPC shift tables");
    }
  }
  for (int bg = 1; bg <= 2; ++bg) {
    ctx->core[bg - 1].resize(51);
    for (int p = 0; p < 51; ++p) {
      if (!build_core_plan(bg, kLiftingSizes[p], ctx->core[bg - 1][static_cast<size_t>(p)])) {
        srsgpu_context_destroy(ctx);
        return fail(SRSGPU_ERR_INVALID_ARG, "cannot solve the LDPC core of BG%d Z=%d", bg, kLiftingSizes[p]);
      }
    }
    if (hipMalloc(&ctx->d_core[bg - 1], 51 * sizeof(core_plan)) != hipSuccess ||
        hipMemcpy(ctx->d_core[bg - 1], ctx->core[bg - 1].data(), 51 * sizeof(core_plan), hipMemcpyHostToDevice) !=
            hipSuccess) {
      srsgpu_context_destroy(ctx);
      return fail(SRSGPU_ERR_HIP, "failed to upload the LDPC core plans");
    }
  }
  if (hipMalloc(&ctx->d_crc_arena, CRC_ARENA_WORDS * sizeof(uint32_t)) != hipSuccess) {
    srsgpu_context_destroy(ctx);
    return fail(SRSGPU_ERR_NO_MEMORY, "failed to allocate the CRC table arena");
  }
  {
    // Slice-by-4 byte tables of the TB / CB CRCs: T_0[v] = v x^order mod g (the byte table), T_k = T_(k-1) advanced
    // by one zero byte.
    const uint32_t      polys[3]  = {0x1864cfbu, 0x1800063u, 0x11021u};
    const int           orders[3] = {24, 24, 16};
    std::vector<uint32_t> tabs(3 * CRC_SLICE_WORDS);
    for (int c = 0; c < 3; ++c) {
      const uint32_t mask = (1u << orders[c]) - 1u;
      uint32_t*      t    = tabs.data() + c * CRC_SLICE_WORDS;
      for (uint32_t v = 0; v < 256; ++v) {
        uint32_t r = v << (orders[c] - 8);
        for (int k = 0; k < 8; ++k) {
          r <<= 1;
          if (r & (1u << orders[c])) {
            r ^= polys[c];
          }
        }
        t[v] = r & mask;
      }
      for (int k = 1; k < 4; ++k) {
        for (uint32_t v = 0; v < 256; ++v) {
          const uint32_t p = t[(k - 1) * 256 + v];
          t[k * 256 + v]   = ((p << 8) ^ t[(p >> (orders[c] - 8)) & 0xffu]) & mask;
        }
      }
    }
    if (hipMalloc(&ctx->d_crc_slice, tabs.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMemcpy(ctx->d_crc_slice, tabs.data(), tabs.size() * sizeof(uint32_t), hipMemcpyHostToDevice) !=
            hipSuccess) {
      srsgpu_context_destroy(ctx);
      return fail(SRSGPU_ERR_HIP, "failed to upload the slice-by-4 CRC tables");
    }
  }
  *out = ctx;
  return SRSGPU_OK;
}

int srsgpu_context_device(const srsgpu_context* ctx)
{
  return ctx == nullptr ? -1 : ctx->device;
}

namespace {

int* context_option(srsgpu_context* ctx, int option)
{
  switch (option) {
    case SRSGPU_OPTION_DECODER_SPLIT:
      return &ctx->opt_decoder_split;
    case SRSGPU_OPTION_DECODER_PAIRS:
      return &ctx->opt_decoder_pairs;
    case SRSGPU_OPTION_DECODER_FUSED_DEMATCH:
      return &ctx->opt_decoder_fused_dematch;
    case SRSGPU_OPTION_ENCODER_BYTE_KERNEL:
      return &ctx->opt_encoder_byte_kernel;
    case SRSGPU_OPTION_ENCODER_ZERO_OUTPUT:
      return &ctx->opt_encoder_zero_output;
    default:
      return nullptr;
  }
}

} // namespace

int srsgpu_context_set_option(srsgpu_context* ctx, int option, int value)
{
  if (ctx == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null context");
  }
  int* slot = context_option(ctx, option);
  if (slot == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "unknown option %d", option);
  }
  const int lo = option == SRSGPU_OPTION_DECODER_SPLIT ? -1 : 0;
  if (value < lo || value > 1) {
    return fail(SRSGPU_ERR_INVALID_ARG, "option %d: invalid value %d", option, value);
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  *slot = value;
  return SRSGPU_OK;
}

int srsgpu_context_get_option(const srsgpu_context* ctx, int option, int* value)
{
  if (ctx == nullptr || value == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  const int* slot = context_option(const_cast<srsgpu_context*>(ctx), option);
  if (slot == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "unknown option %d", option);
  }
  *value = *slot;
  return SRSGPU_OK;
}

void srsgpu_context_destroy(srsgpu_context* ctx)
{
  if (ctx == nullptr) {
    return;
  }
  (void)hipSetDevice(ctx->device);
  for (auto* p : ctx->d_shifts) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  for (auto* p : ctx->d_shifts32) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  for (auto* p : ctx->d_pair_ab2) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  for (auto* p : ctx->d_pair_ab) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  for (auto* p : ctx->d_core) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  for (void* p : {static_cast<void*>(ctx->d_crc_arena), static_cast<void*>(ctx->d_crc_slice),
                  static_cast<void*>(ctx->d_gold_x1),
                  static_cast<void*>(ctx->d_gold_x2_jump), static_cast<void*>(ctx->d_gold_x2_lane),
                  static_cast<void*>(ctx->d_ofdm_twiddles)}) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  delete ctx;
}

} // extern "C"

namespace {

/// Codeblock work split by base graph: one launch per base graph, sized for its largest lifting size. (Splitting
/// further by block size raises the occupancy of the small-Z blocks but serialises launches; measured slower on the
/// 100 MHz slot: 0.82 vs 0.76 ms per 16 slots.)
using dec_key = std::tuple<int, bool, int, bool>;  ///< (base graph, packed kernel, layer bound class, fused dematch)
struct dec_batch {
  std::map<dec_key, std::vector<dec_desc>> groups;
  std::map<dec_key, std::vector<dm_desc>>  fused;  ///< Fused groups: the dm_desc of each codeblock, in group order.
  std::map<dec_key, int>                   threads;
  std::vector<crc_key>*                    crc_refs = nullptr;  ///< The creating call's crc_ref_guard.
};

/// Upper bound of the number of layers decode() uses for an input of nof_llrs LLRs (ldpc_decoder_impl.cpp:110: the
/// trimmed length can only be shorter), rounded up to a compiled class of the packed kernel (8, 16 or all rows).
int layer_class(int bg, int Z, uint32_t nof_llrs)
{
  const int K      = (bg == 1) ? kBG1_K : kBG2_K;
  const int M      = (bg == 1) ? kBG1_M : kBG2_M;
  int       cb_len = static_cast<int>(nof_llrs) + 2 * Z;
  cb_len           = std::max(cb_len, (K + 4) * Z);
  const int bound  = (cb_len + Z - 1) / Z - K;
  return bound <= 8 ? 8 : (bound <= 16 ? 16 : M);
}

/// Validates one decoder configuration (ldpc_decoder_impl.cpp:48-:56, :73-:88) and appends its descriptor.
int add_decoder_cb(srsgpu_context* ctx,
                   uint32_t        i,
                   int             bg,
                   int             Z,
                   int             nof_filler,
                   int             nof_crc_bits,
                   int             max_iter,
                   float           sf,
                   int             crc_poly,
                   bool            early_stop,
                   uint32_t        llr_offset,
                   uint32_t        nof_llrs,
                   uint32_t        out_offset,
                   dec_batch&      batch,
                   const dm_desc*  fused_dm = nullptr)
{
  if (bg != 1 && bg != 2) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid base graph %d", i, bg);
  }
  const int pos = lifting_position(Z);
  if (pos < 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid lifting size %d", i, Z);
  }
  const int K = (bg == 1) ? kBG1_K : kBG2_K;
  const int N = ((bg == 1) ? kBG1_N_FULL : kBG2_N_FULL) - 2;
  if (max_iter <= 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: max iterations must be different to 0", i);
  }
  if (!(sf > 0.0f && sf < 1.0f)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: scaling factor must be between 0 and 1 exclusively", i);
  }
  if (nof_crc_bits != 16 && nof_crc_bits != 24) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid number of CRC bits %d", i, nof_crc_bits);
  }
  if (static_cast<int>(nof_llrs) > N * Z || static_cast<int>(nof_llrs) < (K + 2) * Z) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: input length %u outside [%d, %d]", i, nof_llrs, (K + 2) * Z, N * Z);
  }
  if (nof_filler < 0 || nof_filler >= (K - 2) * Z) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid number of filler bits %d", i, nof_filler);
  }
  dec_desc d{};
  d.llr_offset      = llr_offset;
  d.nof_llr         = nof_llrs;
  d.out_offset      = out_offset;
  d.crc_table       = NO_CRC_TABLE;
  d.div_magic       = static_cast<uint32_t>(((1ULL << 32) + static_cast<uint64_t>(Z) - 1) / static_cast<uint64_t>(Z));
  d.Z               = static_cast<uint16_t>(Z);
  d.zpos            = static_cast<uint16_t>(pos);
  d.nof_significant = static_cast<uint16_t>(K * Z - nof_filler);
  d.max_iter        = static_cast<uint16_t>(max_iter);
  // avx2_support.h:71: identity above .9999, otherwise floor(sf * 2^16) in float arithmetic.
  d.sf16     = (static_cast<double>(sf) >= .9999) ? 65536u
                                                   : static_cast<uint32_t>(static_cast<uint16_t>(sf * 65536U));
  d.sf       = sf;
  d.cb_index = i;
  d.flags    = 0;
  if (crc_poly != SRSGPU_CRC_NONE) {
    int r = get_crc_table(ctx, crc_poly, K * Z - nof_filler, d.crc_table, *batch.crc_refs, false, nof_filler);
    if (r != SRSGPU_OK) {
      return r;
    }
    d.flags = early_stop ? DEC_FLAG_EARLY_STOP : 0u;
  }
  const bool    packed = (Z % 2) == 0;
  const bool    fuse   = fused_dm != nullptr && packed;
  const dec_key key(bg, packed, packed ? layer_class(bg, Z, nof_llrs) : 0, fuse);
  if (fuse) {
    d.flags |= DEC_FLAG_FUSED_DM;
    batch.fused[key].push_back(*fused_dm);
  }
  batch.groups[key].push_back(d);
  const int lanes = packed ? Z / 2 : Z;
  int&      t     = batch.threads[key];
  t               = std::max(t, ((lanes + 63) / 64) * 64);
  return SRSGPU_OK;
}

/// Two-codeblock workgroups (ldpc_decode_pairs_kernel): a codeblock of H = Z / 2 in (64, 96] (Z = 144 ..
/// 192) spans two waves of which the second is partly idle, while two of them fill three waves (Z = 192: 25 % fewer
/// wave-instructions). Moves such codeblocks of `cbs` (and their dm_desc, when fused) into `pairs` / `pair_dms`, two
/// slots per workgroup (codeblocks sharing Z, scaling, iteration limit and CRC mode; an odd one out leaves its second
/// slot empty), keeping the others. Opt-in (SRSGPU_OPTION_DECODER_PAIRS): measured at Z = 192 (8-layer span,
/// tools/decoder_scaling.py, profiles/r5_decoder_pk2_scaling.txt) 2-7 % faster with all 6 iterations (8 192 codeblocks:
/// 676 -> 631 us), equal with early stop at 2 iterations, 8 % slower at 1 024 codeblocks: far from the 25 % fewer
/// waves (the wave shared by both codeblocks runs until the later one stops; 8-byte pair interleave).
void pair_layout_for(const srsgpu_context* ctx, std::vector<dec_desc>& cbs, std::vector<dm_desc>& dms, bool fused,
                     std::vector<dec_desc>& pairs, std::vector<dm_desc>& pair_dms)
{
  if (ctx->opt_decoder_pairs == 0) {
    return;
  }
  std::vector<size_t> idx, rest;
  for (size_t i = 0; i < cbs.size(); ++i) {
    const int H = cbs[i].Z / 2;
    ((H > 64 && H <= 96) ? idx : rest).push_back(i);
  }
  if (idx.empty()) {
    return;
  }
  auto key = [&](size_t i) {
    const dec_desc& d = cbs[i];
    return std::make_tuple(d.Z, d.sf16, d.max_iter, static_cast<uint32_t>(d.flags), d.crc_table == NO_CRC_TABLE);
  };
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return key(a) < key(b); });
  for (size_t k = 0; k < idx.size();) {
    const bool two = k + 1 < idx.size() && key(idx[k + 1]) == key(idx[k]) && cbs[idx[k + 1]].sf == cbs[idx[k]].sf;
    pairs.push_back(cbs[idx[k]]);
    pairs.push_back(two ? cbs[idx[k + 1]] : dec_desc{});
    if (fused) {
      pair_dms.push_back(dms[idx[k]]);
      pair_dms.push_back(two ? dms[idx[k + 1]] : dm_desc{});
    }
    k += two ? 2 : 1;
  }
  std::vector<dec_desc> keep;
  std::vector<dm_desc>  keep_dms;
  for (size_t i : rest) {
    keep.push_back(cbs[i]);
    if (fused) {
      keep_dms.push_back(dms[i]);
    }
  }
  cbs.swap(keep);
  dms.swap(keep_dms);
}

int upload_decoder_plan(srsgpu_context* ctx, int impl, const dec_batch& batch, srsgpu_ldpc_decoder_plan** plan_out)
{
  auto* plan = new srsgpu_ldpc_decoder_plan();
  plan->ctx  = ctx;
  plan->impl = impl;
  auto upload = [&](void** dst, const void* src, size_t bytes) {
    return hipMalloc(dst, bytes) == hipSuccess && hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  for (const auto& kv : batch.groups) {
    const bool            fused = std::get<3>(kv.first);
    std::vector<dec_desc> cbs   = kv.second;
    std::vector<dm_desc>  dms   = fused ? batch.fused.at(kv.first) : std::vector<dm_desc>{};
    if (std::get<1>(kv.first) && std::get<2>(kv.first) <= 16) {
      std::vector<dec_desc> pairs;
      std::vector<dm_desc>  pair_dms;
      pair_layout_for(ctx, cbs, dms, fused, pairs, pair_dms);
      if (!pairs.empty()) {
        srsgpu_ldpc_decoder_plan::group gp;
        gp.bg         = std::get<0>(kv.first);
        gp.packed     = true;
        gp.max_layers = std::get<2>(kv.first);
        gp.pack       = 2;
        gp.threads    = 192;
        gp.count      = static_cast<int>(pairs.size() / 2);
        for (size_t k = 0; k < pairs.size(); ++k) {
          if (pairs[k].nof_llr != 0u) {
            plan->input_llrs += fused ? static_cast<uint64_t>(pair_dms[k].E) + pair_dms[k].N : pairs[k].nof_llr;
          }
        }
        const bool ok = upload(reinterpret_cast<void**>(&gp.d_desc), pairs.data(), pairs.size() * sizeof(dec_desc)) &&
                        (!fused || upload(reinterpret_cast<void**>(&gp.d_dm), pair_dms.data(),
                                          pair_dms.size() * sizeof(dm_desc)));
        plan->groups.push_back(gp);
        if (!ok) {
          srsgpu_ldpc_decoder_plan_destroy(plan);
          return fail(SRSGPU_ERR_HIP, "failed to upload decoder descriptors");
        }
      }
    }
    if (cbs.empty()) {
      continue;
    }
    srsgpu_ldpc_decoder_plan::group g;
    g.bg               = std::get<0>(kv.first);
    g.packed           = std::get<1>(kv.first);
    g.max_layers       = std::get<2>(kv.first);
    g.threads          = batch.threads.at(kv.first);
    g.count            = static_cast<int>(cbs.size());
    // Few codeblocks per launch leave the SIMDs with one or two waves each: the per-codeblock latency (instructions
    // per wave) then sets the kernel time, and the edge-split kernel halves it at ~15 % more total work. Above ~3
    // waves per SIMD of the plain kernel (MI355X: 1024 SIMDs) the launch is throughput-bound and keeps the plain one.
    // SRSGPU_OPTION_DECODER_SPLIT forces either (parity tests).
    if (g.packed) {
      const long waves  = static_cast<long>(g.count) * (g.threads / 64);
      const bool split2 = ctx->opt_decoder_split >= 0 ? (ctx->opt_decoder_split == 1) : (waves < 3L * 1024L);
      if (split2) {
        g.split = 2;
        g.threads *= 2;
      }
    }
    if (!fused) {
      for (const dec_desc& d : cbs) {
        plan->input_llrs += d.nof_llr;
      }
    } else {
      // A fused codeblock reads its E codeword LLRs and writes the N-byte HARQ buffer instead.
      for (const dm_desc& m : dms) {
        plan->input_llrs += static_cast<uint64_t>(m.E) + m.N;
      }
      const size_t dm_bytes = dms.size() * sizeof(dm_desc);
      if (hipMalloc(&g.d_dm, dm_bytes) != hipSuccess ||
          hipMemcpy(g.d_dm, dms.data(), dm_bytes, hipMemcpyHostToDevice) != hipSuccess) {
        plan->groups.push_back(g);
        srsgpu_ldpc_decoder_plan_destroy(plan);
        return fail(SRSGPU_ERR_HIP, "failed to upload fused rate dematcher descriptors");
      }
    }
    const dec_desc* src   = cbs.data();
    const size_t    bytes = cbs.size() * sizeof(dec_desc);
    if (hipMalloc(&g.d_desc, bytes) != hipSuccess ||
        hipMemcpy(g.d_desc, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
      plan->groups.push_back(g);
      srsgpu_ldpc_decoder_plan_destroy(plan);
      return fail(SRSGPU_ERR_HIP, "failed to upload decoder descriptors");
    }
    plan->groups.push_back(g);
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

/// d_cw_llrs / d_harq: the codeword LLRs and the HARQ buffer of the fused groups (PUSCH plans; null otherwise).
/// d_harq_cbs (PUSCH plans, optional): codeblock c's HARQ soft buffer is d_harq_cbs[c] (then d_llrs / d_harq unused).
int execute_decoder_plan(const srsgpu_ldpc_decoder_plan* plan,
                         const int8_t*                   d_llrs,
                         uint8_t*                        d_out,
                         int32_t*                        d_nof_iterations,
                         uint8_t*                        d_cb_crc_ok,
                         hipStream_t                     s,
                         const int8_t*                   d_cw_llrs  = nullptr,
                         int8_t*                         d_harq     = nullptr,
                         int8_t* const*                  d_harq_cbs = nullptr)
{
  for (const auto& g : plan->groups) {
    if (g.pack == 2) {
      if (g.d_dm != nullptr && (d_cw_llrs == nullptr || (d_harq == nullptr && d_harq_cbs == nullptr))) {
        return fail(SRSGPU_ERR_INVALID_ARG, "fused decoder group without codeword LLRs / HARQ buffer");
      }
      launch_ldpc_decode_pairs(g.bg, plan->impl, g.max_layers, g.d_desc, g.count, g.threads,
                               g.d_dm != nullptr ? d_cw_llrs : d_llrs, d_out, d_nof_iterations,
                               plan->ctx->d_pair_ab2[g.bg - 1], plan->ctx->d_crc_arena, d_cb_crc_ok, s, d_harq_cbs,
                               g.d_dm, g.d_dm != nullptr ? d_harq : nullptr);
    } else if (g.packed) {
      if (g.d_dm != nullptr && (d_cw_llrs == nullptr || (d_harq == nullptr && d_harq_cbs == nullptr))) {
        return fail(SRSGPU_ERR_INVALID_ARG, "fused decoder group without codeword LLRs / HARQ buffer");
      }
      launch_ldpc_decode_pk(g.bg, plan->impl, g.max_layers, g.split, g.d_desc, g.count, g.threads,
                            g.d_dm != nullptr ? d_cw_llrs : d_llrs, d_out, d_nof_iterations,
                            plan->ctx->d_pair_ab[g.bg - 1], plan->ctx->d_crc_arena, d_cb_crc_ok, g.d_dm,
                            g.d_dm != nullptr ? d_harq : nullptr, s, d_harq_cbs);
    } else {
      launch_ldpc_decode(g.bg, plan->impl, g.d_desc, g.count, g.threads, d_llrs, d_out, d_nof_iterations,
                         plan->ctx->d_shifts32[g.bg - 1], plan->ctx->d_crc_arena, d_cb_crc_ok, s, d_harq_cbs);
    }
    HIP_TRY(hipGetLastError());
  }
  return SRSGPU_OK;
}

struct pusch_cb_params {
  int      bg, rv, qm, crc_poly, Z, filler, nof_crc_bits, max_iter;
  bool     new_data, early_stop;
  float    sf;
  uint32_t Nref, E, llr_offset, harq_offset, out_offset, cb_index;
};

/// Validates one PUSCH codeblock (ldpc_rate_dematcher_impl.cpp:54-:99 plus the decoder's checks) and appends its
/// dematcher and decoder descriptors.
int add_pusch_cb(srsgpu_context*        ctx,
                 uint32_t               i,
                 const pusch_cb_params& c,
                 dec_batch&             batch,
                 std::vector<dm_desc>&  dms)
{
  static const double shift_bg1[4] = {0, 17, 33, 56};  // ldpc_rate_dematcher_impl.cpp:33
  static const double shift_bg2[4] = {0, 13, 25, 43};
  const int           Z            = c.Z;
  if ((c.bg != 1 && c.bg != 2) || lifting_position(Z) < 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid base graph %d / lifting size %d", i, c.bg, Z);
  }
  const int K    = (c.bg == 1) ? kBG1_K : kBG2_K;
  const int N    = (((c.bg == 1) ? kBG1_N_FULL : kBG2_N_FULL) - 2) * Z;
  const int nsys = (K - 2) * Z;
  const int qm   = c.qm;
  if (c.rv < 0 || c.rv > 3) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: RV should an integer between 0 and 3", i);
  }
  if (qm != 1 && qm != 2 && qm != 4 && qm != 6 && qm != 8) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid modulation order %d", i, qm);
  }
  if (c.E == 0 || c.E % static_cast<uint32_t>(qm) != 0 || c.E > 22u * 384u * 35u) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid rate-matched length %u", i, c.E);
  }
  if (c.Nref > 66u * 384u) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: N_ref %u must be smaller or equal to %u", i, c.Nref, 66u * 384u);
  }
  if (c.filler < 0 || c.filler >= nsys) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid number of filler bits", i);
  }
  const int Ncb = (c.Nref > 0 && static_cast<int>(c.Nref) < N) ? static_cast<int>(c.Nref) : N;
  if (Ncb <= nsys) {
    return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: circular buffer %d shorter than the systematic part", i, Ncb);
  }
  const double sf    = (c.bg == 1 ? shift_bg1 : shift_bg2)[c.rv];
  const int    k0    = static_cast<int>(std::floor((sf * Ncb) / N)) * Z;
  const int    ninfo = nsys - c.filler;
  dm_desc      d{};
  d.llr_offset  = c.llr_offset;
  d.harq_offset = c.harq_offset;
  d.E           = c.E;
  d.N           = static_cast<uint32_t>(N);
  d.Ncb         = static_cast<uint32_t>(Ncb);
  d.nsys        = static_cast<uint32_t>(nsys);
  d.v0          = static_cast<uint32_t>(k0 < ninfo ? k0 : (k0 < nsys ? ninfo : k0 - c.filler));
  d.nof_filler  = static_cast<uint16_t>(c.filler);
  d.Qm          = static_cast<uint8_t>(qm);
  d.new_data    = c.new_data ? 1 : 0;
  d.cb_index    = c.cb_index;
  const uint64_t R = c.E / static_cast<uint32_t>(qm);
  d.r_magic        = ((1ULL << 40) + R - 1) / R;
  // A first transmission from rv 0 of the whole circular buffer that reaches every systematic position without
  // wrapping (ninfo <= E <= V) is a plain copy that defines every HARQ position (copies, fillers, zeroed tail): the
  // packed decoder dematches it itself (ldpc_decode_pk_kernel FUSE) and the rate dematcher skips it.
  // SRSGPU_OPTION_DECODER_FUSED_DEMATCH = 0 keeps every codeblock on the separate rate dematcher (parity tests).
  const bool fuse = ctx->opt_decoder_fused_dematch != 0 && c.new_data && d.v0 == 0 && Ncb == N && static_cast<int>(c.E) >= ninfo &&
                    static_cast<int>(c.E) <= Ncb - c.filler && (Z % 2) == 0;
  if (!fuse) {
    dms.push_back(d);
  }
  // The decoder reads the HARQ buffer up to the last position a new transmission can leave non-zero: the rate
  // dematcher zeroes everything from the end of an incomplete first pass (zero_from), and decode() trims trailing
  // zeros anyway (ldpc_decoder_impl.cpp:94), so the shorter span (whole lifted columns, hence the same soft clamp)
  // decodes identically - and lets the decoder run a kernel sized for fewer layers.
  uint32_t dec_llrs = static_cast<uint32_t>(N);
  if (c.new_data) {
    const int V = Ncb - c.filler;
    if (static_cast<int>(c.E) < V - static_cast<int>(d.v0)) {
      const int vend = static_cast<int>(d.v0) + static_cast<int>(c.E);
      int       kend = vend < ninfo ? vend : vend + c.filler;
      kend           = std::max(kend, nsys) % Ncb;
      if (kend != 0) {
        const int zero_from = N - (Ncb - kend);
        const int span      = std::max((K + 2) * Z, ((zero_from + Z - 1) / Z) * Z);
        dec_llrs            = static_cast<uint32_t>(std::min(N, span));
      }
    }
  }
  return add_decoder_cb(ctx, c.cb_index, c.bg, Z, c.filler, c.nof_crc_bits, c.max_iter, c.sf, c.crc_poly,
                        c.early_stop, c.harq_offset, dec_llrs, c.out_offset, batch, fuse ? &d : nullptr);
}

int upload_pusch_cb_plan(srsgpu_context*             ctx,
                         int                         impl,
                         const dec_batch&            batch,
                         const std::vector<dm_desc>& dms,
                         srsgpu_pusch_cb_plan**      plan_out)
{
  auto* plan    = new srsgpu_pusch_cb_plan();
  plan->ctx     = ctx;
  plan->impl    = impl;
  plan->nof_cbs = static_cast<int>(dms.size());
  int r         = upload_decoder_plan(ctx, impl, batch, &plan->dec);
  if (r != SRSGPU_OK) {
    delete plan;
    return r;
  }
  if (!dms.empty() && (hipMalloc(&plan->d_dm, dms.size() * sizeof(dm_desc)) != hipSuccess ||
                       hipMemcpy(plan->d_dm, dms.data(), dms.size() * sizeof(dm_desc), hipMemcpyHostToDevice) !=
                           hipSuccess)) {
    srsgpu_pusch_cb_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload rate dematcher descriptors");
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

int execute_pusch_cb_plan(const srsgpu_pusch_cb_plan* plan,
                          const int8_t*               d_llrs,
                          int8_t*                     d_harq,
                          uint8_t*                    d_out,
                          int32_t*                    d_nof_iterations,
                          uint8_t*                    d_cb_crc_ok,
                          hipStream_t                 s)
{
  launch_rate_dematch(plan->impl, plan->d_dm, plan->nof_cbs, d_llrs, d_harq, d_cb_crc_ok, s);
  HIP_TRY(hipGetLastError());
  return execute_decoder_plan(plan->dec, d_harq, d_out, d_nof_iterations, d_cb_crc_ok, s, d_llrs, d_harq);
}

} // namespace

extern "C" {

int srsgpu_ldpc_decoder_plan_create(srsgpu_context*                   ctx,
                                    int                               impl,
                                    const srsgpu_ldpc_decoder_config* cfgs,
                                    uint32_t                          nof_cbs,
                                    srsgpu_ldpc_decoder_plan**        plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_cbs > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (impl != SRSGPU_LDPC_IMPL_GENERIC && impl != SRSGPU_LDPC_IMPL_SIMD) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid decoder implementation %d", impl);
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  crc_ref_guard guard(ctx);
  dec_batch     batch;
  batch.crc_refs = &guard.refs;
  for (uint32_t i = 0; i < nof_cbs; ++i) {
    const srsgpu_ldpc_decoder_config& c = cfgs[i];
    int r = add_decoder_cb(ctx, i, c.base_graph, c.lifting_size, c.nof_filler_bits, c.nof_crc_bits, c.max_iterations,
                           c.scaling_factor, c.crc_poly, /*early_stop=*/true, c.llr_offset, c.nof_llrs, c.out_offset,
                           batch);
    if (r != SRSGPU_OK) {
      return r;
    }
  }
  const int r = upload_decoder_plan(ctx, impl, batch, plan_out);
  if (r == SRSGPU_OK) {
    guard.commit((*plan_out)->crc_refs);
  }
  return r;
}

int srsgpu_ldpc_decoder_plan_execute(const srsgpu_ldpc_decoder_plan* plan,
                                     const int8_t*                   d_llrs,
                                     uint8_t*                        d_out,
                                     int32_t*                        d_nof_iterations,
                                     void*                           stream)
{
  if (plan == nullptr || d_llrs == nullptr || d_out == nullptr || d_nof_iterations == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  return execute_decoder_plan(plan, d_llrs, d_out, d_nof_iterations, nullptr, static_cast<hipStream_t>(stream));
}

void srsgpu_ldpc_decoder_plan_destroy(srsgpu_ldpc_decoder_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  if (!plan->crc_refs.empty()) {
    std::lock_guard<std::mutex> lock(plan->ctx->mtx);
    crc_release_locked(plan->ctx, plan->crc_refs);
  }
  for (auto& g : plan->groups) {
    if (g.d_desc != nullptr) {
      (void)hipFree(g.d_desc);
    }
    if (g.d_dm != nullptr) {
      (void)hipFree(g.d_dm);
    }
  }
  delete plan;
}

int srsgpu_ldpc_decode(srsgpu_context*                   ctx,
                       int                               impl,
                       const srsgpu_ldpc_decoder_config* cfgs,
                       uint32_t                          nof_cbs,
                       const int8_t*                     d_llrs,
                       uint8_t*                          d_out,
                       int32_t*                          d_nof_iterations,
                       void*                             stream)
{
  srsgpu_ldpc_decoder_plan* plan = nullptr;
  int                       r    = srsgpu_ldpc_decoder_plan_create(ctx, impl, cfgs, nof_cbs, &plan);
  if (r != SRSGPU_OK) {
    return r;
  }
  r = srsgpu_ldpc_decoder_plan_execute(plan, d_llrs, d_out, d_nof_iterations, stream);
  if (r == SRSGPU_OK) {
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
      r = fail(SRSGPU_ERR_HIP, "decoder execution failed: %s", hipGetErrorString(e));
    }
  }
  srsgpu_ldpc_decoder_plan_destroy(plan);
  return r;
}


int srsgpu_pusch_cb_plan_create(srsgpu_context*               ctx,
                                int                           impl,
                                const srsgpu_pusch_cb_config* cfgs,
                                uint32_t                      nof_cbs,
                                srsgpu_pusch_cb_plan**        plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_cbs > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (impl != SRSGPU_LDPC_IMPL_GENERIC && impl != SRSGPU_LDPC_IMPL_SIMD) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid implementation %d", impl);
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  crc_ref_guard        guard(ctx);
  dec_batch            batch;
  batch.crc_refs = &guard.refs;
  std::vector<dm_desc> dms;
  for (uint32_t i = 0; i < nof_cbs; ++i) {
    const srsgpu_pusch_cb_config& c = cfgs[i];
    pusch_cb_params p{c.base_graph, c.rv, c.modulation_order, c.crc_poly, c.lifting_size, c.nof_filler_bits,
                      c.nof_crc_bits, c.max_iterations, c.new_data != 0, c.use_early_stop != 0, c.scaling_factor,
                      c.Nref, c.rm_length, c.llr_offset, c.harq_offset, c.out_offset, i};
    int r = add_pusch_cb(ctx, i, p, batch, dms);
    if (r != SRSGPU_OK) {
      return r;
    }
  }
  const int r = upload_pusch_cb_plan(ctx, impl, batch, dms, plan_out);
  if (r == SRSGPU_OK) {
    guard.commit((*plan_out)->crc_refs);
  }
  return r;
}

int srsgpu_pusch_cb_plan_execute(const srsgpu_pusch_cb_plan* plan,
                                 const int8_t*               d_llrs,
                                 int8_t*                     d_harq,
                                 uint8_t*                    d_out,
                                 int32_t*                    d_nof_iterations,
                                 uint8_t*                    d_cb_crc_ok,
                                 void*                       stream)
{
  if (plan == nullptr || d_llrs == nullptr || d_harq == nullptr || d_out == nullptr || d_nof_iterations == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  return execute_pusch_cb_plan(plan, d_llrs, d_harq, d_out, d_nof_iterations, d_cb_crc_ok,
                               static_cast<hipStream_t>(stream));
}

void srsgpu_pusch_cb_plan_destroy(srsgpu_pusch_cb_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  if (!plan->crc_refs.empty()) {
    std::lock_guard<std::mutex> lock(plan->ctx->mtx);
    crc_release_locked(plan->ctx, plan->crc_refs);
  }
  if (plan->d_dm != nullptr) {
    (void)hipFree(plan->d_dm);
  }
  srsgpu_ldpc_decoder_plan_destroy(plan->dec);
  delete plan;
}


int srsgpu_pdsch_encoder_plan_create(srsgpu_context*               ctx,
                                     const srsgpu_pdsch_tb_config* cfgs,
                                     uint32_t                      nof_tbs,
                                     srsgpu_pdsch_encoder_plan**   plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_tbs > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  crc_ref_guard            guard(ctx);
  static const double      shift_bg1[4] = {0, 17, 33, 56};  // ldpc_rate_matcher_impl.cpp:34
  static const double      shift_bg2[4] = {0, 13, 25, 43};
  std::vector<tb_crc_desc> tbd(nof_tbs);
  std::vector<enc_desc>    encs[2], encs_pk[2];
  int                      maxz[2]   = {0, 0};
  // SRSGPU_OPTION_ENCODER_BYTE_KERNEL routes every codeblock to the byte kernel (parity checks of both kernels).
  const bool               force_byte_kernel = ctx->opt_encoder_byte_kernel != 0;
  size_t                   out_begin = ~size_t(0), out_end = 0;
  bool                     word_aligned = true;  // every codeblock starts and ends on a 32-bit word boundary
  std::vector<std::pair<size_t, size_t>> cw_ranges;  // [begin, end) bytes of each TB's codeword
  for (uint32_t t = 0; t < nof_tbs; ++t) {
    const srsgpu_pdsch_tb_config& c = cfgs[t];
    const int                     qm = c.modulation_order;
    if (c.rv > 3 || (qm != 1 && qm != 2 && qm != 4 && qm != 6 && qm != 8) || c.cw_offset % 4 != 0) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tb %u: invalid rv, modulation order or unaligned codeword offset", t);
    }
    tb_segmentation seg;
    std::string     err;
    if (!sch_segment(static_cast<int>(c.tbs_bytes) * 8, c.base_graph, qm, c.nof_layers,
                     static_cast<int>(c.nof_ch_symbols), seg, err)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tb %u: %s", t, err.c_str());
    }
    tbd[t] = {c.tb_offset, c.tbs_bytes, seg.tb_crc_len == 24 ? 0x1864cfbu : 0x11021u,
              static_cast<uint32_t>(seg.tb_crc_len), NO_CRC_TABLE};
    // TB CRC from a per-bit table (cached per length); when the arena is full the kernel uses the byte-table method.
    tbd[t].table = try_crc_table(ctx, seg.tb_crc_len == 24 ? SRSGPU_CRC24A : SRSGPU_CRC16,
                                 static_cast<int>(c.tbs_bytes) * 8, guard.refs);
    const int Z    = seg.Z;
    const int pos  = lifting_position(Z);
    const int N    = (((seg.bg == 1) ? kBG1_N_FULL : kBG2_N_FULL) - 2) * Z;
    const int K    = (seg.bg == 1) ? kBG1_K : kBG2_K;
    const int nsys = (K - 2) * Z;
    const int Ncb  = (c.Nref > 0 && static_cast<int>(c.Nref) < N) ? static_cast<int>(c.Nref) : N;
    if (Ncb <= nsys) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tb %u: circular buffer shorter than the systematic part", t);
    }
    const int ninfo = nsys - seg.filler;
    const int k0    = static_cast<int>(std::floor(((seg.bg == 1 ? shift_bg1 : shift_bg2)[c.rv] * Ncb) / N)) * Z;
    const int v0    = k0 < ninfo ? k0 : (k0 < nsys ? ninfo : k0 - seg.filler);
    const int V     = Ncb - seg.filler;
    uint32_t  crc_tab = NO_CRC_TABLE;
    if (seg.cb_crc_len > 0) {
      int r = get_crc_table(ctx, SRSGPU_CRC24B, seg.cbs[0].used, crc_tab, guard.refs);
      if (r != SRSGPU_OK) {
        return r;
      }
    }
    for (int i = 0; i < seg.C; ++i) {
      const cb_segment& cb = seg.cbs[static_cast<size_t>(i)];
      enc_desc          d{};
      d.tb_byte_offset = c.tb_offset;
      d.tb_bit_offset  = static_cast<uint32_t>(cb.tb_offset);
      d.tb_bits        = static_cast<uint32_t>(seg.tbs);
      d.out_bit_offset = c.cw_offset * 8u + static_cast<uint32_t>(cb.cw_offset);
      d.crc_table      = crc_tab;
      d.div_magic      = static_cast<uint32_t>(((1ULL << 32) + static_cast<uint64_t>(Z) - 1) / static_cast<uint64_t>(Z));
      d.E              = static_cast<uint32_t>(cb.E);
      d.Ncb            = static_cast<uint32_t>(Ncb);
      d.v0             = static_cast<uint32_t>(v0);
      d.tb_index       = t;
      d.Z              = static_cast<uint16_t>(Z);
      d.zpos           = static_cast<uint16_t>(pos);
      d.nof_data       = static_cast<uint16_t>(cb.nof_data);
      d.used           = static_cast<uint16_t>(cb.used);
      d.filler         = static_cast<uint16_t>(seg.filler);
      d.tb_crc_len     = static_cast<uint8_t>(seg.tb_crc_len);
      d.Qm             = static_cast<uint8_t>(qm);
      d.tb_crc_table   = tbd[t].table;
      // Last circular-buffer position the rate matcher reads -> extension parity rows to compute.
      int kmax;
      if (cb.E >= V - v0) {
        kmax = Ncb - 1;
      } else {
        const int vend = v0 + cb.E - 1;
        kmax           = vend < ninfo ? vend : vend + seg.filler;
      }
      const int last_col = (kmax + 2 * Z) / Z;  // full-codeblock node index
      const int n_ext    = last_col - (K + 4) + 1;
      d.n_ext            = static_cast<uint8_t>(n_ext < 0 ? 0 : n_ext);
      word_aligned       = word_aligned && (d.out_bit_offset % 32u) == 0u && (cb.E % 32) == 0;
      // Packed kernel: Z % 32 == 0 and byte-aligned codeblock data (and CB CRC position).
      const bool packed = !force_byte_kernel && Z % 32 == 0 && ((cb.tb_offset | cb.nof_data) & 7) == 0 &&
                          (seg.cb_crc_len == 0 || (cb.used & 7) == 0);
      (packed ? encs_pk : encs)[seg.bg - 1].push_back(d);
    }
    maxz[seg.bg - 1] = Z > maxz[seg.bg - 1] ? Z : maxz[seg.bg - 1];
    out_begin        = std::min(out_begin, static_cast<size_t>(c.cw_offset));
    out_end          = std::max(out_end, static_cast<size_t>(c.cw_offset) + (static_cast<size_t>(seg.cw_length) + 31) / 32 * 4);
    word_aligned     = word_aligned && seg.cw_length % 32 == 0;
    cw_ranges.emplace_back(c.cw_offset, static_cast<size_t>(c.cw_offset) + static_cast<size_t>(seg.cw_length) / 8);
  }
  // No memset when every output word is written whole by exactly one codeblock: aligned codeblocks and TB codewords
  // that tile [out_begin, out_end) (no gap left unwritten, no overlap).
  bool tiled = word_aligned;
  if (tiled) {
    std::sort(cw_ranges.begin(), cw_ranges.end());
    for (size_t i = 1; i < cw_ranges.size() && tiled; ++i) {
      tiled = cw_ranges[i].first == cw_ranges[i - 1].second;
    }
  }
  const bool zero_out = !tiled || ctx->opt_encoder_zero_output != 0;
  // TB CRC slices: a TB with a contribution table is spread over TB_CRC_SLICE_BYTES ranges (a max-TBS TB of one
  // workgroup would otherwise serialise ~150 KB of byte-table steps); without a table it stays one slice.
  std::vector<tb_crc_slice> slices;
  for (uint32_t t = 0; t < nof_tbs; ++t) {
    const uint32_t step = tbd[t].table != NO_CRC_TABLE ? TB_CRC_SLICE_BYTES : std::max(tbd[t].nbytes, 1u);
    for (uint32_t b = 0; b < std::max(tbd[t].nbytes, 1u); b += step) {
      slices.push_back({t, b, std::min(b + step, tbd[t].nbytes)});
    }
  }
  auto* plan      = new srsgpu_pdsch_encoder_plan();
  plan->ctx       = ctx;
  plan->nof_tbs   = static_cast<int>(nof_tbs);
  plan->nof_slices = static_cast<int>(slices.size());
  plan->out_begin = nof_tbs ? out_begin : 0;
  plan->out_end   = out_end;
  plan->zero_output = zero_out;
  bool ok         = true;
  if (nof_tbs > 0) {
    ok = hipMalloc(&plan->d_tb, tbd.size() * sizeof(tb_crc_desc)) == hipSuccess &&
         hipMemcpy(plan->d_tb, tbd.data(), tbd.size() * sizeof(tb_crc_desc), hipMemcpyHostToDevice) == hipSuccess &&
         hipMalloc(&plan->d_tb_crc, tbd.size() * sizeof(uint32_t)) == hipSuccess &&
         hipMalloc(&plan->d_slices, slices.size() * sizeof(tb_crc_slice)) == hipSuccess &&
         hipMemcpy(plan->d_slices, slices.data(), slices.size() * sizeof(tb_crc_slice), hipMemcpyHostToDevice) ==
             hipSuccess;
  }
  for (int b = 0; b < 2 && ok; ++b) {
    plan->count[b]    = static_cast<int>(encs[b].size());
    plan->count_pk[b] = static_cast<int>(encs_pk[b].size());
    plan->threads[b]  = ((maxz[b] + 63) / 64) * 64;
    encs[b].insert(encs[b].end(), encs_pk[b].begin(), encs_pk[b].end());
    if (!encs[b].empty()) {
      ok = hipMalloc(&plan->d_enc[b], encs[b].size() * sizeof(enc_desc)) == hipSuccess &&
           hipMemcpy(plan->d_enc[b], encs[b].data(), encs[b].size() * sizeof(enc_desc), hipMemcpyHostToDevice) ==
               hipSuccess;
    }
  }
  if (!ok) {
    srsgpu_pdsch_encoder_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload encoder descriptors");
  }
  plan->inline_tb_crc = plan->count[0] == 0 && plan->count[1] == 0 &&
                        std::all_of(tbd.begin(), tbd.end(), [](const tb_crc_desc& t) {
                          return t.table != NO_CRC_TABLE && t.nbytes <= TB_CRC_INLINE_MAX_BYTES;
                        });
  guard.commit(plan->crc_refs);
  *plan_out = plan;
  return SRSGPU_OK;
}

uint32_t srsgpu_pdsch_encoder_plan_nof_codeblocks(const srsgpu_pdsch_encoder_plan* plan)
{
  return plan == nullptr ? 0u
                         : static_cast<uint32_t>(plan->count[0] + plan->count[1] + plan->count_pk[0] +
                                                 plan->count_pk[1]);
}

int srsgpu_pdsch_encoder_plan_execute(const srsgpu_pdsch_encoder_plan* plan,
                                      const uint8_t*                   d_tbs,
                                      uint8_t*                         d_codewords,
                                      void*                            stream)
{
  if (plan == nullptr || d_tbs == nullptr || d_codewords == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  auto  s  = static_cast<hipStream_t>(stream);
  auto* ev = plan->timer.begin();
  stage_timer::mark(ev, 0, s);
  if (plan->zero_output && plan->out_end > plan->out_begin) {
    HIP_TRY(hipMemsetAsync(d_codewords + plan->out_begin, 0, plan->out_end - plan->out_begin, s));
  }
  if (!plan->inline_tb_crc && plan->nof_tbs > 0) {
    HIP_TRY(hipMemsetAsync(plan->d_tb_crc, 0, static_cast<size_t>(plan->nof_tbs) * sizeof(uint32_t), s));
    launch_tb_crc(plan->d_tb, plan->d_slices, plan->nof_slices, d_tbs, plan->d_tb_crc, plan->ctx->d_crc_arena, s);
    HIP_TRY(hipGetLastError());
  }
  stage_timer::mark(ev, 1, s);
  for (int b = 0; b < 2; ++b) {
    auto* out = reinterpret_cast<uint32_t*>(d_codewords);
    if (plan->count_pk[b] > 0) {
      launch_pdsch_encode_packed(b + 1, plan->d_enc[b] + plan->count[b], plan->count_pk[b], d_tbs, plan->d_tb_crc,
                                 plan->inline_tb_crc ? plan->d_tb : nullptr, out, plan->ctx->d_shifts[b],
                                 plan->ctx->d_core[b], plan->ctx->d_crc_arena, plan->ctx->d_crc_slice, s);
      HIP_TRY(hipGetLastError());
    }
    if (plan->count[b] > 0) {
      launch_pdsch_encode(b + 1, plan->d_enc[b], plan->count[b], plan->threads[b], d_tbs, plan->d_tb_crc, out,
                          plan->ctx->d_shifts[b], plan->ctx->d_core[b], plan->ctx->d_crc_arena, s);
      HIP_TRY(hipGetLastError());
    }
  }
  stage_timer::mark(ev, 2, s);
  return SRSGPU_OK;
}

int srsgpu_pdsch_encoder_plan_enable_timing(srsgpu_pdsch_encoder_plan* plan, int enable)
{
  if (plan == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  plan->timer.stages  = 2;
  plan->timer.enabled = enable != 0;
  return SRSGPU_OK;
}

int srsgpu_pdsch_encoder_plan_stage_times(srsgpu_pdsch_encoder_plan* plan, float* ms, uint32_t* nof_executes)
{
  if (plan == nullptr || ms == nullptr || nof_executes == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  plan->timer.stages = 2;
  if (plan->timer.collect(ms, nof_executes) != 0) {
    return fail(SRSGPU_ERR_HIP, "event synchronisation failed");
  }
  return SRSGPU_OK;
}

void srsgpu_pdsch_encoder_plan_destroy(srsgpu_pdsch_encoder_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  if (!plan->crc_refs.empty()) {
    std::lock_guard<std::mutex> lock(plan->ctx->mtx);
    crc_release_locked(plan->ctx, plan->crc_refs);
  }
  for (void* p : {static_cast<void*>(plan->d_tb), static_cast<void*>(plan->d_tb_crc), static_cast<void*>(plan->d_slices),
                  static_cast<void*>(plan->d_enc[0]),
                  static_cast<void*>(plan->d_enc[1])}) {
    if (p != nullptr) {
      (void)hipFree(p);
    }
  }
  delete plan;
}


int srsgpu_pusch_decoder_plan_create(srsgpu_context*               ctx,
                                     int                           impl,
                                     const srsgpu_pusch_tb_config* cfgs,
                                     uint32_t                      nof_tbs,
                                     srsgpu_pusch_decoder_plan**   plan_out)
{
  if (ctx == nullptr || plan_out == nullptr || (cfgs == nullptr && nof_tbs > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (impl != SRSGPU_LDPC_IMPL_GENERIC && impl != SRSGPU_LDPC_IMPL_SIMD) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid implementation %d", impl);
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  crc_ref_guard            guard(ctx);
  dec_batch                batch;
  batch.crc_refs = &guard.refs;
  std::vector<dm_desc>     dms;
  std::vector<tb_dec_desc> tbs(nof_tbs);
  for (uint32_t t = 0; t < nof_tbs; ++t) {
    const srsgpu_pusch_tb_config& c = cfgs[t];
    tb_segmentation               seg;
    std::string                   err;
    if (!sch_segment(static_cast<int>(c.tbs_bytes) * 8, c.base_graph, c.modulation_order, c.nof_layers,
                     static_cast<int>(c.nof_ch_symbols), seg, err)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "tb %u: %s", t, err.c_str());
    }
    // pusch_decoder_impl.cpp:34 select_crc: CRC24B when segmented, else the TB CRC.
    const int crc_poly = (seg.C > 1) ? SRSGPU_CRC24B : (seg.tbs > 3824 ? SRSGPU_CRC24A : SRSGPU_CRC16);
    const int N        = (((seg.bg == 1) ? kBG1_N_FULL : kBG2_N_FULL) - 2) * seg.Z;
    for (int i = 0; i < seg.C; ++i) {
      const cb_segment& cb = seg.cbs[static_cast<size_t>(i)];
      const uint32_t    ci = c.cb_offset + static_cast<uint32_t>(i);
      pusch_cb_params   p{seg.bg, c.rv, c.modulation_order, crc_poly, seg.Z, seg.filler,
                        seg.C > 1 ? 24 : seg.tb_crc_len, c.max_iterations, c.new_data != 0, c.use_early_stop != 0,
                        c.scaling_factor, c.Nref, static_cast<uint32_t>(cb.E),
                        c.llr_offset + static_cast<uint32_t>(cb.cw_offset),
                        c.harq_offset + static_cast<uint32_t>(i) * static_cast<uint32_t>(N), ci * CB_MSG_STRIDE, ci};
      int r = add_pusch_cb(ctx, ci, p, batch, dms);
      if (r != SRSGPU_OK) {
        return r;
      }
    }
    tb_dec_desc& d = tbs[t];
    d.first_cb     = c.cb_offset;
    d.nof_cbs      = static_cast<uint32_t>(seg.C);
    d.tbs_bits     = static_cast<uint32_t>(seg.tbs);
    d.cb_data_bits = static_cast<uint32_t>(seg.C > 1 ? seg.cbs[0].used : seg.tbs);
    d.data_magic   = static_cast<uint32_t>(((1ULL << 32) + d.cb_data_bits - 1) / d.cb_data_bits);
    d.tb_offset    = c.tb_offset;
    d.tb_index     = t;
    d.crc_table    = (seg.C > 1) ? try_crc_table(ctx, SRSGPU_CRC24A, seg.tbs, guard.refs) : NO_CRC_TABLE;
  }
  auto* plan    = new srsgpu_pusch_decoder_plan();
  plan->ctx     = ctx;
  plan->nof_tbs = static_cast<int>(nof_tbs);
  // 1 024 lanes when a TB is large (its CRC chain per lane shrinks 4x); one wave when every TB is a single small
  // codeblock (copy only: the codeblock CRC covers it; block_crc_bytes, which needs 256 lanes, is never reached).
  const bool any_large = std::any_of(tbs.begin(), tbs.end(), [](const tb_dec_desc& t) {
    return t.tbs_bits / 8u > TB_CRC_INLINE_MAX_BYTES;
  });
  const bool all_small_single = std::all_of(tbs.begin(), tbs.end(), [](const tb_dec_desc& t) {
    return t.nof_cbs == 1 && t.tbs_bits / 8u <= 2048u;
  });
  plan->tb_threads = any_large ? 1024 : (all_small_single ? 64 : 256);
  // Few large segmented TBs (at most 8, every one segmented, byte-aligned and with a CRC table, and AT LEAST one of them
  // above the inline size - the plan's smaller segmented TBs are then sliced too, which is correct, only not needed): the TB
  // stage runs over TB_SLICE_BYTES slices, several workgroups per TB, instead of one 1024-lane workgroup per TB, whose
  // byte copy and CRC chain take ~15 us for a 37 KB TB. That latency is what a slot processor's one-PDU slot waits for
  // (UL one-PDU slot batch +3 %); with many TBs per launch the single workgroups already fill the GPU and the slices'
  // per-workgroup overhead costs throughput (test-mode bench, 32 TBs: 308.7k vs 304.4k slots/s sliced), so those keep
  // one workgroup per TB (profiles/r4_tb_sliced_ab.txt).
  const bool sliceable = !tbs.empty() && std::all_of(tbs.begin(), tbs.end(), [](const tb_dec_desc& t) {
    return t.nof_cbs > 1 && t.crc_table != NO_CRC_TABLE && (t.cb_data_bits & 7u) == 0;
  });
  std::vector<tb_slice> slices;
  if (sliceable && any_large && tbs.size() <= 8) {
    for (uint32_t t = 0; t < tbs.size(); ++t) {
      const uint32_t bytes = tbs[t].tbs_bits / 8u;
      const uint32_t n     = (bytes + TB_SLICE_BYTES - 1) / TB_SLICE_BYTES;
      for (uint32_t k = 0; k < n; ++k) {
        slices.push_back({t, k * TB_SLICE_BYTES, std::min(bytes, (k + 1) * TB_SLICE_BYTES), n});
      }
    }
  }
  int r         = upload_pusch_cb_plan(ctx, impl, batch, dms, &plan->cbs);
  if (r != SRSGPU_OK) {
    delete plan;
    return r;
  }
  if (nof_tbs > 0 && (hipMalloc(&plan->d_tb, tbs.size() * sizeof(tb_dec_desc)) != hipSuccess ||
                      hipMemcpy(plan->d_tb, tbs.data(), tbs.size() * sizeof(tb_dec_desc), hipMemcpyHostToDevice) !=
                          hipSuccess)) {
    srsgpu_pusch_decoder_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload transport block descriptors");
  }
  if (!slices.empty()) {
    if (hipMalloc(&plan->d_slices, slices.size() * sizeof(tb_slice)) != hipSuccess ||
        hipMemcpy(plan->d_slices, slices.data(), slices.size() * sizeof(tb_slice), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMalloc(&plan->d_tb_acc, 2 * tbs.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(plan->d_tb_acc, 0, 2 * tbs.size() * sizeof(uint32_t)) != hipSuccess) {
      srsgpu_pusch_decoder_plan_destroy(plan);
      return fail(SRSGPU_ERR_HIP, "failed to upload transport block slices");
    }
    plan->nof_slices = static_cast<int>(slices.size());
  }
  guard.commit(plan->crc_refs);
  *plan_out = plan;
  return SRSGPU_OK;
}

namespace {
/// The TB stage of a decoder plan: sliced over several workgroups per TB, or one workgroup per TB.
void launch_plan_tb_stage(const srsgpu_pusch_decoder_plan* plan, uint8_t* d_cb_crc_ok, const uint8_t* d_cb_msgs,
                          uint8_t* d_tbs, uint8_t* d_tb_crc_ok, hipStream_t s)
{
  if (plan->nof_slices > 0) {
    launch_pusch_tb_sliced(plan->d_tb, plan->d_slices, plan->nof_slices, d_cb_crc_ok, d_cb_msgs, d_tbs, d_tb_crc_ok,
                           plan->ctx->d_crc_arena, plan->d_tb_acc, plan->d_tb_acc + plan->nof_tbs, s);
  } else {
    launch_pusch_tb(plan->d_tb, plan->nof_tbs, plan->tb_threads, d_cb_crc_ok, d_cb_msgs, d_tbs, d_tb_crc_ok,
                    plan->ctx->d_crc_arena, s);
  }
}
} // namespace

uint32_t srsgpu_pusch_decoder_plan_nof_codeblocks(const srsgpu_pusch_decoder_plan* plan)
{
  return plan == nullptr ? 0u : static_cast<uint32_t>(plan->cbs->nof_cbs);
}

uint64_t srsgpu_pusch_decoder_plan_decoder_input_llrs(const srsgpu_pusch_decoder_plan* plan)
{
  return (plan == nullptr || plan->cbs == nullptr || plan->cbs->dec == nullptr) ? 0u : plan->cbs->dec->input_llrs;
}

namespace {
int execute_pusch_decoder_plan(const srsgpu_pusch_decoder_plan* plan,
                               const int8_t*                    d_llrs,
                               int8_t*                          d_harq,
                               int8_t* const*                   d_harq_cbs,
                               uint8_t*                         d_cb_crc_ok,
                               uint8_t*                         d_cb_msgs,
                               int32_t*                         d_cb_nof_iterations,
                               uint8_t*                         d_tbs,
                               uint8_t*                         d_tb_crc_ok,
                               hipStream_t                      s)
{
  auto* ev  = plan->timer.begin();
  auto* evd = plan->timer_dec.begin();
  stage_timer::mark(ev, 0, s);
  launch_rate_dematch(plan->cbs->impl, plan->cbs->d_dm, plan->cbs->nof_cbs, d_llrs, d_harq, d_cb_crc_ok, s,
                      d_harq_cbs);
  HIP_TRY(hipGetLastError());
  stage_timer::mark(ev, 1, s);
  stage_timer::mark(evd, 0, s);
  int r = execute_decoder_plan(plan->cbs->dec, d_harq, d_cb_msgs, d_cb_nof_iterations, d_cb_crc_ok, s, d_llrs, d_harq,
                               d_harq_cbs);
  if (r != SRSGPU_OK) {
    return r;
  }
  stage_timer::mark(evd, 1, s);
  stage_timer::mark(ev, 2, s);
  launch_plan_tb_stage(plan, d_cb_crc_ok, d_cb_msgs, d_tbs, d_tb_crc_ok, s);
  HIP_TRY(hipGetLastError());
  stage_timer::mark(ev, 3, s);
  return SRSGPU_OK;
}
} // namespace

int srsgpu_pusch_decoder_plan_execute(const srsgpu_pusch_decoder_plan* plan,
                                      const int8_t*                    d_llrs,
                                      int8_t*                          d_harq,
                                      uint8_t*                         d_cb_crc_ok,
                                      uint8_t*                         d_cb_msgs,
                                      int32_t*                         d_cb_nof_iterations,
                                      uint8_t*                         d_tbs,
                                      uint8_t*                         d_tb_crc_ok,
                                      void*                            stream)
{
  if (plan == nullptr || d_llrs == nullptr || d_harq == nullptr || d_cb_crc_ok == nullptr || d_cb_msgs == nullptr ||
      d_cb_nof_iterations == nullptr || d_tbs == nullptr || d_tb_crc_ok == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  return execute_pusch_decoder_plan(plan, d_llrs, d_harq, nullptr, d_cb_crc_ok, d_cb_msgs, d_cb_nof_iterations, d_tbs,
                                    d_tb_crc_ok, static_cast<hipStream_t>(stream));
}

int srsgpu_pusch_decoder_plan_execute_arena(const srsgpu_pusch_decoder_plan* plan,
                                            const int8_t*                    d_llrs,
                                            int8_t* const*                   d_harq_cbs,
                                            uint8_t*                         d_cb_crc_ok,
                                            uint8_t*                         d_cb_msgs,
                                            int32_t*                         d_cb_nof_iterations,
                                            uint8_t*                         d_tbs,
                                            uint8_t*                         d_tb_crc_ok,
                                            void*                            stream)
{
  if (plan == nullptr || d_llrs == nullptr || d_harq_cbs == nullptr || d_cb_crc_ok == nullptr ||
      d_cb_msgs == nullptr || d_cb_nof_iterations == nullptr || d_tbs == nullptr || d_tb_crc_ok == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  return execute_pusch_decoder_plan(plan, d_llrs, nullptr, d_harq_cbs, d_cb_crc_ok, d_cb_msgs, d_cb_nof_iterations,
                                    d_tbs, d_tb_crc_ok, static_cast<hipStream_t>(stream));
}

int srsgpu_pusch_decoder_plan_assemble(const srsgpu_pusch_decoder_plan* plan,
                                       uint8_t*                         d_cb_crc_ok,
                                       const uint8_t*                   d_cb_msgs,
                                       uint8_t*                         d_tbs,
                                       uint8_t*                         d_tb_crc_ok,
                                       void*                            stream)
{
  if (plan == nullptr || d_cb_crc_ok == nullptr || d_cb_msgs == nullptr || d_tbs == nullptr ||
      d_tb_crc_ok == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  launch_plan_tb_stage(plan, d_cb_crc_ok, d_cb_msgs, d_tbs, d_tb_crc_ok, static_cast<hipStream_t>(stream));
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

int srsgpu_pusch_decoder_plan_enable_timing(srsgpu_pusch_decoder_plan* plan, int enable)
{
  if (plan == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  plan->timer.stages      = 3;
  plan->timer.enabled     = enable == 1;
  plan->timer_dec.stages  = 1;
  plan->timer_dec.enabled = enable == 2;
  return SRSGPU_OK;
}

int srsgpu_pusch_decoder_plan_stage_times(srsgpu_pusch_decoder_plan* plan, float* ms, uint32_t* nof_executes)
{
  if (plan == nullptr || ms == nullptr || nof_executes == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  plan->timer.stages     = 3;
  plan->timer_dec.stages = 1;
  float    dec_ms = 0;
  uint32_t n = 0, n_dec = 0;
  if (plan->timer.collect(ms, &n) != 0 || plan->timer_dec.collect(&dec_ms, &n_dec) != 0) {
    return fail(SRSGPU_ERR_HIP, "event synchronisation failed");
  }
  ms[1] += dec_ms;
  *nof_executes = n > n_dec ? n : n_dec;
  return SRSGPU_OK;
}

void srsgpu_pusch_decoder_plan_destroy(srsgpu_pusch_decoder_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  if (!plan->crc_refs.empty()) {
    std::lock_guard<std::mutex> lock(plan->ctx->mtx);
    crc_release_locked(plan->ctx, plan->crc_refs);
  }
  srsgpu_pusch_cb_plan_destroy(plan->cbs);
  if (plan->d_tb != nullptr) {
    (void)hipFree(plan->d_tb);
  }
  if (plan->d_slices != nullptr) {
    (void)hipFree(plan->d_slices);
  }
  if (plan->d_tb_acc != nullptr) {
    (void)hipFree(plan->d_tb_acc);
  }
  delete plan;
}

#ifdef LDPC_DEC_PROFILE
/// Instrumented builds only: phase stamps of the last decoder launch (see ldpc_decoder.hip, DEC_STAMP).
int srsgpu_debug_decoder_profile(uint64_t* dst, uint32_t n, int packed)
{
  return packed ? srsgpu::debug_read_decoder_profile_pk(dst, n) : srsgpu::debug_read_decoder_profile(dst, n);
}
#endif
#ifdef CHEST_PROFILE
/// Instrumented builds only: phase stamps of the last estimator launch (pusch_chest.hip, CHEST_STAMP).
int srsgpu_debug_chest_profile(uint64_t* dst, uint32_t n)
{
  return srsgpu::debug_read_chest_profile(dst, n);
}
#endif
#ifdef ENC_PROFILE
/// Instrumented builds only: phase stamps of the last packed-encoder launch (ldpc_encoder.hip, ENC_STAMP).
int srsgpu_debug_encoder_profile(uint64_t* dst, uint32_t n)
{
  return srsgpu::debug_read_encoder_profile(dst, n);
}
#endif

} // extern "C"
