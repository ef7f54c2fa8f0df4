// Host side of the srsgpu C ABI (include/srsgpu_phy.h): contexts, validation mirroring the reference's assertions,
// CRC early-stop tables and work-descriptor plans. No compute happens on the host: every codeblock is processed by the
// HIP kernels; a missing/unsupported device makes every call fail loudly (there is no CPU fallback).
#include "srsgpu_phy.h"
#include "ldpc_base_graphs.h"
#include "srsgpu_internal.h"
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

using namespace srsgpu;

namespace {

thread_local std::string g_last_error = "";

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...)
{
  char    buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                                                  \
  do {                                                                                                                 \
    hipError_t err_ = (expr);                                                                                          \
    if (err_ != hipSuccess) {                                                                                          \
      return fail(SRSGPU_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(err_));                                    \
    }                                                                                                                  \
  } while (0)

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

constexpr size_t CRC_ARENA_WORDS = 4u << 20;  // 16 MiB of contribution tables

} // namespace

struct srsgpu_context {
  int                                  device      = 0;
  uint16_t*                            d_shifts[2] = {nullptr, nullptr};
  uint32_t*                            d_crc_arena = nullptr;
  size_t                               crc_used    = 0;
  std::map<std::pair<int, int>, size_t> crc_tables;
  std::mutex                           mtx;
};

struct srsgpu_ldpc_decoder_plan {
  srsgpu_context* ctx            = nullptr;
  int             impl           = SRSGPU_LDPC_IMPL_SIMD;
  dec_desc*       d_desc[2]      = {nullptr, nullptr};
  int             count[2]       = {0, 0};
  int             threads[2]     = {64, 64};
};

namespace {

/// Contribution table of every message bit to the CRC remainder: P[i] = x^(order + L - 1 - i) mod g(x), so that
/// CRC(m) = XOR of P[i] over the set bits m_i (the calculate() of crc_calculator_generic_impl.cpp:136 is linear).
int get_crc_table(srsgpu_context* ctx, int poly, int L, uint32_t& offset)
{
  auto key = std::make_pair(poly, L);
  auto it  = ctx->crc_tables.find(key);
  if (it != ctx->crc_tables.end()) {
    offset = static_cast<uint32_t>(it->second);
    return SRSGPU_OK;
  }
  unsigned order;
  uint64_t g;
  if (!crc_params(poly, order, g)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid CRC polynomial %d", poly);
  }
  if (ctx->crc_used + static_cast<size_t>(L) > CRC_ARENA_WORDS) {
    return fail(SRSGPU_ERR_NO_MEMORY, "CRC table arena exhausted");
  }
  std::vector<uint32_t> tab(static_cast<size_t>(L));
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
  HIP_TRY(hipMemcpy(ctx->d_crc_arena + ctx->crc_used, tab.data(), tab.size() * sizeof(uint32_t),
                    hipMemcpyHostToDevice));
  offset = static_cast<uint32_t>(ctx->crc_used);
  ctx->crc_tables.emplace(key, ctx->crc_used);
  ctx->crc_used += static_cast<size_t>(L);
  return SRSGPU_OK;
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
    if (hipMalloc(&ctx->d_shifts[bg - 1], tab.size() * sizeof(uint16_t)) != hipSuccess ||
        hipMemcpy(ctx->d_shifts[bg - 1], tab.data(), tab.size() * sizeof(uint16_t), hipMemcpyHostToDevice) !=
            hipSuccess) {
      srsgpu_context_destroy(ctx);
      return fail(SRSGPU_ERR_HIP, "failed to upload LDPC shift tables");
    }
  }
  if (hipMalloc(&ctx->d_crc_arena, CRC_ARENA_WORDS * sizeof(uint32_t)) != hipSuccess) {
    srsgpu_context_destroy(ctx);
    return fail(SRSGPU_ERR_NO_MEMORY, "failed to allocate the CRC table arena");
  }
  *out = ctx;
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
  if (ctx->d_crc_arena != nullptr) {
    (void)hipFree(ctx->d_crc_arena);
  }
  delete ctx;
}

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
  std::vector<dec_desc> descs[2];
  int                   maxz[2] = {0, 0};
  for (uint32_t i = 0; i < nof_cbs; ++i) {
    const srsgpu_ldpc_decoder_config& c = cfgs[i];
    if (c.base_graph != 1 && c.base_graph != 2) {
      return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid base graph %d", i, c.base_graph);
    }
    const int Z   = c.lifting_size;
    const int pos = lifting_position(Z);
    if (pos < 0) {
      return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid lifting size %d", i, Z);
    }
    const int K = (c.base_graph == 1) ? kBG1_K : kBG2_K;
    const int N = ((c.base_graph == 1) ? kBG1_N_FULL : kBG2_N_FULL) - 2;
    // ldpc_decoder_impl.cpp:48-:56
    if (c.max_iterations == 0) {
      return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: max iterations must be different to 0", i);
    }
    if (!(c.scaling_factor > 0.0f && c.scaling_factor < 1.0f)) {
      return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: scaling factor must be between 0 and 1 exclusively", i);
    }
    if (c.nof_crc_bits != 16 && c.nof_crc_bits != 24) {
      return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid number of CRC bits %d", i, c.nof_crc_bits);
    }
    // ldpc_decoder_impl.cpp:73-:88
    if (static_cast<int>(c.nof_llrs) > N * Z || static_cast<int>(c.nof_llrs) < (K + 2) * Z) {
      return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: input length %u outside [%d, %d]", i, c.nof_llrs, (K + 2) * Z,
                  N * Z);
    }
    if (c.nof_filler_bits >= (K - 2) * Z) {
      return fail(SRSGPU_ERR_INVALID_ARG, "cb %u: invalid number of filler bits %d", i, c.nof_filler_bits);
    }
    dec_desc d{};
    d.llr_offset      = c.llr_offset;
    d.nof_llr         = c.nof_llrs;
    d.out_offset      = c.out_offset;
    d.crc_table       = NO_CRC_TABLE;
    d.div_magic       = static_cast<uint32_t>(((1ULL << 32) + static_cast<uint64_t>(Z) - 1) / static_cast<uint64_t>(Z));
    d.Z               = static_cast<uint16_t>(Z);
    d.zpos            = static_cast<uint16_t>(pos);
    d.nof_significant = static_cast<uint16_t>(K * Z - c.nof_filler_bits);
    d.max_iter        = c.max_iterations;
    // avx2_support.h:71: identity above .9999, otherwise floor(sf * 2^16) in float arithmetic.
    d.sf16     = (static_cast<double>(c.scaling_factor) >= .9999)
                     ? 65536u
                     : static_cast<uint32_t>(static_cast<uint16_t>(c.scaling_factor * 65536U));
    d.sf       = c.scaling_factor;
    d.cb_index = i;
    if (c.crc_poly != SRSGPU_CRC_NONE) {
      int r = get_crc_table(ctx, c.crc_poly, K * Z - c.nof_filler_bits, d.crc_table);
      if (r != SRSGPU_OK) {
        return r;
      }
    }
    descs[c.base_graph - 1].push_back(d);
    maxz[c.base_graph - 1] = Z > maxz[c.base_graph - 1] ? Z : maxz[c.base_graph - 1];
  }
  auto* plan = new srsgpu_ldpc_decoder_plan();
  plan->ctx  = ctx;
  plan->impl = impl;
  for (int b = 0; b < 2; ++b) {
    plan->count[b]   = static_cast<int>(descs[b].size());
    plan->threads[b] = ((maxz[b] + 63) / 64) * 64;
    if (plan->count[b] == 0) {
      continue;
    }
    if (hipMalloc(&plan->d_desc[b], descs[b].size() * sizeof(dec_desc)) != hipSuccess ||
        hipMemcpy(plan->d_desc[b], descs[b].data(), descs[b].size() * sizeof(dec_desc), hipMemcpyHostToDevice) !=
            hipSuccess) {
      srsgpu_ldpc_decoder_plan_destroy(plan);
      return fail(SRSGPU_ERR_HIP, "failed to upload decoder descriptors");
    }
  }
  *plan_out = plan;
  return SRSGPU_OK;
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
  auto s = static_cast<hipStream_t>(stream);
  for (int b = 0; b < 2; ++b) {
    if (plan->count[b] == 0) {
      continue;
    }
    launch_ldpc_decode(b + 1, plan->impl, plan->d_desc[b], plan->count[b], plan->threads[b], d_llrs, d_out,
                       d_nof_iterations, plan->ctx->d_shifts[b], plan->ctx->d_crc_arena, s);
    HIP_TRY(hipGetLastError());
  }
  return SRSGPU_OK;
}

void srsgpu_ldpc_decoder_plan_destroy(srsgpu_ldpc_decoder_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  for (auto* p : plan->d_desc) {
    if (p != nullptr) {
      (void)hipFree(p);
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

} // extern "C"
