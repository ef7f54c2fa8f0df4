// Host side of the OFDM modulator / demodulator C ABI (include/srsgpu_phy.h): configuration checks with the
// reference's conditions (ofdm_modulator_impl.cpp:41-:44, ofdm_demodulator_impl.cpp:53-:68), cyclic-prefix lengths,
// the TS 38.211 section 5.4 phase-compensation coefficients (computed in double like phase_compensation_lut.h:50) and
// one job per (grid, port, symbol).
#include "capi_internal.h"
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstddef>
#include <vector>

using namespace srsgpu;

struct srsgpu_ofdm_plan {
  srsgpu_context*       ctx        = nullptr;
  bool                  inverse    = true;  ///< Modulator (inverse DFT) or demodulator.
  uint32_t              dft_size   = 0;
  uint32_t              nsc        = 0;
  uint32_t              window_off = 0;
  uint32_t              nof_ports  = 0;
  ofdm_job*             d_jobs     = nullptr;
  int                   nof_jobs   = 0;
  float*                d_scratch  = nullptr;  ///< Split sizes: one N-point complex row per job.
  std::vector<uint64_t> offsets;     ///< Sample offset of (grid, port); one extra entry = total.
  uint64_t              grid_words = 0;  ///< uint32 words of the plan's grids (all grids, ports and symbols).
};

namespace {

/// Cyclic prefix of symbol `symbol` of the subframe in samples (cyclic_prefix.h:93: kappa units (144 >> mu), +16 for
/// symbols 0 and 7 * 2^mu, extended 512 >> mu; one kappa unit is 2^mu * N / 2048 samples at N * scs).
uint32_t cp_samples(uint32_t mu, uint32_t N, bool extended, uint32_t symbol)
{
  uint32_t units;
  if (extended) {
    units = 512u >> mu;
  } else {
    units = 144u >> mu;
    if (symbol == 0 || symbol == 7u * (1u << mu)) {
      units += 16;
    }
  }
  return static_cast<uint32_t>((static_cast<uint64_t>(units) << mu) * N / 2048u);
}

int ensure_twiddles(srsgpu_context* ctx)
{
  if (ctx->d_ofdm_twiddles != nullptr) {
    return SRSGPU_OK;
  }
  std::vector<float> tw(2 * OFDM_MAX_DFT);
  for (uint32_t m = 0; m < OFDM_MAX_DFT; ++m) {
    const double a = -2.0 * M_PI * static_cast<double>(m) / static_cast<double>(OFDM_MAX_DFT);
    tw[2 * m]      = static_cast<float>(std::cos(a));
    tw[2 * m + 1]  = static_cast<float>(std::sin(a));
  }
  float* d = nullptr;
  if (hipMalloc(&d, tw.size() * sizeof(float)) != hipSuccess ||
      hipMemcpy(d, tw.data(), tw.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
    if (d != nullptr) {
      (void)hipFree(d);
    }
    return fail(SRSGPU_ERR_HIP, "failed to upload the DFT twiddle table");
  }
  ctx->d_ofdm_twiddles = d;
  return SRSGPU_OK;
}

int plan_create(srsgpu_context*           ctx,
                bool                      inverse,
                const srsgpu_ofdm_config* cfg,
                uint32_t                  nof_grids,
                uint32_t                  nof_ports,
                const uint32_t*           slot_index,
                srsgpu_ofdm_plan**        plan_out,
                uint32_t                  first_symbol = 0,
                uint32_t                  nof_symbols  = ~0u)
{
  if (ctx == nullptr || cfg == nullptr || plan_out == nullptr || (slot_index == nullptr && nof_grids > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  const uint32_t N   = cfg->dft_size;
  const uint32_t mu  = cfg->numerology;
  const uint32_t nsc = 12u * cfg->bw_rb;
  // The generic DFT's sizes (dft_processor_generic_impl.cpp:211-230): one LDS transform up to 8192 points, the
  // two-kernel split above (9216 .. 98304).
  const uint32_t m = (N % 3 == 0) ? N / 3 : N;
  const bool     pow2_ok = N >= 128 && N <= 8192 && (N & (N - 1)) == 0;
  const bool     x3_ok   = N % 3 == 0 && m >= 128 && m <= 2048 && (m & (m - 1)) == 0;
  if (!pow2_ok && !x3_ok && N != 4608 && ofdm_split_factor(N) == 0) {
    return fail(SRSGPU_ERR_INVALID_ARG,
                "DFT size %u not supported (2^n 128..8192, 3 x 2^m 384..6144, 4608, 9216, 12288, 18432, 24576, 36864, "
                "49152, 98304)",
                N);
  }
  if (mu > 4 || cfg->bw_rb == 0 || nsc >= N) {
    return fail(SRSGPU_ERR_INVALID_ARG, "the DFT size (%u) must be greater than the resource grid size (%u)", N, nsc);
  }
  if (!std::isnormal(cfg->scale)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "invalid scaling factor %g", static_cast<double>(cfg->scale));
  }
  const uint32_t woff = inverse ? 0u : cfg->nof_samples_window_offset;
  if (woff != 0 && woff >= 144u * N / 2048u) {
    return fail(SRSGPU_ERR_INVALID_ARG, "the DFT window offset (%u) must be lower than %u", woff, 144u * N / 2048u);
  }
  if (nof_ports == 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "no ports");
  }
  const bool     ext   = cfg->cp_extended != 0;
  const uint32_t nsymb = ext ? 12u : 14u;
  const uint32_t nslot = 1u << mu;  // slots per subframe
  // Symbol range of every grid (the symbol-granularity plans: ofdm_symbol_(de)modulator): whole slots by default.
  if (nof_symbols == ~0u) {
    nof_symbols = nsymb - std::min(first_symbol, nsymb);
  }
  if (nof_symbols == 0 || first_symbol + nof_symbols > nsymb) {
    return fail(SRSGPU_ERR_INVALID_ARG, "symbols [%u, %u) outside the %u symbols of a slot", first_symbol,
                first_symbol + nof_symbols, nsymb);
  }
  // Phase compensation per symbol of the subframe (phase_compensation_lut.h:50), times the scale, in float.
  const double              srate = 15e3 * static_cast<double>(1u << mu) * N;
  std::vector<std::complex<float>> coef(nsymb * nslot);
  {
    const double sign_two_pi = (inverse ? -1.0 : 1.0) * 2.0 * M_PI;
    uint64_t     offset      = 0;
    for (uint32_t s = 0; s < nsymb * nslot; ++s) {
      offset += cp_samples(mu, N, ext, s);
      const double              t  = static_cast<double>(offset) / srate;
      const std::complex<float> ph = static_cast<std::complex<float>>(std::polar(1.0, sign_two_pi * cfg->center_freq_hz * t));
      coef[s]                      = ph * cfg->scale;
      offset += N;
    }
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  int r = ensure_twiddles(ctx);
  if (r != SRSGPU_OK) {
    return r;
  }
  auto* plan       = new srsgpu_ofdm_plan();
  plan->ctx        = ctx;
  plan->inverse    = inverse;
  plan->dft_size   = N;
  plan->nsc        = nsc;
  plan->window_off = woff;
  plan->nof_ports  = nof_ports;
  std::vector<ofdm_job> jobs;
  uint64_t              pos = 0;
  for (uint32_t g = 0; g < nof_grids; ++g) {
    if (slot_index[g] >= nslot) {
      delete plan;
      return fail(SRSGPU_ERR_INVALID_ARG, "grid %u: slot index %u exceeds the %u slots per subframe", g, slot_index[g],
                  nslot);
    }
    for (uint32_t p = 0; p < nof_ports; ++p) {
      plan->offsets.push_back(pos);
      for (uint32_t i = 0; i < nof_symbols; ++i) {
        const uint32_t l   = first_symbol + i;
        const uint32_t s   = nsymb * slot_index[g] + l;
        const uint32_t cp  = cp_samples(mu, N, ext, s);
        ofdm_job       jb{};
        jb.grid_offset     = ((g * nof_ports + p) * nof_symbols + i) * nsc;
        jb.sample_offset   = static_cast<uint32_t>(pos);
        jb.cp_len          = cp;
        jb.coef_re         = coef[s].real();
        jb.coef_im         = coef[s].imag();
        jobs.push_back(jb);
        pos += cp + N;
      }
    }
  }
  plan->offsets.push_back(pos);
  plan->grid_words = static_cast<uint64_t>(nof_grids) * nof_ports * nof_symbols * nsc;
  if (pos >= (1ull << 32) || static_cast<uint64_t>(nof_grids) * nof_ports * nof_symbols * nsc >= (1ull << 32)) {
    delete plan;
    return fail(SRSGPU_ERR_INVALID_ARG, "batch too large for 32-bit offsets");
  }
  plan->nof_jobs = static_cast<int>(jobs.size());
  if (!jobs.empty() && (hipMalloc(&plan->d_jobs, jobs.size() * sizeof(ofdm_job)) != hipSuccess ||
                        hipMemcpy(plan->d_jobs, jobs.data(), jobs.size() * sizeof(ofdm_job), hipMemcpyHostToDevice) !=
                            hipSuccess)) {
    srsgpu_ofdm_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload OFDM jobs");
  }
  if (!jobs.empty() && ofdm_split_factor(N) != 0 &&
      hipMalloc(&plan->d_scratch, jobs.size() * static_cast<size_t>(N) * 2 * sizeof(float)) != hipSuccess) {
    srsgpu_ofdm_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to allocate the split-transform scratch (%zu MB)",
                jobs.size() * static_cast<size_t>(N) * 8 / (1u << 20));
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

} // namespace

extern "C" {

int srsgpu_ofdm_modulator_plan_create(srsgpu_context*           ctx,
                                      const srsgpu_ofdm_config* cfg,
                                      uint32_t                  nof_grids,
                                      uint32_t                  nof_ports,
                                      const uint32_t*           slot_index,
                                      srsgpu_ofdm_plan**        plan)
{
  return plan_create(ctx, true, cfg, nof_grids, nof_ports, slot_index, plan);
}

int srsgpu_ofdm_demodulator_plan_create(srsgpu_context*           ctx,
                                        const srsgpu_ofdm_config* cfg,
                                        uint32_t                  nof_grids,
                                        uint32_t                  nof_ports,
                                        const uint32_t*           slot_index,
                                        srsgpu_ofdm_plan**        plan)
{
  return plan_create(ctx, false, cfg, nof_grids, nof_ports, slot_index, plan);
}

int srsgpu_ofdm_modulator_symbols_plan_create(srsgpu_context*           ctx,
                                              const srsgpu_ofdm_config* cfg,
                                              uint32_t                  nof_ports,
                                              uint32_t                  slot_index,
                                              uint32_t                  first_symbol,
                                              uint32_t                  nof_symbols,
                                              srsgpu_ofdm_plan**        plan)
{
  return plan_create(ctx, true, cfg, 1, nof_ports, &slot_index, plan, first_symbol, nof_symbols);
}

int srsgpu_ofdm_demodulator_symbols_plan_create(srsgpu_context*           ctx,
                                                const srsgpu_ofdm_config* cfg,
                                                uint32_t                  nof_ports,
                                                uint32_t                  slot_index,
                                                uint32_t                  first_symbol,
                                                uint32_t                  nof_symbols,
                                                srsgpu_ofdm_plan**        plan)
{
  return plan_create(ctx, false, cfg, 1, nof_ports, &slot_index, plan, first_symbol, nof_symbols);
}

int srsgpu_ofdm_plan_concat(srsgpu_context*                ctx,
                            const srsgpu_ofdm_plan* const* members,
                            uint32_t                       nof_members,
                            srsgpu_ofdm_plan**             plan_out)
{
  if (ctx == nullptr || members == nullptr || plan_out == nullptr || nof_members == 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument or no member plans");
  }
  const srsgpu_ofdm_plan* first = members[0];
  if (first == nullptr) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null member plan");
  }
  std::lock_guard<std::mutex> lock(ctx->mtx);
  HIP_TRY(hipSetDevice(ctx->device));
  std::vector<ofdm_job> jobs;
  uint64_t              samples = 0;
  uint64_t              words   = 0;
  auto*                 plan    = new srsgpu_ofdm_plan();
  plan->ctx        = ctx;
  plan->inverse    = first->inverse;
  plan->dft_size   = first->dft_size;
  plan->nsc        = first->nsc;
  plan->window_off = first->window_off;
  plan->nof_ports  = first->nof_ports;
  for (uint32_t i = 0; i < nof_members; ++i) {
    const srsgpu_ofdm_plan* m = members[i];
    // One kernel runs every job: the members must agree on what the launch takes from the plan.
    if (m == nullptr || m->ctx != ctx || m->inverse != first->inverse || m->dft_size != first->dft_size ||
        m->nsc != first->nsc || m->window_off != first->window_off || m->nof_ports != first->nof_ports) {
      delete plan;
      return fail(SRSGPU_ERR_INVALID_ARG,
                  "member plan %u differs from the first in context, direction, DFT size, bandwidth, window offset or "
                  "ports",
                  i);
    }
    const size_t base = jobs.size();
    jobs.resize(base + m->nof_jobs);
    if (m->nof_jobs > 0 && hipMemcpy(jobs.data() + base, m->d_jobs, m->nof_jobs * sizeof(ofdm_job),
                                     hipMemcpyDeviceToHost) != hipSuccess) {
      delete plan;
      return fail(SRSGPU_ERR_HIP, "failed to read member plan %u's jobs", i);
    }
    for (size_t j = base; j != jobs.size(); ++j) {
      jobs[j].grid_offset += static_cast<uint32_t>(words);
      jobs[j].sample_offset += static_cast<uint32_t>(samples);
    }
    for (size_t k = 0; k + 1 < m->offsets.size(); ++k) {
      plan->offsets.push_back(m->offsets[k] + samples);
    }
    samples += m->offsets.empty() ? 0 : m->offsets.back();
    words += m->grid_words;
    if (samples >= (1ull << 32) || words >= (1ull << 32)) {
      delete plan;
      return fail(SRSGPU_ERR_INVALID_ARG, "batch too large for 32-bit offsets");
    }
  }
  plan->offsets.push_back(samples);
  plan->grid_words = words;
  plan->nof_jobs   = static_cast<int>(jobs.size());
  if (!jobs.empty() && (hipMalloc(&plan->d_jobs, jobs.size() * sizeof(ofdm_job)) != hipSuccess ||
                        hipMemcpy(plan->d_jobs, jobs.data(), jobs.size() * sizeof(ofdm_job), hipMemcpyHostToDevice) !=
                            hipSuccess)) {
    srsgpu_ofdm_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to upload OFDM jobs");
  }
  if (!jobs.empty() && ofdm_split_factor(plan->dft_size) != 0 &&
      hipMalloc(&plan->d_scratch, jobs.size() * static_cast<size_t>(plan->dft_size) * 2 * sizeof(float)) !=
          hipSuccess) {
    srsgpu_ofdm_plan_destroy(plan);
    return fail(SRSGPU_ERR_HIP, "failed to allocate the split-transform scratch");
  }
  *plan_out = plan;
  return SRSGPU_OK;
}

static_assert(sizeof(srsgpu_ofdm_job) == sizeof(ofdm_job) && offsetof(srsgpu_ofdm_job, sample_offset) ==
                  offsetof(ofdm_job, sample_offset) && offsetof(srsgpu_ofdm_job, cp_len) == offsetof(ofdm_job, cp_len) &&
                  offsetof(srsgpu_ofdm_job, coef_re) == offsetof(ofdm_job, coef_re),
              "srsgpu_ofdm_job is the kernel's job layout");

int srsgpu_ofdm_plan_get_jobs(const srsgpu_ofdm_plan* plan, srsgpu_ofdm_job* jobs, uint32_t capacity, uint32_t* nof_jobs)
{
  if (plan == nullptr || nof_jobs == nullptr || (jobs == nullptr && capacity > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  *nof_jobs      = static_cast<uint32_t>(plan->nof_jobs);
  const size_t n = std::min<size_t>(capacity, static_cast<size_t>(plan->nof_jobs));
  if (n > 0) {
    std::lock_guard<std::mutex> lock(plan->ctx->mtx);
    HIP_TRY(hipSetDevice(plan->ctx->device));
    HIP_TRY(hipMemcpy(jobs, plan->d_jobs, n * sizeof(ofdm_job), hipMemcpyDeviceToHost));
  }
  return SRSGPU_OK;
}

int srsgpu_ofdm_jobs_execute(const srsgpu_ofdm_plan* plan,
                             const srsgpu_ofdm_job*  d_jobs,
                             uint32_t                nof_jobs,
                             const void*             d_in,
                             void*                   d_out,
                             void*                   stream)
{
  if (plan == nullptr || d_in == nullptr || d_out == nullptr || (d_jobs == nullptr && nof_jobs > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (ofdm_split_factor(plan->dft_size) != 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "job lists do not run the split DFT sizes (%u points)", plan->dft_size);
  }
  if (nof_jobs == 0) {
    return SRSGPU_OK;
  }
  const auto* jobs = reinterpret_cast<const ofdm_job*>(d_jobs);
  if (plan->inverse) {
    launch_ofdm(true, plan->dft_size, jobs, static_cast<int>(nof_jobs), plan->nsc, 0, plan->ctx->d_ofdm_twiddles,
                static_cast<const uint32_t*>(d_in), nullptr, nullptr, static_cast<float*>(d_out), nullptr,
                static_cast<hipStream_t>(stream));
  } else {
    launch_ofdm(false, plan->dft_size, jobs, static_cast<int>(nof_jobs), plan->nsc, plan->window_off,
                plan->ctx->d_ofdm_twiddles, nullptr, static_cast<uint32_t*>(d_out), static_cast<const float*>(d_in),
                nullptr, nullptr, static_cast<hipStream_t>(stream));
  }
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

int srsgpu_ofdm_jobs_execute_direct(const srsgpu_ofdm_plan*       plan,
                                    const srsgpu_ofdm_direct_job* d_jobs,
                                    uint32_t                      nof_jobs,
                                    void*                         stream)
{
  if (plan == nullptr || (d_jobs == nullptr && nof_jobs > 0)) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument");
  }
  if (ofdm_split_factor(plan->dft_size) != 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "job lists do not run the split DFT sizes (%u points)", plan->dft_size);
  }
  if (!launch_ofdm_direct(plan->inverse, plan->dft_size, d_jobs, static_cast<int>(nof_jobs), plan->nsc,
                          plan->inverse ? 0u : plan->window_off, plan->ctx->d_ofdm_twiddles,
                          static_cast<hipStream_t>(stream))) {
    return fail(SRSGPU_ERR_INVALID_ARG, "unsupported DFT size %u", plan->dft_size);
  }
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

uint64_t srsgpu_ofdm_plan_nof_grid_words(const srsgpu_ofdm_plan* plan)
{
  return plan == nullptr ? 0 : plan->grid_words;
}

uint64_t srsgpu_ofdm_plan_nof_samples(const srsgpu_ofdm_plan* plan)
{
  return (plan == nullptr || plan->offsets.empty()) ? 0 : plan->offsets.back();
}

uint64_t srsgpu_ofdm_plan_sample_offset(const srsgpu_ofdm_plan* plan, uint32_t grid, uint32_t port)
{
  if (plan == nullptr || port >= plan->nof_ports) {
    return 0;
  }
  const size_t i = static_cast<size_t>(grid) * plan->nof_ports + port;
  return i < plan->offsets.size() ? plan->offsets[i] : 0;
}

int srsgpu_ofdm_modulator_plan_execute(const srsgpu_ofdm_plan* plan,
                                       const uint32_t*         d_grids,
                                       float*                  d_samples,
                                       void*                   stream)
{
  if (plan == nullptr || d_grids == nullptr || d_samples == nullptr || !plan->inverse) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument or not a modulator plan");
  }
  launch_ofdm(true, plan->dft_size, plan->d_jobs, plan->nof_jobs, plan->nsc, 0, plan->ctx->d_ofdm_twiddles, d_grids,
              nullptr, nullptr, d_samples, plan->d_scratch, static_cast<hipStream_t>(stream));
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

int srsgpu_ofdm_modulator_plan_execute_twin(const srsgpu_ofdm_plan* plan,
                                            const uint32_t*         d_grids,
                                            const uint32_t*         d_twin,
                                            float*                  d_samples,
                                            void*                   stream)
{
  if (plan == nullptr || d_grids == nullptr || d_twin == nullptr || d_samples == nullptr || !plan->inverse) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument or not a modulator plan");
  }
  if (ofdm_split_factor(plan->dft_size) != 0) {
    return fail(SRSGPU_ERR_INVALID_ARG, "no twin grid for the split DFT size %u", plan->dft_size);
  }
  launch_ofdm(true, plan->dft_size, plan->d_jobs, plan->nof_jobs, plan->nsc, 0, plan->ctx->d_ofdm_twiddles, d_grids,
              nullptr, nullptr, d_samples, plan->d_scratch, static_cast<hipStream_t>(stream), d_twin);
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

int srsgpu_ofdm_demodulator_plan_execute(const srsgpu_ofdm_plan* plan,
                                         const float*            d_samples,
                                         uint32_t*               d_grids,
                                         void*                   stream)
{
  if (plan == nullptr || d_grids == nullptr || d_samples == nullptr || plan->inverse) {
    return fail(SRSGPU_ERR_INVALID_ARG, "null argument or not a demodulator plan");
  }
  launch_ofdm(false, plan->dft_size, plan->d_jobs, plan->nof_jobs, plan->nsc, plan->window_off,
              plan->ctx->d_ofdm_twiddles, nullptr, d_grids, d_samples, nullptr, plan->d_scratch,
              static_cast<hipStream_t>(stream));
  HIP_TRY(hipGetLastError());
  return SRSGPU_OK;
}

void srsgpu_ofdm_plan_destroy(srsgpu_ofdm_plan* plan)
{
  if (plan == nullptr) {
    return;
  }
  if (plan->d_jobs != nullptr) {
    (void)hipFree(plan->d_jobs);
  }
  if (plan->d_scratch != nullptr) {
    (void)hipFree(plan->d_scratch);
  }
  delete plan;
}

} // extern "C"
