// PUSCH DM-RS channel estimator on gfx950: per (transmission, rx port, DM-RS CDM group) one workgroup computes the
// least-squares pilot estimates averaged over the DM-RS symbols, the raised-cosine frequency-domain smoothing with
// virtual edge pilots, RSRP / EPRE / noise variance, and writes the linearly interpolated estimate of every RE of every
// allocated symbol (bf16) into the slot's channel-estimate buffer.
//
// Reference (behaviour, not code): lib/phy/upper/signal_processors/dmrs_pusch_estimator_impl.cpp:69 (DM-RS sequence,
// c_init per symbol), port_channel_estimator_average_impl.cpp:154 (compute_hop: LSE, "average" time strategy, FD
// smoothing, RSRP / EPRE, interpolation; :422 noise; :103 bounds), port_channel_estimator_helpers.cpp:203 (filter,
// virtual pilots :307), support/interpolator/interpolator_linear_impl.cpp:29.
//
// The open-source reference estimates one layer (port 1000). Two layers of a CDM group (ports 1000/1001, 1002/1003)
// are an extension: the frequency cover code w_f = (+1, -1) is removed by combining the LSEs of adjacent pilot pairs
// (the channel is taken as flat over the pair), then each layer is smoothed and interpolated like layer 0. The noise
// variance comes from CDM group 0's residual with every layer of the group subtracted.
//
// Sizes: up to 275 RB x 6 pilots per symbol; 256 threads; the pilots' LSEs live in LDS with 12 virtual-pilot slots on
// each side. HBM traffic per workgroup: the D DM-RS symbols' pilots of one port (read twice: the second pass, for the
// noise residual, hits L2) and 4 B per estimated RE per layer (the dominant term).
#include "gold_device.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {

constexpr int CHEST_THREADS    = 256;
constexpr int CHEST_MAX_PILOTS = 275 * 6;
constexpr int CHEST_VP         = 12;  // MAX_V_PILOTS
constexpr int CHEST_E          = CHEST_MAX_PILOTS + 2 * CHEST_VP;

struct cpx {
  float x, y;
};
__device__ __forceinline__ cpx bf16c(uint32_t u)
{
  return {__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
__device__ __forceinline__ uint32_t bf16_bits(float v)
{
  const uint32_t u = __float_as_uint(v);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ uint32_t to_bf16c(cpx v)
{
  return bf16_bits(v.x) | (bf16_bits(v.y) << 16);
}

/// Sum over the workgroup (every thread gets the result).
__device__ __forceinline__ float block_sum(float v, float* scratch)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v += __shfl_xor(v, o);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    scratch[threadIdx.x / 64] = v;
  }
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < CHEST_THREADS / 64; ++w) {
    s += scratch[w];
  }
  return s;
}

/// DM-RS QPSK symbol m of the sequence of initial state c_init (amplitude 1/sqrt(2)): bits c(2m), c(2m + 1).
__device__ __forceinline__ cpx dmrs_symbol(uint32_t c_init,
                                           uint32_t m,
                                           const uint32_t* __restrict__ x1,
                                           const uint32_t* __restrict__ x2_jump,
                                           const uint32_t* __restrict__ x2_lane)
{
  const uint32_t n    = 2 * m;
  const uint32_t w    = n >> 5;
  const uint32_t word = gold_word(c_init, w, w >> 6, x1, x2_jump, x2_lane);
  const uint32_t sh   = 31u - (n & 31u);  // MSB first; n even: both bits in this word
  const float    a    = 0.70710678f;
  return {((word >> sh) & 1u) ? -a : a, ((word >> (sh - 1)) & 1u) ? -a : a};
}

/// Linear-regression extrapolation of nv virtual pilots (compute_v_pilots): |p| and the unwrapped arg of the base
/// pilots over x = 0..nv-1, evaluated at x = -nv..-1 (start) or nv..2nv-1 (end). One thread.
__device__ void virtual_pilots(const cpx* base, int nv, bool is_start, cpx* out)
{
  float ab[CHEST_VP], ar[CHEST_VP];
  float prev = 0.f;
  for (int i = 0; i < nv; ++i) {
    ab[i]   = sqrtf(base[i].x * base[i].x + base[i].y * base[i].y);
    float a = atan2f(base[i].y, base[i].x);
    if (i > 0) {  // unwrap: keep |a - prev| <= pi
      const float twopi = 6.28318531f;
      a += twopi * rintf((prev - a) / twopi);
    }
    ar[i] = a;
    prev  = a;
  }
  const float n         = static_cast<float>(nv);
  const float mean_x    = static_cast<float>(nv * (nv - 1)) / 2.0f / n;
  const float norm_x_sq = static_cast<float>((nv - 1) * nv * (2 * nv - 1)) / 6.0f;
  float       mab = 0.f, mar = 0.f, dab = 0.f, dar = 0.f;
  for (int i = 0; i < nv; ++i) {
    mab += ab[i];
    mar += ar[i];
    dab += ab[i] * static_cast<float>(i);
    dar += ar[i] * static_cast<float>(i);
  }
  mab /= n;
  mar /= n;
  const float den   = norm_x_sq - n * mean_x * mean_x;
  const float s_abs = (dab - mean_x * mab * n) / den;
  const float i_abs = mab - s_abs * mean_x;
  const float s_arg = (dar - mean_x * mar * n) / den;
  const float i_arg = mar - s_arg * mean_x;
  for (int i = 0; i < nv; ++i) {
    const float xv  = static_cast<float>(i + (is_start ? -nv : nv));
    const float rho = s_abs * xv + i_abs;
    const float ph  = s_arg * xv + i_arg + (rho > 0.f ? 0.f : 3.14159265f);
    float       s, c;
    sincosf(ph, &s, &c);
    out[i] = {fabsf(rho) * c, fabsf(rho) * s};
  }
}

__global__ __launch_bounds__(CHEST_THREADS) void pusch_chest_kernel(const chest_job* __restrict__ jobs,
                                                                    const uint32_t* __restrict__ grids,
                                                                    uint32_t* __restrict__ ce,
                                                                    float* __restrict__ noise_var,
                                                                    float* __restrict__ metrics,
                                                                    const uint32_t* __restrict__ x1,
                                                                    const uint32_t* __restrict__ x2_jump,
                                                                    const uint32_t* __restrict__ x2_lane)
{
  __shared__ cpx   E[2][CHEST_E];             // enlarged LSE per layer of the group (zero outside the span)
  __shared__ cpx   F[2][CHEST_MAX_PILOTS];    // smoothed pilots
  __shared__ float taps[32];
  __shared__ float scratch[CHEST_THREADS / 64];

  const chest_job& jb  = jobs[blockIdx.x];
  const int        tid = static_cast<int>(threadIdx.x);
  const int        N   = jb.nof_pilots;       // pilots per DM-RS symbol
  const int        GL  = jb.group_layers;     // layers of this CDM group (1 or 2)
  const float      beta = jb.beta;
  const int        per_rb = jb.pilots_per_rb;

  for (int i = tid; i < 2 * CHEST_E; i += CHEST_THREADS) {
    (&E[0][0])[i] = {0.f, 0.f};
  }
  if (tid < 32) {
    taps[tid] = jb.taps[tid];
  }
  __syncthreads();

  // Pass 1: LSE summed over the DM-RS symbols, EPRE.
  float epre_acc = 0.f;
  for (int i = tid; i < N; i += CHEST_THREADS) {
    const int      rb = i / per_rb;
    const uint32_t k  = static_cast<uint32_t>(rb * 12 + ((jb.pattern >> (4 * (i - rb * per_rb))) & 15u));
    cpx            z  = {0.f, 0.f};
    for (int s = 0; s < jb.nof_dmrs; ++s) {
      const uint32_t l = jb.dmrs_symbols[s];
      const cpx      y = bf16c(grids[jb.grid_base + l * jb.nsc + k]);
      const cpx      p = dmrs_symbol(jb.c_init[s], jb.seq_offset + static_cast<uint32_t>(i), x1, x2_jump, x2_lane);
      z.x += y.x * p.x + y.y * p.y;  // y conj(p)
      z.y += y.y * p.x - y.x * p.y;
      epre_acc += y.x * y.x + y.y * y.y;
    }
    E[0][CHEST_VP + i] = z;
  }
  __syncthreads();
  // Remove the cover code of a two-layer group (pairs of adjacent pilots), then scale by 1 / (beta D).
  const float scale = 1.0f / beta / static_cast<float>(jb.nof_dmrs);
  if (GL == 2) {
    // One thread per pilot pair (N is even): h0 = (z_2j + z_2j+1) / 2, h1 = (z_2j - z_2j+1) / 2 on both pilots.
    for (int j = tid; j < N / 2; j += CHEST_THREADS) {
      const cpx a = E[0][CHEST_VP + 2 * j], b = E[0][CHEST_VP + 2 * j + 1];
      const cpx h0 = {(a.x + b.x) * 0.5f * scale, (a.y + b.y) * 0.5f * scale};
      const cpx h1 = {(a.x - b.x) * 0.5f * scale, (a.y - b.y) * 0.5f * scale};
      E[0][CHEST_VP + 2 * j] = E[0][CHEST_VP + 2 * j + 1] = h0;
      E[1][CHEST_VP + 2 * j] = E[1][CHEST_VP + 2 * j + 1] = h1;
    }
  } else {
    for (int i = tid; i < N; i += CHEST_THREADS) {
      E[0][CHEST_VP + i] = {E[0][CHEST_VP + i].x * scale, E[0][CHEST_VP + i].y * scale};
    }
  }
  __syncthreads();

  // Frequency-domain smoothing.
  const int nt = jb.ntaps;
  const int c  = nt / 2;
  if (jb.fd == CHEST_FD_FILTER) {
    const int nv = jb.nof_v_pilots;
    if (tid < 2 * GL) {
      const int ly = tid >> 1;
      if ((tid & 1) == 0) {
        virtual_pilots(&E[ly][CHEST_VP], nv, true, &E[ly][CHEST_VP - nv]);
      } else {
        virtual_pilots(&E[ly][CHEST_VP + N - nv], nv, false, &E[ly][CHEST_VP + N]);
      }
    }
    __syncthreads();
    for (int i = tid; i < N; i += CHEST_THREADS) {
      for (int ly = 0; ly < GL; ++ly) {
        cpx acc = {0.f, 0.f};
        for (int j = 0; j < nt; ++j) {
          const int e = CHEST_VP + i - c + j;  // symmetric taps: correlation == convolution
          if (e >= CHEST_VP - nv && e < CHEST_VP + N + nv) {
            acc.x += taps[j] * E[ly][e].x;
            acc.y += taps[j] * E[ly][e].y;
          }
        }
        F[ly][i] = acc;
      }
    }
  } else if (jb.fd == CHEST_FD_MEAN) {
    for (int ly = 0; ly < GL; ++ly) {
      float sx = 0.f, sy = 0.f;
      for (int i = tid; i < N; i += CHEST_THREADS) {
        sx += E[ly][CHEST_VP + i].x;
        sy += E[ly][CHEST_VP + i].y;
      }
      sx = block_sum(sx, scratch) / static_cast<float>(N);
      sy = block_sum(sy, scratch) / static_cast<float>(N);
      for (int i = tid; i < N; i += CHEST_THREADS) {
        F[ly][i] = {sx, sy};
      }
    }
  } else {
    for (int i = tid; i < N; i += CHEST_THREADS) {
      for (int ly = 0; ly < GL; ++ly) {
        F[ly][i] = E[ly][CHEST_VP + i];
      }
    }
  }
  __syncthreads();

  // Pass 2: RSRP of layer 0 and the noise residual (group 0 only).
  float rsrp_acc = 0.f, noise_acc = 0.f;
  for (int i = tid; i < N; i += CHEST_THREADS) {
    const cpx f0 = F[0][i];
    rsrp_acc += f0.x * f0.x + f0.y * f0.y;
    if (jb.group == 0) {
      cpx h = f0;
      if (GL == 2) {  // layer 1 carries w_f = -1 on odd pilots
        const cpx  f1 = F[1][i];
        const bool od = (i & 1) != 0;
        h             = {f0.x + (od ? -f1.x : f1.x), f0.y + (od ? -f1.y : f1.y)};
      }
      const int      rb = i / per_rb;
      const uint32_t k  = static_cast<uint32_t>(rb * 12 + ((jb.pattern >> (4 * (i - rb * per_rb))) & 15u));
      for (int s = 0; s < jb.nof_dmrs; ++s) {
        const cpx y = bf16c(grids[jb.grid_base + jb.dmrs_symbols[s] * jb.nsc + k]);
        const cpx p = dmrs_symbol(jb.c_init[s], jb.seq_offset + static_cast<uint32_t>(i), x1, x2_jump, x2_lane);
        // predicted = beta h p
        const cpx q  = {beta * (h.x * p.x - h.y * p.y), beta * (h.x * p.y + h.y * p.x)};
        const float ex = y.x - q.x, ey = y.y - q.y;
        noise_acc += ex * ex + ey * ey;
      }
    }
  }
  const float nof_pilots = static_cast<float>(N * jb.nof_dmrs);
  const float epre       = block_sum(epre_acc, scratch) / nof_pilots;
  const float rsrp       = block_sum(rsrp_acc, scratch) * beta * beta / static_cast<float>(N);
  const float noise_sum  = block_sum(noise_acc, scratch);
  if (tid == 0 && jb.group == 0) {
    const float nv    = fmaxf(rsrp / 1e10f, noise_sum / (nof_pilots - 1.f));
    noise_var[jb.noise_slot] = nv;
    if (metrics != nullptr) {
      float* m = metrics + 4 * jb.noise_slot;
      m[0]     = rsrp;
      m[1]     = epre;
      m[2]     = nv;
      m[3]     = (nv != 0.f) ? rsrp / beta / beta / nv : 1000.f;
    }
  }

  // Interpolation to every RE of the allocation, the same estimate for every symbol ("average" strategy).
  const int nre    = jb.nof_rb * 12;
  const int offset = jb.interp_offset;
  const int stride = jb.interp_stride;
  const int last   = offset + (N - 1) * stride;
  for (int k = tid; k < nre; k += CHEST_THREADS) {
    for (int ly = 0; ly < GL; ++ly) {
      cpx v;
      if (k <= offset) {
        v = F[ly][0];
      } else if (k >= last) {
        v = F[ly][N - 1];
      } else {
        const int   i  = (k - offset) / stride;
        const float w  = static_cast<float>((k - offset) - i * stride) / static_cast<float>(stride);
        const cpx   a  = F[ly][i], b = F[ly][i + 1];
        v              = {(b.x - a.x) * w + a.x, (b.y - a.y) * w + a.y};
      }
      const uint32_t u    = to_bf16c(v);
      uint32_t*      dst  = ce + jb.ce_base + ly * jb.ce_layer_stride + static_cast<uint32_t>(k);
      for (int l = jb.first_symbol; l < jb.first_symbol + jb.nof_symbols; ++l) {
        dst[l * jb.nsc] = u;
      }
    }
  }
}

} // namespace

void launch_pusch_chest(const chest_job* d_jobs,
                        int              nof_jobs,
                        const uint32_t*  d_grids,
                        uint32_t*        d_ce,
                        float*           d_noise_var,
                        float*           d_metrics,
                        const uint32_t*  d_x1,
                        const uint32_t*  d_x2_jump,
                        const uint32_t*  d_x2_lane,
                        hipStream_t      stream)
{
  if (nof_jobs <= 0) {
    return;
  }
  hipLaunchKernelGGL(pusch_chest_kernel, dim3(static_cast<unsigned>(nof_jobs)), dim3(CHEST_THREADS), 0, stream, d_jobs,
                     d_grids, d_ce, d_noise_var, d_metrics, d_x1, d_x2_jump, d_x2_lane);
}

} // namespace srsgpu
