// PUSCH DM-RS channel estimator on gfx950: per (transmission, rx port, DM-RS CDM group) one wavefront computes the
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
// One wavefront per job (a UE's allocation is a few RBs: tens of pilots) keeps the many small jobs of a slot batch
// resident together (dynamic LDS sized by the plan's largest job). The DM-RS sequence words of every DM-RS symbol are
// staged in LDS once (the plan's resident sequence words, filled at plan creation by gold_fill_kernel); the edge regression of the virtual pilots runs on
// the lanes (one 32-lane half per band edge, unwrap as a prefix sum); reductions are wave shuffles. HBM traffic per job:
// the D DM-RS symbols' pilots of one port (read twice: the second pass, for the noise residual, hits L2) and 4 B per
// estimated RE per layer (the dominant term).
#include "gold_device.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {

constexpr int CHEST_THREADS = 64;  // one wavefront
constexpr int CHEST_VP      = 12;  // MAX_V_PILOTS

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

/// Sum over the wavefront (every lane gets the result).
__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v += __shfl_xor(v, o);
  }
  return v;
}

/// Sum over a 32-lane half of the wavefront.
__device__ __forceinline__ float half_sum(float v)
{
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    v += __shfl_xor(v, o, 32);
  }
  return v;
}

/// Layout of the dynamic LDS of a job (sizes from the plan's largest job).
struct chest_lds {
  cpx*      E;     ///< [2][N + 2 CHEST_VP] enlarged LSE per layer of the group (zero outside the filled span)
  cpx*      F;     ///< [2][N] smoothed pilots
  uint32_t* seq;   ///< [D][W] DM-RS sequence words (MSB first) per DM-RS symbol
  float*    taps;  ///< [32]
};

/// DM-RS QPSK symbol i of DM-RS symbol s from the staged sequence words (amplitude 1/sqrt(2)).
__device__ __forceinline__ cpx pilot(const uint32_t* seq, int W, int s, uint32_t n0, int i)
{
  const uint32_t n    = 2 * static_cast<uint32_t>(i) + (n0 & 31u);  // bit index relative to the first staged word
  const uint32_t word = seq[s * W + (n >> 5)];
  const uint32_t sh   = 31u - (n & 31u);  // even n: both bits in the same word
  const float    a    = 0.70710678f;
  return {((word >> sh) & 1u) ? -a : a, ((word >> (sh - 1)) & 1u) ? -a : a};
}

/// compute_v_pilots on the lanes: lanes 0..nv-1 of the first half extrapolate the band start from E[VP .. VP+nv),
/// lanes 32..32+nv-1 the band end from E[VP+N-nv .. VP+N): linear regression of |p| and the unwrapped arg over
/// x = 0..nv-1, evaluated at x = -nv..-1 (start) or nv..2nv-1 (end).
__device__ __forceinline__ void virtual_pilots(cpx* E, int N, int nv)
{
  const int   lane = static_cast<int>(threadIdx.x);
  const int   side = lane >> 5;
  const int   j    = lane & 31;
  const bool  act  = j < nv;
  const cpx   b    = act ? E[CHEST_VP + (side ? N - nv : 0) + j] : cpx{1.f, 0.f};
  const float ab   = act ? sqrtf(b.x * b.x + b.y * b.y) : 0.f;
  const float a    = atan2f(b.y, b.x);
  // Unwrap: arg_j + 2 pi c_j with c_j = sum_{m <= j} rint((a_{m-1} - a_m) / 2 pi) (prefix sum within the half).
  const float twopi = 6.28318531f;
  const float prev  = __shfl_up(a, 1, 32);
  float       c     = (j > 0 && act) ? rintf((prev - a) / twopi) : 0.f;
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    const float t = __shfl_up(c, o, 32);
    c += (j >= o) ? t : 0.f;
  }
  const float ar        = act ? a + twopi * c : 0.f;
  const float n         = static_cast<float>(nv);
  const float mean_x    = static_cast<float>(nv * (nv - 1)) / 2.0f / n;
  const float norm_x_sq = static_cast<float>((nv - 1) * nv * (2 * nv - 1)) / 6.0f;
  const float mab       = half_sum(ab) / n;
  const float mar       = half_sum(ar) / n;
  const float dab       = half_sum(ab * static_cast<float>(j));
  const float dar       = half_sum(ar * static_cast<float>(j));
  const float den       = norm_x_sq - n * mean_x * mean_x;
  const float s_abs     = (dab - mean_x * mab * n) / den;
  const float i_abs     = mab - s_abs * mean_x;
  const float s_arg     = (dar - mean_x * mar * n) / den;
  const float i_arg     = mar - s_arg * mean_x;
  if (act) {
    const float xv  = static_cast<float>(j + (side ? nv : -nv));
    const float rho = s_abs * xv + i_abs;
    const float ph  = s_arg * xv + i_arg + (rho > 0.f ? 0.f : 3.14159265f);
    float       sn, cs;
    sincosf(ph, &sn, &cs);
    E[(side ? CHEST_VP + N : CHEST_VP - nv) + j] = {fabsf(rho) * cs, fabsf(rho) * sn};
  }
}

__global__ __launch_bounds__(CHEST_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void pusch_chest_kernel(const chest_job* __restrict__ jobs,
                                                                    int max_pilots,
                                                                    int max_dmrs,
                                                                    int max_words,
                                                                    const uint32_t* __restrict__ grids,
                                                                    uint32_t* __restrict__ ce,
                                                                    float* __restrict__ noise_var,
                                                                    float* __restrict__ metrics,
                                                                    const uint32_t* __restrict__ gseq)
{
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const int  EN = max_pilots + 2 * CHEST_VP;
  chest_lds  L;
  L.E    = reinterpret_cast<cpx*>(lds_raw);
  L.F    = L.E + 2 * EN;
  L.seq  = reinterpret_cast<uint32_t*>(L.F + 2 * max_pilots);
  L.taps = reinterpret_cast<float*>(L.seq + max_dmrs * max_words);
  (void)max_dmrs;

  const chest_job& jb     = jobs[blockIdx.x];
  const int        lane   = static_cast<int>(threadIdx.x);
  const int        N      = jb.nof_pilots;
  const int        GL     = jb.group_layers;
  const int        D      = jb.nof_dmrs;
  const float      beta   = jb.beta;
  const int        per_rb = jb.pilots_per_rb;
  const uint32_t   n0     = 2 * jb.seq_offset;  // first sequence bit of the allocation
  const uint32_t   w0     = n0 >> 5;
  const int        W      = max_words;
  cpx* const       E0     = L.E;
  cpx* const       E1     = L.E + EN;

  // Stage: zeroed enlarged buffers, taps, the sequence words of every DM-RS symbol.
  for (int i = lane; i < 2 * EN; i += CHEST_THREADS) {
    L.E[i] = {0.f, 0.f};
  }
  if (lane < 32) {
    L.taps[lane] = jb.taps[lane];
  }
  const int nwords = static_cast<int>(((n0 & 31u) + 2u * static_cast<uint32_t>(N) + 31u) >> 5);
  for (int s = 0; s < D; ++s) {  // the plan's resident sequence words (gold_fill_kernel at plan creation)
    for (int wl = lane; wl < nwords; wl += CHEST_THREADS) {
      L.seq[s * W + wl] = gseq[jb.gseq_base + static_cast<uint32_t>(s * nwords + wl)];
    }
  }
  __syncthreads();

  // Pass 1: LSE summed over the DM-RS symbols, EPRE.
  float epre_acc = 0.f;
  for (int i = lane; i < N; i += CHEST_THREADS) {
    const int      rb = i / per_rb;
    const uint32_t k  = static_cast<uint32_t>(rb * 12 + ((jb.pattern >> (4 * (i - rb * per_rb))) & 15u));
    cpx            z  = {0.f, 0.f};
    for (int s = 0; s < D; ++s) {
      const cpx y = bf16c(grids[jb.grid_base + jb.dmrs_symbols[s] * jb.nsc + k]);
      const cpx p = pilot(L.seq, W, s, n0, i);
      z.x += y.x * p.x + y.y * p.y;  // y conj(p)
      z.y += y.y * p.x - y.x * p.y;
      epre_acc += y.x * y.x + y.y * y.y;
    }
    E0[CHEST_VP + i] = z;
  }
  __syncthreads();
  // Remove the cover code of a two-layer group (pairs of adjacent pilots), then scale by 1 / (beta D).
  const float scale = 1.0f / beta / static_cast<float>(D);
  if (GL == 2) {
    for (int j = lane; j < N / 2; j += CHEST_THREADS) {
      const cpx a  = E0[CHEST_VP + 2 * j], b = E0[CHEST_VP + 2 * j + 1];
      const cpx h0 = {(a.x + b.x) * 0.5f * scale, (a.y + b.y) * 0.5f * scale};
      const cpx h1 = {(a.x - b.x) * 0.5f * scale, (a.y - b.y) * 0.5f * scale};
      E0[CHEST_VP + 2 * j] = E0[CHEST_VP + 2 * j + 1] = h0;
      E1[CHEST_VP + 2 * j] = E1[CHEST_VP + 2 * j + 1] = h1;
    }
  } else {
    for (int i = lane; i < N; i += CHEST_THREADS) {
      E0[CHEST_VP + i] = {E0[CHEST_VP + i].x * scale, E0[CHEST_VP + i].y * scale};
    }
  }
  __syncthreads();

  // Frequency-domain smoothing.
  const int nt = jb.ntaps;
  const int c  = nt / 2;
  for (int ly = 0; ly < GL; ++ly) {
    cpx* E = ly ? E1 : E0;
    cpx* F = L.F + ly * max_pilots;
    if (jb.fd == CHEST_FD_FILTER) {
      const int nv = jb.nof_v_pilots;
      virtual_pilots(E, N, nv);
      __syncthreads();
      for (int i = lane; i < N; i += CHEST_THREADS) {
        cpx acc = {0.f, 0.f};
        for (int j = 0; j < nt; ++j) {
          const int e = CHEST_VP + i - c + j;  // symmetric taps: correlation == convolution
          if (e >= CHEST_VP - nv && e < CHEST_VP + N + nv) {
            acc.x += L.taps[j] * E[e].x;
            acc.y += L.taps[j] * E[e].y;
          }
        }
        F[i] = acc;
      }
    } else if (jb.fd == CHEST_FD_MEAN) {
      float sx = 0.f, sy = 0.f;
      for (int i = lane; i < N; i += CHEST_THREADS) {
        sx += E[CHEST_VP + i].x;
        sy += E[CHEST_VP + i].y;
      }
      sx = wave_sum(sx) / static_cast<float>(N);
      sy = wave_sum(sy) / static_cast<float>(N);
      for (int i = lane; i < N; i += CHEST_THREADS) {
        F[i] = {sx, sy};
      }
    } else {
      for (int i = lane; i < N; i += CHEST_THREADS) {
        F[i] = E[CHEST_VP + i];
      }
    }
  }
  __syncthreads();

  // Pass 2: RSRP of layer 0 and the noise residual (group 0 only).
  const cpx* F0 = L.F;
  const cpx* F1 = L.F + max_pilots;
  float      rsrp_acc = 0.f, noise_acc = 0.f;
  for (int i = lane; i < N; i += CHEST_THREADS) {
    const cpx f0 = F0[i];
    rsrp_acc += f0.x * f0.x + f0.y * f0.y;
    if (jb.group == 0) {
      cpx h = f0;
      if (GL == 2) {  // layer 1 carries w_f = -1 on odd pilots
        const cpx  f1 = F1[i];
        const bool od = (i & 1) != 0;
        h             = {f0.x + (od ? -f1.x : f1.x), f0.y + (od ? -f1.y : f1.y)};
      }
      const int      rb = i / per_rb;
      const uint32_t k  = static_cast<uint32_t>(rb * 12 + ((jb.pattern >> (4 * (i - rb * per_rb))) & 15u));
      for (int s = 0; s < D; ++s) {
        const cpx   y  = bf16c(grids[jb.grid_base + jb.dmrs_symbols[s] * jb.nsc + k]);
        const cpx   p  = pilot(L.seq, W, s, n0, i);
        const cpx   q  = {beta * (h.x * p.x - h.y * p.y), beta * (h.x * p.y + h.y * p.x)};  // beta h p
        const float ex = y.x - q.x, ey = y.y - q.y;
        noise_acc += ex * ex + ey * ey;
      }
    }
  }
  const float nof_pilots = static_cast<float>(N * D);
  const float epre       = wave_sum(epre_acc) / nof_pilots;
  const float rsrp       = wave_sum(rsrp_acc) * beta * beta / static_cast<float>(N);
  const float noise_sum  = wave_sum(noise_acc);
  if (lane == 0 && jb.group == 0) {
    const float nv           = fmaxf(rsrp / 1e10f, noise_sum / (nof_pilots - 1.f));
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
  for (int k = lane; k < nre; k += CHEST_THREADS) {
    for (int ly = 0; ly < GL; ++ly) {
      const cpx* F = L.F + ly * max_pilots;
      cpx        v;
      if (k <= offset) {
        v = F[0];
      } else if (k >= last) {
        v = F[N - 1];
      } else {
        const int   i = (k - offset) / stride;
        const float w = static_cast<float>((k - offset) - i * stride) / static_cast<float>(stride);
        const cpx   a = F[i], b = F[i + 1];
        v             = {(b.x - a.x) * w + a.x, (b.y - a.y) * w + a.y};
      }
      const uint32_t u   = to_bf16c(v);
      uint32_t*      dst = ce + jb.ce_base + ly * jb.ce_layer_stride + static_cast<uint32_t>(k);
      for (int l = jb.first_symbol; l < jb.first_symbol + jb.nof_symbols; ++l) {
        dst[l * jb.nsc] = u;
      }
    }
  }
}

} // namespace

size_t pusch_chest_lds_bytes(int max_pilots, int max_dmrs, int max_words)
{
  return (2 * static_cast<size_t>(max_pilots + 2 * CHEST_VP) + 2 * static_cast<size_t>(max_pilots)) * sizeof(cpx) +
         static_cast<size_t>(max_dmrs) * static_cast<size_t>(max_words) * 4 + 32 * 4;
}

void launch_pusch_chest(const chest_job* d_jobs,
                        int              nof_jobs,
                        int              max_pilots,
                        int              max_dmrs,
                        int              max_words,
                        const uint32_t*  d_grids,
                        uint32_t*        d_ce,
                        float*           d_noise_var,
                        float*           d_metrics,
                        const uint32_t*  d_seq,
                        hipStream_t      stream)
{
  if (nof_jobs <= 0) {
    return;
  }
  const size_t lds = pusch_chest_lds_bytes(max_pilots, max_dmrs, max_words);
  hipLaunchKernelGGL(pusch_chest_kernel, dim3(static_cast<unsigned>(nof_jobs)), dim3(CHEST_THREADS),
                     static_cast<unsigned>(lds), stream, d_jobs, max_pilots, max_dmrs, max_words, d_grids, d_ce,
                     d_noise_var, d_metrics, d_seq);
}

} // namespace srsgpu
