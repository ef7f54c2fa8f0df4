// PUSCH demodulator on gfx950: channel equalization + soft demapping + descrambling of every data RE of every PUSCH
// transmission of a batch of slots, straight from the rx grids and channel estimates to the codeword LLR buffer.
//
// Reference (behaviour, not code): lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.cpp:272 (RE order,
// descrambling), equalization/channel_equalizer_generic_impl.cpp:286 (dispatch), equalize_zf_1xn.h:128 (ZF 1 x N),
// equalize_zf_2xn.h:180 (ZF 2 x N), channel_modulation/demodulation_mapper_*.cpp (SIMD arithmetic: safe reciprocal
// noise, near-zero parts, avx2_helpers.h:121 quantisation).
//
// Work decomposition (like the PDSCH modulator): a workgroup owns 8192 codeword LLRs of one transmission (the REs
// whose first LLR falls in them). The four waves first stage the 8192 + 32 descrambling-sequence bits in LDS (Gold
// sequence by GF(2) jumps, gold_device.h). Then every lane takes one RE: it loads the P received values and the L x P
// channel estimates (consecutive lanes read consecutive subcarriers: coalesced 4-byte loads), equalizes, demaps the
// L * Qm LLRs, flips the signs the sequence selects and stages the bytes in LDS; the workgroup finally writes its
// contiguous LLR range with dword stores. HBM-bound: (P + L P) x 4 B in and L Qm B out per RE.
#include "gold_device.h"
#include "srsgpu_internal.h"

#pragma clang fp contract(off)

namespace srsgpu {
namespace {

constexpr int DEMOD_THREADS = 256;
constexpr int DEMOD_OUT_BYTES = MOD_CHUNK_WORDS * 32 + 64;

struct cpx {
  float x, y;
};
__device__ __forceinline__ cpx cmk(float x, float y)
{
  return {x, y};
}
__device__ __forceinline__ cpx bf16c(uint32_t u)
{
  return {__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
__device__ __forceinline__ cpx cmul(cpx a, cpx b)
{
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
/// a * conj(b)
__device__ __forceinline__ cpx cmulc(cpx a, cpx b)
{
  return {a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y};
}
__device__ __forceinline__ cpx cadd(cpx a, cpx b)
{
  return {a.x + b.x, a.y + b.y};
}
__device__ __forceinline__ cpx csub(cpx a, cpx b)
{
  return {a.x - b.x, a.y - b.y};
}
__device__ __forceinline__ cpx cscale(cpx a, float s)
{
  return {a.x * s, a.y * s};
}
__device__ __forceinline__ bool isnormal_f(float v)
{
  return __builtin_isnormal(v);
}

/// SIMD quantizer: v * 120 / range, clipped to +-120, rounded half to even.
__device__ __forceinline__ int quantize(float v, float scale)
{
  float x = v * scale;
  x       = fminf(fmaxf(x, -120.f), 120.f);
  return static_cast<int>(__builtin_rintf(x));  // NaN cannot occur: rcp = 0 for invalid noise
}

/// Soft demapping of one equalized symbol into qm LLRs (stream order: re, im of bit pair 0, then pair 1, ...).
__device__ __forceinline__ void demap(cpx s, float nvar, uint32_t qm, const demap_pair_table* tab, int* llr)
{
  const float rcp = (nvar > 0.f) ? 1.f / nvar : 0.f;
  const float part[2] = {s.x, s.y};
  if (qm == 2) {
    const float g = 2.0f * 1.41421356f;  // 2 * M_SQRT2f32
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      llr[k] = quantize((g * part[k]) * rcp, 120.f / 24.f);
    }
    return;
  }
  if (qm == 4) {
    const float a = 0.316227766f;  // 1 / sqrt(10) in float
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float x   = part[k];
      const float f   = (4.f * a) * x;
      const float l01 = (fabsf(x) > 2.f * a) ? 2.f * f - copysignf(0.8f, x) : f;
      const float l23 = 0.8f - fabsf(f);
      const bool  nz  = fabsf(x) <= 1e-9f;
      llr[k]          = nz ? 0 : quantize(l01 * rcp, 6.f);
      llr[2 + k]      = nz ? 0 : quantize(l23 * rcp, 6.f);
    }
    return;
  }
  const demap_pair_table* t = tab + (qm == 6 ? 0 : 3);
#pragma unroll
  for (uint32_t kb = 0; kb < 4; ++kb) {
    if (kb >= qm / 2) {
      break;
    }
    const demap_pair_table& p = t[kb];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float x   = part[k];
      int         idx = static_cast<int>(floorf(x / p.width)) + static_cast<int>(p.count / 2);
      idx             = min(max(idx, 0), static_cast<int>(p.count) - 1);
      const float l   = (p.slope[idx] * x + p.intercept[idx]) * rcp;
      llr[2 * kb + k] = (fabsf(x) <= 1e-9f) ? 0 : quantize(l, 6.f);
    }
  }
}

/// Unbiased linear MMSE for L layers: A = H^H H + nv I, x = A^-1 H^H y, g_l = 1 - nv [A^-1]_ll,
/// eq_l = x_l / g_l, var_l = nv [A^-1]_ll / g_l (Gauss-Jordan on the Hermitian positive definite A).
template <int L>
__device__ __forceinline__ void equalize_mmse(const cpx* y, const cpx (*h)[4], uint32_t P, float nv, cpx* eq,
                                              float* var)
{
  cpx A[L][L], B[L][L], m[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      cpx s = cmk(0.f, 0.f);
      #pragma unroll
      for (uint32_t p = 0; p < 4; ++p) {  // unrolled: register arrays stay in VGPRs
        if (p >= P) {
          break;
        }
        s = cadd(s, cmulc(h[j][p], h[i][p]));  // conj(h_pi) h_pj
      }
      A[i][j] = s;
      B[i][j] = cmk(i == j ? 1.f : 0.f, 0.f);
    }
    A[i][i].x += nv;
    cpx s = cmk(0.f, 0.f);
    #pragma unroll
    for (uint32_t p = 0; p < 4; ++p) {  // unrolled: register arrays stay in VGPRs
        if (p >= P) {
          break;
        }
      s = cadd(s, cmulc(y[p], h[i][p]));  // conj(h_pi) y_p
    }
    m[i] = s;
  }
#pragma unroll
  for (int c = 0; c < L; ++c) {
    const float d   = A[c][c].x;  // real positive pivot (Hermitian PD)
    const float rcp = 1.f / d;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      A[c][j] = cscale(A[c][j], rcp);
      B[c][j] = cscale(B[c][j], rcp);
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
      if (i != c) {
        const cpx f = A[i][c];
#pragma unroll
        for (int j = 0; j < L; ++j) {
          A[i][j] = csub(A[i][j], cmul(f, A[c][j]));
          B[i][j] = csub(B[i][j], cmul(f, B[c][j]));
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < L; ++i) {
    cpx x = cmk(0.f, 0.f);
#pragma unroll
    for (int j = 0; j < L; ++j) {
      x = cadd(x, cmul(B[i][j], m[j]));
    }
    const float aii = B[i][i].x;
    const float g   = 1.f - nv * aii;
    if (isnormal_f(g) && g > 0.f && isnormal_f(nv * aii)) {
      const float rg = 1.f / g;
      eq[i]          = cscale(x, rg);
      var[i]         = (nv * aii) * rg;
    } else {
      eq[i]  = cmk(0.f, 0.f);
      var[i] = __builtin_inff();
    }
  }
}

__global__ __launch_bounds__(DEMOD_THREADS) void pusch_demodulate_kernel(const demod_desc* __restrict__ descs,
                                                                         const mod_chunk* __restrict__ chunks,
                                                                         const demap_pair_table* __restrict__ tables,
                                                                         const uint32_t* __restrict__ grids,
                                                                         const uint32_t* __restrict__ ce,
                                                                         const float* __restrict__ noise_var,
                                                                         int8_t* __restrict__ llrs,
                                                                         const uint32_t* __restrict__ x1,
                                                                         const uint32_t* __restrict__ x2_jump,
                                                                         const uint32_t* __restrict__ x2_lane)
{
  __shared__ uint32_t         seq[MOD_CHUNK_WORDS + 1];
  __shared__ demap_pair_table tab[DEMAP_TABLES];
  __shared__ int8_t           out[DEMOD_OUT_BYTES];
  const mod_chunk             ch     = chunks[blockIdx.x];
  const demod_desc&           d      = descs[ch.tx];
  const uint32_t              tid    = threadIdx.x;
  const uint32_t              nwords = (d.nof_llrs + 31u) >> 5;
  {
    const uint32_t w = ch.word0 + tid;
    const uint32_t c = __builtin_amdgcn_readfirstlane(w >> 6);  // word0 % 256 == 0: wave-uniform jump
    seq[tid]         = (w < nwords) ? gold_word(d.c_init, w, c, x1, x2_jump, x2_lane) : 0u;
    if (tid == 0) {
      const uint32_t w2      = ch.word0 + MOD_CHUNK_WORDS;
      seq[MOD_CHUNK_WORDS] = (w2 < nwords) ? gold_word(d.c_init, w2, w2 >> 6, x1, x2_jump, x2_lane) : 0u;
    }
    const uint32_t* src = reinterpret_cast<const uint32_t*>(tables);
    uint32_t*       dst = reinterpret_cast<uint32_t*>(tab);
    for (uint32_t i = tid; i < sizeof(tab) / 4; i += DEMOD_THREADS) {
      dst[i] = src[i];
    }
  }
  const uint32_t qm = d.qm, L = d.L, P = d.P, Lq = L * qm;
  float          nv[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    nv[p] = noise_var[4 * d.tx + p];
  }
  float nv_max = nv[0];
#pragma unroll
  for (uint32_t p = 1; p < 4; ++p) {
    nv_max = (p < P) ? fmaxf(nv_max, nv[p]) : nv_max;
  }
  __syncthreads();

  const uint32_t first_llr = ch.re_begin * Lq;  // first LLR the workgroup writes
  for (uint32_t r = ch.re_begin + tid; r < ch.re_end; r += DEMOD_THREADS) {
    // Symbol and subcarrier of the RE.
    uint32_t l = 0;
#pragma unroll
    for (int j = 1; j < 15; ++j) {
      l += (d.sym_cum[j] <= r) ? 1u : 0u;
    }
    const uint32_t k = r - d.sym_cum[l];
    uint32_t       sc;
    if ((d.dmrs_mask >> l) & 1u) {
      const uint32_t nd  = d.nd_dmrs;
      const uint32_t prb = k / nd;
      sc                 = prb * 12u + static_cast<uint32_t>((d.dmrs_lut >> (4u * (k - prb * nd))) & 15u);
    } else {
      sc = k;
    }
    const uint32_t ge = d.grid_base + l * d.nsc + sc;
    const uint32_t ee = d.ce_base + l * d.nsc + sc;
    cpx            y[4], h[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p < static_cast<int>(P)) {
        y[p] = bf16c(grids[ge + p * d.port_stride]);
#pragma unroll
        for (int ly = 0; ly < 4; ++ly) {
          if (ly < static_cast<int>(L)) {
            h[ly][p] = bf16c(ce[ee + ly * d.ce_layer_stride + p * d.port_stride]);
          }
        }
      }
    }
    cpx   eq[4];
    float var[4];
    if (L == 1) {
      // ZF 1 x N (MMSE with one layer is the same, channel_equalizer_generic_impl.cpp:343).
      float ch_mod_sq = 0.f, nvar_acc = 0.f;
      cpx   acc       = cmk(0.f, 0.f);
      #pragma unroll
      for (uint32_t p = 0; p < 4; ++p) {  // unrolled: register arrays stay in VGPRs
        if (p >= P) {
          break;
        }
        const float norm = h[0][p].x * h[0][p].x + h[0][p].y * h[0][p].y;
        if (isnormal_f(norm) && isnormal_f(nv[p]) && nv[p] > 0.f) {
          ch_mod_sq += norm;
          nvar_acc += norm * nv[p];
          acc = cadd(acc, cmulc(y[p], h[0][p]));
        }
      }
      if (isnormal_f(ch_mod_sq) && isnormal_f(nvar_acc)) {
        const float rcp = 1.f / ch_mod_sq;
        eq[0]           = cscale(acc, rcp);
        var[0]          = nvar_acc * rcp * rcp;
      } else {
        eq[0]  = cmk(0.f, 0.f);
        var[0] = __builtin_inff();
      }
    } else if (L == 2 && d.eq == DEMOD_EQ_ZF) {
      // ZF 2 x N with the largest noise variance.
      eq[0] = eq[1] = cmk(0.f, 0.f);
      var[0] = var[1] = __builtin_inff();
      if (isnormal_f(nv_max) && nv_max >= 0.f) {
        float n0 = 0.f, n1 = 0.f;
        cpx   xi = cmk(0.f, 0.f), m0 = cmk(0.f, 0.f), m1 = cmk(0.f, 0.f);
        #pragma unroll
        for (uint32_t p = 0; p < 4; ++p) {  // unrolled: register arrays stay in VGPRs
        if (p >= P) {
          break;
        }
          n0 += h[0][p].x * h[0][p].x + h[0][p].y * h[0][p].y;
          n1 += h[1][p].x * h[1][p].x + h[1][p].y * h[1][p].y;
          xi = cadd(xi, cmulc(h[1][p], h[0][p]));  // conj(h0) h1
          m0 = cadd(m0, cmulc(y[p], h[0][p]));
          m1 = cadd(m1, cmulc(y[p], h[1][p]));
        }
        const float d_pinv = n0 * n1 - (xi.x * xi.x + xi.y * xi.y);
        if (isnormal_f(d_pinv)) {
          const float rcp = 1.f / d_pinv;
          eq[0]           = cscale(csub(cscale(m0, n1), cmul(xi, m1)), rcp);
          eq[1]           = cscale(csub(cscale(m1, n0), cmulc(m0, xi)), rcp);
          var[0]          = nv_max * n1 * rcp;
          var[1]          = nv_max * n0 * rcp;
        }
      }
    } else if (L == 2) {
      equalize_mmse<2>(y, h, P, nv_max, eq, var);
    } else if (L == 3) {
      equalize_mmse<3>(y, h, P, nv_max, eq, var);
    } else {
      equalize_mmse<4>(y, h, P, nv_max, eq, var);
    }

    // Demap, descramble (sequence bits of the RE's LLRs, MSB-first words staged in LDS) and stage the bytes.
    const uint32_t o  = r * Lq - ch.word0 * 32u;
    const uint32_t wi = o >> 5;
    const uint64_t sb = ((static_cast<uint64_t>(seq[wi]) << 32) | seq[wi + 1]) << (o & 31u);
    const uint32_t ob = r * Lq - first_llr;
    for (uint32_t ly = 0; ly < L; ++ly) {
      int v[8];
      demap(eq[ly], var[ly], qm, tab, v);
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        if (j < qm) {
          const uint32_t bit = static_cast<uint32_t>(sb >> (63u - (ly * qm + j))) & 1u;
          out[ob + ly * qm + j] = static_cast<int8_t>(bit ? -v[j] : v[j]);
        }
      }
    }
  }
  __syncthreads();

  // Contiguous LLR range [first_llr, re_end * Lq) of the codeword: bytes up to dword alignment, then dwords.
  const uint32_t n    = (ch.re_end - ch.re_begin) * Lq;
  int8_t*        dst  = llrs + d.llr_offset + first_llr;
  const uint32_t head = min(n, static_cast<uint32_t>((4u - (reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u));
  if (tid < head) {
    dst[tid] = out[tid];
  }
  const uint32_t nw = (n - head) / 4;
  for (uint32_t i = tid; i < nw; i += DEMOD_THREADS) {
    const uint32_t b = head + 4 * i;
    const uint32_t v = static_cast<uint8_t>(out[b]) | (static_cast<uint32_t>(static_cast<uint8_t>(out[b + 1])) << 8) |
                       (static_cast<uint32_t>(static_cast<uint8_t>(out[b + 2])) << 16) |
                       (static_cast<uint32_t>(static_cast<uint8_t>(out[b + 3])) << 24);
    reinterpret_cast<uint32_t*>(dst + head)[i] = v;
  }
  const uint32_t tail0 = head + 4 * nw;
  if (tail0 + tid < n) {
    dst[tail0 + tid] = out[tail0 + tid];
  }
}

} // namespace

void launch_pusch_demodulate(const demod_desc*       d_desc,
                             const mod_chunk*        d_chunks,
                             int                     nof_chunks,
                             const demap_pair_table* d_tables,
                             const uint32_t*         d_grids,
                             const uint32_t*         d_ch_est,
                             const float*            d_noise_var,
                             int8_t*                 d_llrs,
                             const uint32_t*         d_x1,
                             const uint32_t*         d_x2_jump,
                             const uint32_t*         d_x2_lane,
                             hipStream_t             stream)
{
  if (nof_chunks <= 0) {
    return;
  }
  hipLaunchKernelGGL(pusch_demodulate_kernel, dim3(static_cast<unsigned>(nof_chunks)), dim3(DEMOD_THREADS), 0, stream,
                     d_desc, d_chunks, d_tables, d_grids, d_ch_est, d_noise_var, d_llrs, d_x1, d_x2_jump, d_x2_lane);
}

} // namespace srsgpu
