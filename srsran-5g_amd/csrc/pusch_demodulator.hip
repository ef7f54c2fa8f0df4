// PUSCH demodulator on gfx950: channel equalization + soft demapping + descrambling of every data RE of every PUSCH
// transmission of a batch of slots, straight from the rx grids and channel estimates to the codeword LLR buffer.
//
// Reference (behaviour, not code): lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.cpp:272 (RE order,
// descrambling), equalization/channel_equalizer_generic_impl.cpp:286 (dispatch), equalize_zf_1xn.h:128 (ZF 1 x N),
// equalize_zf_2xn.h:180 (ZF 2 x N), channel_modulation/demodulation_mapper_*.cpp (SIMD arithmetic: safe reciprocal
// noise, near-zero parts, avx2_helpers.h:121 quantisation).
//
// Work decomposition (like the PDSCH modulator): a workgroup owns 32768 codeword LLRs of one transmission (the REs
// whose first LLR falls in them). The four waves first stage the 32768 + 32 descrambling-sequence bits in LDS (the plan's
// precomputed Gold sequence words, gold_fill_kernel). Then every lane takes one RE: it loads the P received values and the L x P
// channel estimates (consecutive lanes read consecutive subcarriers: coalesced 4-byte loads), equalizes, demaps the
// L * Qm LLRs, flips the signs the sequence selects and stages the bytes in LDS; the workgroup finally writes its
// contiguous LLR range with dword stores. HBM-bound: (P + L P) x 4 B in and L Qm B out per RE.
#include "gold_device.h"
#include "srsgpu_internal.h"

// Contraction (FMA) is allowed in the equalizer; the demapper keeps the reference's separately rounded mul / add.
#pragma clang fp contract(fast)

namespace srsgpu {
namespace {

constexpr int DEMOD_THREADS = 256;
constexpr int DEMOD_OUT_BYTES = DEMOD_CHUNK_WORDS * 32 + 64;

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

/// Soft demapping of one equalized symbol into QM LLRs (stream order: re, im of bit pair 0, then pair 1, ...),
/// following the SIMD demappers (demodulation_mapper_qam*.cpp, avx2_helpers.h: reciprocal-width interval index,
/// separately rounded slope * x + intercept, per-component near-zero masking).
template <int QM>
__device__ __forceinline__ void demap(cpx s, float nvar, const demap_pair_table* tab, int* llr)
{
#pragma clang fp contract(off)
  const float rcp     = (nvar > 0.f) ? 1.f / nvar : 0.f;
  const float part[2] = {s.x, s.y};
  if constexpr (QM == 2) {
    const float g = 2.0f * 1.41421356f;  // 2 * M_SQRT2f32
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      llr[k] = quantize((g * part[k]) * rcp, 120.f / 24.f);
    }
  } else if constexpr (QM == 4) {
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
  } else {
    // Every bit pair but the last shares its interval width and count (2a, 2^(QM/2) intervals; the last: 4a, half as
    // many — demodulation_mapper_qam64.cpp:49/:62/:75, _qam256.cpp:48/:82/:116/:150; the host asserts it), so the
    // interval index of the first pairs is computed once per component.
    const demap_pair_table* t = tab + (QM == 6 ? 0 : 3);
    constexpr int           NP  = QM / 2;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float x      = part[k];
      const bool  nz     = fabsf(x) <= 1e-9f;
      const int   cnt0   = static_cast<int>(t[0].count);
      const int   idx0   = min(max(static_cast<int>(floorf(x * t[0].inv_width)) + cnt0 / 2, 0), cnt0 - 1);
      const int   cntl   = static_cast<int>(t[NP - 1].count);
      const int   idxl   = min(max(static_cast<int>(floorf(x * t[NP - 1].inv_width)) + cntl / 2, 0), cntl - 1);
#pragma unroll
      for (int kb = 0; kb < NP; ++kb) {
        const int    idx = (kb == NP - 1) ? idxl : idx0;
        const float2 sl  = *reinterpret_cast<const float2*>(t[kb].piece[idx]);
        const float  l   = (sl.x * x + sl.y) * rcp;
        llr[2 * kb + k]  = nz ? 0 : quantize(l, 6.f);
      }
    }
  }
}

template <int L>
__device__ __forceinline__ void equalize_mmse(const cpx* y, const cpx (*h)[4], uint32_t P, float nv, cpx* eq,
                                              float* var)
{
  // Ports p >= P hold zeros (load_re leaves them zero), so the sums run over all four without guards.
  (void)P;
  cpx A[L][L], m[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    float dsum = nv;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      dsum += h[i][p].x * h[i][p].x + h[i][p].y * h[i][p].y;
    }
    A[i][i] = cmk(dsum, 0.f);
#pragma unroll
    for (int j = i + 1; j < L; ++j) {
      cpx s = cmk(0.f, 0.f);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        s = cadd(s, cmulc(h[j][p], h[i][p]));  // conj(h_ip) h_jp
      }
      A[i][j] = s;
    }
    cpx s = cmk(0.f, 0.f);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      s = cadd(s, cmulc(y[p], h[i][p]));  // conj(h_ip) y_p
    }
    m[i] = s;
  }
  // Cholesky: R_ii = sqrt(A_ii - sum_k<i |R_ki|^2), R_ij = (A_ij - sum_k<i conj(R_ki) R_kj) / R_ii.
  cpx   R[L][L];
  float rinv[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    float d = A[i][i].x;
#pragma unroll
    for (int k = 0; k < i; ++k) {
      d -= R[k][i].x * R[k][i].x + R[k][i].y * R[k][i].y;
    }
    rinv[i] = __builtin_amdgcn_rsqf(fmaxf(d, 0.f));  // 1 / R_ii (v_rsq, 1 ulp: the extension has no reference)
#pragma unroll
    for (int j = i + 1; j < L; ++j) {
      cpx s = A[i][j];
#pragma unroll
      for (int k = 0; k < i; ++k) {
        s = csub(s, cmulc(R[k][j], R[k][i]));  // conj(R_ki) R_kj
      }
      R[i][j] = cscale(s, rinv[i]);
    }
  }
  // T = R^-1 (upper triangular): T_ii = 1 / R_ii, T_ij = -(sum_{k=i}^{j-1} T_ik R_kj) / R_jj.
  cpx T[L][L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    T[i][i] = cmk(rinv[i], 0.f);
#pragma unroll
    for (int j = i + 1; j < L; ++j) {
      cpx s = cmul(T[i][i], R[i][j]);
#pragma unroll
      for (int k = i + 1; k < j; ++k) {
        s = cadd(s, cmul(T[i][k], R[k][j]));
      }
      T[i][j] = cscale(s, -rinv[j]);
    }
  }
  // z = T^H m (lower triangular: z_j = sum_{i<=j} conj(T_ij) m_i), x = T z.
  cpx z[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    cpx s = cmk(0.f, 0.f);
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      s = cadd(s, cmulc(m[i], T[i][j]));
    }
    z[j] = s;
  }
#pragma unroll
  for (int i = 0; i < L; ++i) {
    cpx   x   = cmk(0.f, 0.f);
    float aii = 0.f;
#pragma unroll
    for (int j = i; j < L; ++j) {
      x = cadd(x, cmul(T[i][j], z[j]));
      aii += T[i][j].x * T[i][j].x + T[i][j].y * T[i][j].y;
    }
    const float g = 1.f - nv * aii;
    if (isnormal_f(g) && g > 0.f && isnormal_f(nv * aii)) {
      const float rg = __builtin_amdgcn_rcpf(g);
      eq[i]          = cscale(x, rg);
      var[i]         = (nv * aii) * rg;
    } else {
      eq[i]  = cmk(0.f, 0.f);
      var[i] = __builtin_inff();
    }
  }
}

/// Transmission parameters of a workgroup, uniform across it.
struct demod_uniform {
  const demod_desc*       d;
  uint32_t                re_begin, re_end, word0;
  float                   nv[4], nv_max;
  const demap_pair_table* tables;  ///< Global demapper tables (staged into LDS for Qm >= 6).
  const uint32_t*         gseq;    ///< The plan's precomputed descrambling sequences.
  const cpx*              rot;     ///< LDS [14][4 layers][4 ports] CFO rotations (demod_desc::ce_cfo), else null.
};

/// Round-to-nearest-even float -> bf16 pair (adt/bf16.h), the estimator's storage rounding.
__device__ __forceinline__ uint32_t to_bf16c(cpx v)
{
  const uint32_t a = __float_as_uint(v.x), b = __float_as_uint(v.y);
  return ((a + 0x7fffu + ((a >> 16) & 1u)) >> 16) | (((b + 0x7fffu + ((b >> 16) & 1u)) >> 16) << 16);
}

/// Stages the chunk's descrambling words (and the first word of the next chunk) and, for 64/256QAM, the demapper
/// tables in LDS. The caller synchronises.
__device__ __forceinline__ void stage_chunk(const demod_uniform& u, uint32_t* seq, demap_pair_table* tab)
{
  const demod_desc& d      = *u.d;
  const uint32_t    tid    = threadIdx.x;
  const uint32_t    nwords = (d.nof_llrs + 31u) >> 5;
  for (uint32_t j = tid; j < DEMOD_CHUNK_WORDS; j += DEMOD_THREADS) {
    const uint32_t w = u.word0 + j;
    seq[j]           = (w < nwords) ? u.gseq[d.seq_word_offset + w] : 0u;
  }
  if (tid == 0) {
    const uint32_t w2      = u.word0 + DEMOD_CHUNK_WORDS;
    seq[DEMOD_CHUNK_WORDS] = (w2 < nwords) ? u.gseq[d.seq_word_offset + w2] : 0u;
  }
  if (d.qm >= 6) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(u.tables);
    uint32_t*       dst = reinterpret_cast<uint32_t*>(tab);
    for (uint32_t i = tid; i < DEMAP_TABLES * sizeof(demap_pair_table) / 4; i += DEMOD_THREADS) {
      dst[i] = src[i];
    }
  }
}

/// Issues the loads of RE r: the P received values and the L x P channel estimates (raw bf16 pairs).
template <int L>
__device__ __forceinline__ void load_re(const demod_desc& d,
                                        uint32_t          r,
                                        const uint32_t* __restrict__ grids,
                                        const uint32_t* __restrict__ ce,
                                        uint32_t (&yw)[4],
                                        uint32_t (&hw)[L][4],
                                        uint32_t& sym)
{
  // Symbol and subcarrier of the RE.
  uint32_t l = 0;
#pragma unroll
  for (int j = 1; j < 15; ++j) {
    l += (d.sym_cum[j] <= r) ? 1u : 0u;
  }
  const uint32_t k = r - d.sym_cum[l];
  sym              = l;
  uint32_t       sc;
  if ((d.dmrs_mask >> l) & 1u) {
    const uint32_t nd  = d.nd_dmrs;
    const uint32_t prb = k / nd;
    sc                 = prb * 12u + static_cast<uint32_t>((d.dmrs_lut >> (4u * (k - prb * nd))) & 15u);
  } else {
    sc = k;
  }
  const uint32_t ge = d.grid_base + l * d.nsc + sc;
  const uint32_t ee = d.ce_base + (d.ce_compact ? 0u : l * d.nsc) + sc;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (p < static_cast<int>(d.P)) {
      yw[p] = grids[ge + p * d.port_stride];
#pragma unroll
      for (int ly = 0; ly < L; ++ly) {
        hw[ly][p] = ce[ee + ly * d.ce_layer_stride + p * d.port_stride];
      }
    }
  }
}

/// Every RE of the chunk owned by this lane: loads, equalization (L layers), demapping (QM bits per layer),
/// descrambling and the packed LLR bytes into the LDS output buffer. L and QM are compile-time so that every register
/// array has static indices and the RE's L * QM bytes are assembled in registers.
template <int L, int QM>
__device__ __forceinline__ void demod_res(const demod_uniform& u,
                                          demap_pair_table*    tab,
                                          const uint32_t* __restrict__ grids,
                                          const uint32_t* __restrict__ ce,
                                          uint32_t*       seq,
                                          uint32_t*       out32)
{
  constexpr uint32_t LQ = L * QM;
  const demod_desc&  d  = *u.d;
  const uint32_t     P  = d.P;
  const bool         zf = d.eq == DEMOD_EQ_ZF;
  // The first RE's loads are in flight while the chunk's sequence is generated.
  uint32_t r = u.re_begin + threadIdx.x;
  uint32_t yw[4] = {}, hw[L][4] = {}, sym = 0;
  if (r < u.re_end) {
    load_re<L>(d, r, grids, ce, yw, hw, sym);
  }
  stage_chunk(u, seq, tab);
  __syncthreads();
  for (bool first = true; r < u.re_end; r += DEMOD_THREADS, first = false) {
#if SRSGPU_DEMOD_PREFETCH
    // The next RE's loads fly while this one is equalised and demapped.
    (void)first;
    uint32_t       nyw[4] = {}, nhw[L][4] = {}, nsym = 0;
    const uint32_t rn     = r + DEMOD_THREADS;
    if (rn < u.re_end) {
      load_re<L>(d, rn, grids, ce, nyw, nhw, nsym);
    }
#else
    if (!first) {
      load_re<L>(d, r, grids, ce, yw, hw, sym);
    }
#endif
    cpx y[4], h[L][4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      y[p] = bf16c(yw[p]);
#pragma unroll
      for (int ly = 0; ly < L; ++ly) {
        h[ly][p] = bf16c(hw[ly][p]);
      }
    }
    if (u.rot != nullptr) {
      // Compact estimate with CFO compensation: the symbol's estimate the reference estimator stores,
      // bf16(bf16(h) e^{j 2 pi t_l cfo}) (port_channel_estimator_average_impl.cpp:128).
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#pragma unroll
        for (int ly = 0; ly < L; ++ly) {
          h[ly][p] = bf16c(to_bf16c(cmul(h[ly][p], u.rot[(sym * 4 + ly) * 4 + p])));
        }
      }
    }
    cpx   eq[L];
    float var[L];
    if constexpr (L == 1) {
      // ZF 1 x N (MMSE with one layer is the same, channel_equalizer_generic_impl.cpp:343).
      float ch_mod_sq = 0.f, nvar_acc = 0.f;
      cpx   acc       = cmk(0.f, 0.f);
#pragma unroll
      for (uint32_t p = 0; p < 4; ++p) {
        if (p < P) {
          const float norm = h[0][p].x * h[0][p].x + h[0][p].y * h[0][p].y;
          if (isnormal_f(norm) && isnormal_f(u.nv[p]) && u.nv[p] > 0.f) {
            ch_mod_sq += norm;
            nvar_acc += norm * u.nv[p];
            acc = cadd(acc, cmulc(y[p], h[0][p]));
          }
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
    } else {
      bool done = false;
      if constexpr (L == 2) {
        if (zf) {
          // ZF 2 x N with the largest noise variance.
          done  = true;
          eq[0] = eq[1] = cmk(0.f, 0.f);
          var[0] = var[1] = __builtin_inff();
          if (isnormal_f(u.nv_max) && u.nv_max >= 0.f) {
            float n0 = 0.f, n1 = 0.f;
            cpx   xi = cmk(0.f, 0.f), m0 = cmk(0.f, 0.f), m1 = cmk(0.f, 0.f);
#pragma unroll
            for (uint32_t p = 0; p < 4; ++p) {
              if (p < P) {
                n0 += h[0][p].x * h[0][p].x + h[0][p].y * h[0][p].y;
                n1 += h[1][p].x * h[1][p].x + h[1][p].y * h[1][p].y;
                xi = cadd(xi, cmulc(h[1][p], h[0][p]));  // conj(h0) h1
                m0 = cadd(m0, cmulc(y[p], h[0][p]));
                m1 = cadd(m1, cmulc(y[p], h[1][p]));
              }
            }
            const float d_pinv = n0 * n1 - (xi.x * xi.x + xi.y * xi.y);
            if (isnormal_f(d_pinv)) {
              const float rcp = 1.f / d_pinv;
              eq[0]           = cscale(csub(cscale(m0, n1), cmul(xi, m1)), rcp);
              eq[1]           = cscale(csub(cscale(m1, n0), cmulc(m0, xi)), rcp);
              var[0]          = u.nv_max * n1 * rcp;
              var[1]          = u.nv_max * n0 * rcp;
            }
          }
        }
      }
      if (!done) {
        equalize_mmse<L>(y, h, P, u.nv_max, eq, var);
      }
    }

    // Demap, descramble (sequence bits of the RE's LLRs, MSB-first words staged in LDS) and pack the bytes.
    const uint32_t o  = r * LQ - u.word0 * 32u;
    const uint32_t wi = o >> 5;
    const uint64_t sb = ((static_cast<uint64_t>(seq[wi]) << 32) | seq[wi + 1]) << (o & 31u);
    uint32_t       pk[(LQ + 3) / 4] = {};
#pragma unroll
    for (int ly = 0; ly < L; ++ly) {
      int v[QM];
      demap<QM>(eq[ly], var[ly], tab, v);
#pragma unroll
      for (int j = 0; j < QM; ++j) {
        const int      b   = ly * QM + j;
        const uint32_t bit = static_cast<uint32_t>(sb >> (63 - b)) & 1u;
        const uint32_t s8  = static_cast<uint8_t>(static_cast<int8_t>(bit ? -v[j] : v[j]));
        pk[b / 4] |= s8 << (8 * (b % 4));
      }
    }
    const uint32_t ob = (r - u.re_begin) * LQ;
    if constexpr (LQ % 4 == 0) {
#pragma unroll
      for (uint32_t i = 0; i < LQ / 4; ++i) {
        out32[ob / 4 + i] = pk[i];
      }
    } else {
      uint8_t* out8 = reinterpret_cast<uint8_t*>(out32);
#pragma unroll
      for (uint32_t b = 0; b < LQ; ++b) {
        out8[ob + b] = static_cast<uint8_t>(pk[b / 4] >> (8 * (b % 4)));
      }
    }
#if SRSGPU_DEMOD_PREFETCH
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      yw[p] = nyw[p];
#pragma unroll
      for (int ly = 0; ly < L; ++ly) {
        hw[ly][p] = nhw[ly][p];
      }
    }
    sym = nsym;
#endif
  }
}

template <int QM>
__device__ __forceinline__ void demod_res_qm(const demod_uniform& u, demap_pair_table* tab,
                                             const uint32_t* __restrict__ grids, const uint32_t* __restrict__ ce,
                                             uint32_t* seq, uint32_t* out32)
{
  switch (u.d->L) {
    case 1: demod_res<1, QM>(u, tab, grids, ce, seq, out32); break;
    case 2: demod_res<2, QM>(u, tab, grids, ce, seq, out32); break;
    case 3: demod_res<3, QM>(u, tab, grids, ce, seq, out32); break;
    default: demod_res<4, QM>(u, tab, grids, ce, seq, out32); break;
  }
}

#ifdef SRSGPU_DEMOD_WAVES  // occupancy experiments: waves per SIMD forced by the register allocator
#define DEMOD_OCCUPANCY __attribute__((amdgpu_waves_per_eu(SRSGPU_DEMOD_WAVES, SRSGPU_DEMOD_WAVES)))
#else
#define DEMOD_OCCUPANCY
#endif
__global__ __launch_bounds__(DEMOD_THREADS) DEMOD_OCCUPANCY void pusch_demodulate_kernel(const demod_desc* __restrict__ descs,
                                                                         const mod_chunk* __restrict__ chunks,
                                                                         const demap_pair_table* __restrict__ tables,
                                                                         const uint32_t* __restrict__ grids,
                                                                         const uint32_t* __restrict__ ce,
                                                                         const float* __restrict__ noise_var,
                                                                         int8_t* __restrict__ llrs,
                                                                         const uint32_t* __restrict__ gseq)
{
  __shared__ uint32_t         seq[DEMOD_CHUNK_WORDS + 1];
  __shared__ demap_pair_table tab[DEMAP_TABLES];
  __shared__ uint32_t         out32[DEMOD_OUT_BYTES / 4];
  __shared__ cpx              rot[14 * 16];
  const mod_chunk             ch     = chunks[blockIdx.x];
  const demod_desc&           d      = descs[ch.tx];
  const uint32_t              tid    = threadIdx.x;
  demod_uniform u;
  u.d        = &d;
  u.re_begin = ch.re_begin;
  u.re_end   = ch.re_end;
  u.word0    = ch.word0;
  u.tables   = tables;
  u.gseq     = gseq;
  u.rot      = nullptr;
  if (d.ce_cfo) {
    // Per (symbol, layer, port) rotation by the estimator's CFO (float bits next to the compact row); the caller's
    // first barrier (after stage_chunk) publishes them.
    for (uint32_t i = tid; i < 14u * 16u; i += DEMOD_THREADS) {
      const uint32_t l = i >> 4, ly = (i >> 2) & 3u, p = i & 3u;
      float          c = 0.f;
      if (ly < d.L && p < d.P) {
        c = __uint_as_float(ce[d.ce_base + ly * d.ce_layer_stride + p * d.port_stride + d.nsc]);
      }
      float sn, cs;
      sincosf(6.283185307f * d.epochs[l] * c, &sn, &cs);
      rot[i] = cmk(cs, sn);
    }
    u.rot = rot;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    u.nv[p] = noise_var[4 * d.tx + p];
  }
  u.nv_max = u.nv[0];
#pragma unroll
  for (uint32_t p = 1; p < 4; ++p) {
    u.nv_max = (p < d.P) ? fmaxf(u.nv_max, u.nv[p]) : u.nv_max;
  }

  switch (d.qm) {
    case 2: demod_res_qm<2>(u, tab, grids, ce, seq, out32); break;
    case 4: demod_res_qm<4>(u, tab, grids, ce, seq, out32); break;
    case 6: demod_res_qm<6>(u, tab, grids, ce, seq, out32); break;
    default: demod_res_qm<8>(u, tab, grids, ce, seq, out32); break;
  }
  __syncthreads();

  // Contiguous LLR range [re_begin * Lq, re_end * Lq) of the codeword, staged from LDS byte 0. With s = dst & 3, the
  // aligned global word j holds staged bytes 4 j - s .. 4 j - s + 3: two LDS words funnel-shifted, one dword store.
  const uint32_t Lq  = static_cast<uint32_t>(d.L) * d.qm;
  const uint32_t n   = (ch.re_end - ch.re_begin) * Lq;
  int8_t*        dst = llrs + d.llr_offset + ch.re_begin * Lq;
  const uint32_t s   = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst) & 3u);
  uint32_t*      g32 = reinterpret_cast<uint32_t*>(dst - s);
  const uint32_t j0  = (s == 0) ? 0u : 1u;       // first full word
  const uint32_t j1  = (n + s) / 4;               // end of the full words
  for (uint32_t j = j0 + tid; j < j1; j += DEMOD_THREADS) {
    g32[j] = (s == 0) ? out32[j] : __builtin_amdgcn_alignbyte(out32[j], out32[j - 1], 4u - s);
  }
  const uint8_t* out8 = reinterpret_cast<const uint8_t*>(out32);
  if (s != 0 && tid < min(4u - s, n)) {  // head bytes before the first full word
    dst[tid] = static_cast<int8_t>(out8[tid]);
  }
  const uint32_t t0 = (j1 > 0 ? 4u * j1 - s : 0u);  // tail bytes after the last full word
  if (j1 >= j0 && t0 + tid < n && tid < 4u) {
    dst[t0 + tid] = static_cast<int8_t>(out8[t0 + tid]);
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
                             const uint32_t*         d_seq,
                             hipStream_t             stream)
{
  if (nof_chunks <= 0) {
    return;
  }
  hipLaunchKernelGGL(pusch_demodulate_kernel, dim3(static_cast<unsigned>(nof_chunks)), dim3(DEMOD_THREADS), 0, stream,
                     d_desc, d_chunks, d_tables, d_grids, d_ch_est, d_noise_var, d_llrs, d_seq);
}

} // namespace srsgpu
