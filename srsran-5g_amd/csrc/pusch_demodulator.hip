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
#include <cstdlib>

#include "common.h"
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

/// ZF 1 x N (MMSE with one layer is the same, channel_equalizer_generic_impl.cpp:343; equalize_zf_1xn.h:128): ports
/// with an abnormal channel or noise variance are skipped, nvar = sum |h|^2 nv / (sum |h|^2)^2.
__device__ __forceinline__ void equalize_zf1(const cpx* y, const cpx* h, uint32_t P, const float* nv, cpx& eq,
                                             float& var)
{
  float ch_mod_sq = 0.f, nvar_acc = 0.f;
  cpx   acc       = cmk(0.f, 0.f);
#pragma unroll
  for (uint32_t p = 0; p < 4; ++p) {
    if (p < P) {
      const float norm = h[p].x * h[p].x + h[p].y * h[p].y;
      if (isnormal_f(norm) && isnormal_f(nv[p]) && nv[p] > 0.f) {
        ch_mod_sq += norm;
        nvar_acc += norm * nv[p];
        acc = cadd(acc, cmulc(y[p], h[p]));
      }
    }
  }
  if (isnormal_f(ch_mod_sq) && isnormal_f(nvar_acc)) {
    const float rcp = 1.f / ch_mod_sq;
    eq              = cscale(acc, rcp);
    var             = nvar_acc * rcp * rcp;
  } else {
    eq  = cmk(0.f, 0.f);
    var = __builtin_inff();
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
  const uint16_t*         crbs;    ///< The plan's CRB lists (demod_desc::crb_list).
  float*                  lacc;    ///< LDS [14][4] statistics accumulators, or null without statistics.
};

/// Constellation point of QM hard decisions (LLR <= 0 -> bit 1, log_likelihood_ratio.cpp hard_decision) of one layer,
/// TS 38.211 section 5.1 as modulation_mapper_lut_impl.cpp:39 tabulates it: per component s_j = 1 - 2 b_j,
/// s0 (2^(h-1) - s2 (2^(h-2) - ... (2 - s_{2(h-1)}))) / sqrt(average power). The EVM calculator re-modulates these.
template <int QM>
__device__ __forceinline__ cpx hard_point(const int* v)
{
  constexpr int   H   = QM / 2;
  constexpr float AMP = QM == 2 ? 0.70710678f : QM == 4 ? 0.31622777f : QM == 6 ? 0.15430335f : 0.076696499f;
  float           c[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    float inner = 1.f;
    if constexpr (H > 1) {
      inner = 2.f - ((v[2 * (H - 1) + k] <= 0) ? -1.f : 1.f);
#pragma unroll
      for (int j = H - 2; j >= 1; --j) {
        inner = static_cast<float>(1 << (H - j)) - ((v[2 * j + k] <= 0) ? -1.f : 1.f) * inner;
      }
    }
    c[k] = ((v[k] <= 0) ? -inner : inner) * AMP;
  }
  return cmk(c[0], c[1]);
}

/// Per-lane statistics of the REs of one OFDM symbol, flushed into the workgroup's LDS accumulators.
struct lane_stats {
  uint32_t sym = 0xffffffffu;
  float    nv = 0.f, cnt = 0.f, e2 = 0.f, n = 0.f;

  __device__ __forceinline__ void flush(float* lacc)
  {
    if (sym != 0xffffffffu) {
      atomicAdd(&lacc[4 * sym + 0], nv);
      atomicAdd(&lacc[4 * sym + 1], cnt);
      atomicAdd(&lacc[4 * sym + 2], e2);
      atomicAdd(&lacc[4 * sym + 3], n);
    }
    nv = cnt = e2 = n = 0.f;
  }
  /// One equalized symbol: the finite noise variances (filter_infinite_and_accumulate, pusch_demodulator_impl.cpp:
  /// 225) and the squared error to the hard-decision point (evm_calculator_generic_impl.cpp).
  template <int QM>
  __device__ __forceinline__ void add(cpx eq, float var, const int* v)
  {
    if (!__builtin_isinf(var)) {
      nv += var;
      cnt += 1.f;
    }
    const cpx e = csub(hard_point<QM>(v), eq);
    e2 += e.x * e.x + e.y * e.y;
    n += 1.f;
  }
};

/// Round-to-nearest-even float -> bf16 pair (adt/bf16.h), the estimator's storage rounding.
__device__ __forceinline__ uint32_t to_bf16c(cpx v)
{
  const uint32_t a = __float_as_uint(v.x), b = __float_as_uint(v.y);
  return ((a + 0x7fffu + ((a >> 16) & 1u)) >> 16) | (((b + 0x7fffu + ((b >> 16) & 1u)) >> 16) << 16);
}

/// Stages the chunk's descrambling words (and the first word of the next chunk) and, for 64/256QAM, the demapper
/// tables in LDS. The caller synchronises.
template <int T>
__device__ __forceinline__ void stage_chunk(const demod_uniform& u, uint32_t* seq, demap_pair_table* tab)
{
  const demod_desc& d      = *u.d;
  const uint32_t    tid    = threadIdx.x;
  const uint32_t    nwords = (d.nof_llrs + 31u) >> 5;
  // The words the chunk's REs read (o >> 5 and the next one, demod_res): at most DEMOD_CHUNK_WORDS + 1, fewer for the
  // short chunks of a small plan.
  const uint32_t Lq    = static_cast<uint32_t>(d.L) * d.qm;
  const uint32_t need  = ((u.re_end * Lq + 31u) >> 5) - u.word0 + 1u;
  const uint32_t stage = need < DEMOD_CHUNK_WORDS + 1u ? need : DEMOD_CHUNK_WORDS + 1u;
  for (uint32_t j = tid; j < stage; j += T) {
    const uint32_t w = u.word0 + j;
    seq[j]           = (w < nwords) ? u.gseq[d.seq_word_offset + w] : 0u;
  }
  if (d.qm >= 6) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(u.tables);
    uint32_t*       dst = reinterpret_cast<uint32_t*>(tab);
    for (uint32_t i = tid; i < DEMAP_TABLES * sizeof(demap_pair_table) / 4; i += T) {
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
                                        const uint16_t* __restrict__ crbs,
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
  const bool     dm = (d.dmrs_mask >> l) & 1u;
  if (d.crb_list == DEMOD_CONTIGUOUS) {
    if (dm) {
      const uint32_t nd  = d.nd_dmrs;
      const uint32_t prb = k / nd;
      sc                 = prb * 12u + static_cast<uint32_t>((d.dmrs_lut >> (4u * (k - prb * nd))) & 15u);
    } else {
      sc = k;
    }
  } else {
    // CRB-mask allocation (pusch_demodulator_impl.cpp:290 rb_mask kron the PRB's RE pattern): the p-th allocated
    // PRB of the symbol is the p-th entry of the transmission's CRB list.
    const uint32_t per = dm ? static_cast<uint32_t>(d.nd_dmrs) : 12u;
    const uint32_t prb = k / per;
    const uint32_t kk  = k - prb * per;
    sc = static_cast<uint32_t>(crbs[d.crb_list + prb]) * 12u +
         (dm ? static_cast<uint32_t>((d.dmrs_lut >> (4u * kk)) & 15u) : kk);
  }
  const uint32_t ge = d.grid_base + l * d.nsc + sc;
  const uint32_t ee = d.ce_base + (d.ce_compact ? 0u : l * d.nsc) + sc;
  // Unsigned 32-bit byte offsets from the buffers' SGPR bases (saddr loads, no 64-bit address arithmetic per load).
  const char* gb = reinterpret_cast<const char*>(grids);
  const char* cb = reinterpret_cast<const char*>(ce);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (p < static_cast<int>(d.P)) {
      yw[p] = *reinterpret_cast<const uint32_t*>(gb + (ge + p * d.port_stride) * 4u);
#pragma unroll
      for (int ly = 0; ly < L; ++ly) {
        hw[ly][p] = *reinterpret_cast<const uint32_t*>(cb + (ee + ly * d.ce_layer_stride + p * d.port_stride) * 4u);
      }
    }
  }
}

/// Noise variances (per port and their maximum) and, for compact estimates with CFO compensation, the per (symbol,
/// layer, port) rotation by the estimator's CFO (float bits next to the compact row). The caller synchronises before
/// the rotations are read.
__device__ __forceinline__ void setup_uniform(const demod_desc& d, const uint32_t* __restrict__ ce,
                                              const float* __restrict__ noise_var, cpx* rot, demod_uniform& u)
{
  u.rot = nullptr;
  if (d.ce_cfo) {
    // Only the transmission's L layers' entries (every port slot p < 4: the RE loop reads them all; unused ports get
    // the identity): 56 sincos per workgroup for one layer instead of 224, before the workgroup's first barrier.
    const uint32_t nl = d.L;
    for (uint32_t j = threadIdx.x; j < 14u * 4u * nl; j += blockDim.x) {
      const uint32_t l = j / (4u * nl), ly = (j / 4u) % nl, p = j & 3u;
      const uint32_t i = (l * 4u + ly) * 4u + p;
      float          c = 0.f;
      if (p < d.P) {
        c = __uint_as_float(ce[d.ce_base + ly * d.ce_layer_stride + p * d.port_stride + d.nsc + d.cfo_sc]);
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
}

/// Every RE of the chunk owned by this lane: loads, equalization (L layers), demapping (QM bits per layer),
/// descrambling and the packed LLR bytes into the LDS output buffer. L and QM are compile-time so that every register
/// array has static indices and the RE's L * QM bytes are assembled in registers.
template <int L, int QM, bool STATS, int T>
__device__ __forceinline__ void demod_res(demod_uniform        u,
                                          demap_pair_table*    tab,
                                          const uint32_t* __restrict__ grids,
                                          const uint32_t* __restrict__ ce,
                                          const float* __restrict__ noise_var,
                                          cpx*            rot,
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
    load_re<L>(d, r, grids, ce, u.crbs, yw, hw, sym);
  }
  stage_chunk<T>(u, seq, tab);
  // The noise variances and CFO rotations are needed from the first equalisation on: their loads follow the RE's and
  // the sequence's, so the three fly together after the descriptor (chunk -> descriptor -> data, two dependent steps).
  setup_uniform(d, ce, noise_var, rot, u);
  __syncthreads();
  lane_stats st;
  for (bool first = true; r < u.re_end; r += T, first = false) {
    if (!first) {
      load_re<L>(d, r, grids, ce, u.crbs, yw, hw, sym);
    }
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
          const cpx r = u.rot[(sym * 4 + ly) * 4 + p];
          cpx       o;
          cmul_fused(h[ly][p].x, h[ly][p].y, r.x, r.y, o.x, o.y);  // as the estimator's per-symbol layout
          h[ly][p] = bf16c(to_bf16c(o));
        }
      }
    }
    cpx   eq[L];
    float var[L];
    if constexpr (L == 1) {
      equalize_zf1(y, h[0], P, u.nv, eq[0], var[0]);
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
    if (STATS && sym != st.sym) {
      st.flush(u.lacc);
      st.sym = sym;
    }
#pragma unroll
    for (int ly = 0; ly < L; ++ly) {
      int v[QM];
      demap<QM>(eq[ly], var[ly], tab, v);
      if constexpr (STATS) {
        st.add<QM>(eq[ly], var[ly], v);
      }
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
  }
  if constexpr (STATS) {
    st.flush(u.lacc);
  }
}

template <int QM, bool STATS, int T>
__device__ __forceinline__ void demod_res_qm(const demod_uniform& u, demap_pair_table* tab,
                                             const uint32_t* __restrict__ grids, const uint32_t* __restrict__ ce,
                                             const float* __restrict__ noise_var, cpx* rot, uint32_t* seq,
                                             uint32_t* out32)
{
  switch (u.d->L) {
    case 1: demod_res<1, QM, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
    case 2: demod_res<2, QM, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
    case 3: demod_res<3, QM, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
    default: demod_res<4, QM, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
  }
}

/// Statistics of OFDM symbol l from its accumulators v[4 l .. 4 l + 3] (pusch_demodulator_impl.cpp:406
/// on_provisional_stats): SINR dB and EVM, NaN for a symbol without data.
__device__ __forceinline__ void symbol_stats(const float* v, int l, float* __restrict__ o)
{
  const float nv = v[4 * l], cnt = v[4 * l + 1], e2 = v[4 * l + 2], n = v[4 * l + 3];
  if (n == 0.f) {
    o[2 * l] = o[2 * l + 1] = __builtin_nanf("");
    return;
  }
  o[2 * l]     = (cnt > 0.f && nv > 0.f) ? -10.f * log10f(nv / cnt) : __builtin_inff();
  o[2 * l + 1] = sqrtf(e2 / n);
}

/// Statistics of the whole transmission (pusch_demodulator_impl.cpp:432 on_end_stats) from its accumulators.
__device__ __forceinline__ void total_stats(const float* v, float* __restrict__ o)
{
  float tot_nv = 0.f, tot_cnt = 0.f, tot_evm = 0.f, tot_n = 0.f;
  for (int l = 0; l < 14; ++l) {
    const float n = v[4 * l + 3];
    if (n != 0.f) {
      tot_nv += v[4 * l];
      tot_cnt += v[4 * l + 1];
      tot_evm += n * sqrtf(v[4 * l + 2] / n);
      tot_n += n;
    }
  }
  const float nan = __builtin_nanf("");
  o[28] = tot_n == 0.f ? nan : ((tot_cnt > 0.f && tot_nv > 0.f) ? -10.f * log10f(tot_nv / tot_cnt) : __builtin_inff());
  o[29] = tot_n == 0.f ? nan : tot_evm / tot_n;
}

/// STATS: also accumulate the post-equalization statistics (a separate instantiation, so that the plain kernel keeps
/// its register budget).
template <bool STATS, int T>
__global__ __launch_bounds__(T) void pusch_demodulate_kernel(const demod_desc* __restrict__ descs,
                                                                         const mod_chunk* __restrict__ chunks,
                                                                         const demap_pair_table* __restrict__ tables,
                                                                         const uint32_t* __restrict__ grids,
                                                                         const uint32_t* __restrict__ ce,
                                                                         const float* __restrict__ noise_var,
                                                                         int8_t* __restrict__ llrs,
                                                                         const uint32_t* __restrict__ gseq,
                                                                         const uint16_t* __restrict__ crbs,
                                                                         float* __restrict__ acc)
{
  __shared__ uint32_t         seq[DEMOD_CHUNK_WORDS + 1];
  __shared__ demap_pair_table tab[DEMAP_TABLES];
  __shared__ uint32_t         out32[DEMOD_OUT_BYTES / 4];
  __shared__ cpx              rot[14 * 16];
  __shared__ float            lacc[DEMOD_ACC_PER_TX + 1];
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
  u.crbs     = crbs;
  u.lacc     = nullptr;
  if (STATS) {
    // Zeroed before the caller's first barrier (after stage_chunk).
    for (uint32_t i = tid; i < static_cast<uint32_t>(DEMOD_ACC_PER_TX); i += T) {
      lacc[i] = 0.f;
    }
    u.lacc = lacc;
  }

  switch (d.qm) {
    case 2: demod_res_qm<2, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
    case 4: demod_res_qm<4, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
    case 6: demod_res_qm<6, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
    default: demod_res_qm<8, STATS, T>(u, tab, grids, ce, noise_var, rot, seq, out32); break;
  }
  __syncthreads();
  if (STATS && tid < static_cast<uint32_t>(DEMOD_ACC_PER_TX) && lacc[tid] != 0.f) {
    atomicAdd(&acc[DEMOD_ACC_PER_TX * d.tx + tid], lacc[tid]);
  }

  // Contiguous LLR range [re_begin * Lq, re_end * Lq) of the codeword, staged from LDS byte 0. With s = dst & 3, the
  // aligned global word j holds staged bytes 4 j - s .. 4 j - s + 3: two LDS words funnel-shifted, one dword store.
  const uint32_t Lq  = static_cast<uint32_t>(d.L) * d.qm;
  const uint32_t n   = (ch.re_end - ch.re_begin) * Lq;
  int8_t*        dst = llrs + d.llr_offset + ch.re_begin * Lq;
  const uint32_t s   = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst) & 3u);
  uint32_t*      g32 = reinterpret_cast<uint32_t*>(dst - s);
  const uint32_t j0  = (s == 0) ? 0u : 1u;       // first full word
  const uint32_t j1  = (n + s) / 4;               // end of the full words
  for (uint32_t j = j0 + tid; j < j1; j += T) {
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


// ---------------------------------------------------------------------------------------------------------------------
// Transform precoding (DFT-s-OFDM, pusch_demodulator_impl.cpp:346, transform_precoder_dft_impl.cpp): one workgroup per
// (transmission, OFDM symbol). Its M data REs are equalized (ZF 1 x N, one layer) into LDS, the valid noise variances
// replaced by their mean (deprecode_ofdm_symbol_noise), the M-point inverse DFT taken in LDS (Stockham autosort,
// radices 4, 2, 3, 5: M = 12 x 2^a 3^b 5^c) and scaled by 1 / sqrt(M), then demapped, descrambled and written like
// the chunked kernel. M <= 12 x 270 = 3240.
// ---------------------------------------------------------------------------------------------------------------------
constexpr int      TP_THREADS = 256;
constexpr uint32_t TP_MAX_M   = 3240;

/// Noise variance classes kept per RE across the inverse DFT: valid ones become the symbol's mean.
constexpr uint8_t TP_VALID = 0, TP_INF = 1, TP_OTHER = 2;

template <int R>
__device__ __forceinline__ void small_idft(cpx* v)
{
  // Inverse (e^{+j 2 pi t u / R}) R-point DFT, R = 2, 3, 4, 5.
  if constexpr (R == 2) {
    const cpx a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  } else if constexpr (R == 4) {
    const cpx a = cadd(v[0], v[2]), b = csub(v[0], v[2]);
    const cpx c = cadd(v[1], v[3]), d = csub(v[1], v[3]);
    const cpx jd = cmk(-d.y, d.x);  // +j d
    v[0] = cadd(a, c);
    v[2] = csub(a, c);
    v[1] = cadd(b, jd);
    v[3] = csub(b, jd);
  } else if constexpr (R == 3) {
    const float c1 = -0.5f, s1 = 0.866025404f;
    const cpx   a = v[0], b = v[1], c = v[2];
    const cpx   t = cadd(b, c), dlt = csub(b, c);
    const cpx   m = cmk(a.x + c1 * t.x, a.y + c1 * t.y);
    const cpx   jd = cmk(-s1 * dlt.y, s1 * dlt.x);
    v[0] = cadd(a, t);
    v[1] = cadd(m, jd);
    v[2] = csub(m, jd);
  } else {
    const float c1 = 0.309016994f, s1 = 0.951056516f, c2 = -0.809016994f, s2 = 0.587785252f;
    const cpx   a = v[0];
    const cpx   t1 = cadd(v[1], v[4]), d1 = csub(v[1], v[4]);
    const cpx   t2 = cadd(v[2], v[3]), d2 = csub(v[2], v[3]);
    const cpx   m1 = cmk(a.x + c1 * t1.x + c2 * t2.x, a.y + c1 * t1.y + c2 * t2.y);
    const cpx   m2 = cmk(a.x + c2 * t1.x + c1 * t2.x, a.y + c2 * t1.y + c1 * t2.y);
    const cpx   n1 = cmk(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y);   // (s1 d1 + s2 d2)
    const cpx   n2 = cmk(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y);   // (s2 d1 - s1 d2)
    v[0] = cadd(a, cadd(t1, t2));
    v[1] = cadd(m1, cmk(-n1.y, n1.x));
    v[4] = csub(m1, cmk(-n1.y, n1.x));
    v[2] = cadd(m2, cmk(-n2.y, n2.x));
    v[3] = csub(m2, cmk(-n2.y, n2.x));
  }
}

/// One Stockham pass of radix R over M points (Ns = product of the previous radices): src -> dst.
template <int R>
__device__ __forceinline__ void stockham_pass(const cpx* src, cpx* dst, uint32_t M, uint32_t Ns)
{
  const uint32_t stride = M / R;
  for (uint32_t j = threadIdx.x; j < stride; j += TP_THREADS) {
    const uint32_t k = j % Ns;
    cpx            v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v[r] = src[j + r * stride];
    }
    if (k != 0) {
      // Twiddle e^{+j 2 pi r k / (Ns R)} (sincospi of an exact rational).
#pragma unroll
      for (int r = 1; r < R; ++r) {
        float sn, cs;
        sincospif(2.f * static_cast<float>(r * k) / static_cast<float>(Ns * R), &sn, &cs);
        v[r] = cmul(v[r], cmk(cs, sn));
      }
    }
    small_idft<R>(v);
    const uint32_t o = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      dst[o + r * Ns] = v[r];
    }
  }
}

/// Wave + workgroup sum of two floats (TP_THREADS / 64 waves); every thread gets the totals.
__device__ __forceinline__ void block_sum2(float& a, float& b, float* scratch)
{
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  const uint32_t w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63u) == 0) {
    scratch[2 * w]     = a;
    scratch[2 * w + 1] = b;
  }
  __syncthreads();
  a = b = 0.f;
#pragma unroll
  for (int i = 0; i < TP_THREADS / 64; ++i) {
    a += scratch[2 * i];
    b += scratch[2 * i + 1];
  }
}

template <int QM>
__device__ __forceinline__ void tp_demap_store(const demod_desc& d, const cpx* x, const uint8_t* cls, float mean,
                                               uint32_t M, uint32_t base, const demap_pair_table* tab,
                                               const uint32_t* __restrict__ gseq, int8_t* __restrict__ llrs,
                                               float (&st)[4])
{
  const float    scale  = 1.f / sqrtf(static_cast<float>(M));  // transform_precoder_dft_impl.cpp scaling_factor
  const uint32_t nwords = (d.nof_llrs + 31u) >> 5;
  for (uint32_t k = threadIdx.x; k < M; k += TP_THREADS) {
    const cpx   eq  = cscale(x[k], scale);
    const float var = cls[k] == TP_VALID ? mean : (cls[k] == TP_INF ? __builtin_inff() : 0.f);
    int         v[QM];
    demap<QM>(eq, var, tab, v);
    if (!__builtin_isinf(var)) {
      st[0] += var;
      st[1] += 1.f;
    }
    const cpx e = csub(hard_point<QM>(v), eq);
    st[2] += e.x * e.x + e.y * e.y;
    st[3] += 1.f;
    const uint32_t pos = (base + k) * QM;
    const uint32_t wi  = pos >> 5;
    const uint64_t w0  = gseq[d.seq_word_offset + wi];
    const uint64_t w1  = (wi + 1 < nwords) ? gseq[d.seq_word_offset + wi + 1] : 0u;
    const uint64_t sb  = ((w0 << 32) | w1) << (pos & 31u);
    int8_t*        dst = llrs + d.llr_offset + pos;
#pragma unroll
    for (int j = 0; j < QM; ++j) {
      const uint32_t bit = static_cast<uint32_t>(sb >> (63 - j)) & 1u;
      dst[j]             = static_cast<int8_t>(bit ? -v[j] : v[j]);
    }
  }
}

__global__ __launch_bounds__(TP_THREADS) void pusch_demodulate_tp_kernel(const demod_desc* __restrict__ descs,
                                                                        const demod_tp_job* __restrict__ jobs,
                                                                        const demap_pair_table* __restrict__ tables,
                                                                        const uint32_t* __restrict__ grids,
                                                                        const uint32_t* __restrict__ ce,
                                                                        const float* __restrict__ noise_var,
                                                                        int8_t* __restrict__ llrs,
                                                                        const uint32_t* __restrict__ gseq,
                                                                        const uint16_t* __restrict__ crbs,
                                                                        float* __restrict__ acc)
{
  __shared__ cpx              xa[TP_MAX_M], xb[TP_MAX_M];
  __shared__ uint8_t          cls[TP_MAX_M];
  __shared__ demap_pair_table tab[DEMAP_TABLES];
  __shared__ cpx              rot[14 * 16];
  __shared__ float            scratch[2 * (TP_THREADS / 64)];
  const demod_tp_job          job = jobs[blockIdx.x];
  const demod_desc&           d   = descs[job.tx];
  const uint32_t              l   = job.symbol;
  const uint32_t              base = d.sym_cum[l];
  const uint32_t              M    = static_cast<uint32_t>(d.sym_cum[l + 1]) - base;  // host-checked <= TP_MAX_M
  demod_uniform               u;
  setup_uniform(d, ce, noise_var, rot, u);
  if (d.qm >= 6) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(tables);
    uint32_t*       dst = reinterpret_cast<uint32_t*>(tab);
    for (uint32_t i = threadIdx.x; i < DEMAP_TABLES * sizeof(demap_pair_table) / 4; i += TP_THREADS) {
      dst[i] = src[i];
    }
  }
  __syncthreads();

  // Equalization of the symbol's M REs (one layer).
  float vsum = 0.f, vcnt = 0.f;
  for (uint32_t k = threadIdx.x; k < M; k += TP_THREADS) {
    uint32_t yw[4] = {}, hw[1][4] = {}, sym = 0;
    load_re<1>(d, base + k, grids, ce, crbs, yw, hw, sym);
    cpx y[4], h[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      y[p] = bf16c(yw[p]);
      h[p] = bf16c(hw[0][p]);
      if (u.rot != nullptr) {
        const cpx r = u.rot[(sym * 4) * 4 + p];
        cpx       o;
        cmul_fused(h[p].x, h[p].y, r.x, r.y, o.x, o.y);
        h[p] = bf16c(to_bf16c(o));
      }
    }
    cpx   eq;
    float var;
    equalize_zf1(y, h, d.P, u.nv, eq, var);
    xa[k] = eq;
    // transform_precoder_dft_impl.cpp deprecode_ofdm_symbol_noise: valid = positive, not NaN, not infinite.
    const bool valid = var > 0.f && !__builtin_isnan(var) && !__builtin_isinf(var);
    cls[k]           = valid ? TP_VALID : (__builtin_isinf(var) ? TP_INF : TP_OTHER);
    if (valid) {
      vsum += var;
      vcnt += 1.f;
    }
  }
  block_sum2(vsum, vcnt, scratch);
  const float mean = vcnt > 0.f ? vsum / vcnt : 0.f;
  __syncthreads();

  // Inverse DFT (unnormalised), Stockham radix 4, 2, 3, 5 passes; the same factorisation in every thread.
  cpx*     src = xa;
  cpx*     dst = xb;
  uint32_t rem = M, Ns = 1;
  while (rem > 1) {
    if (rem % 4 == 0) {
      stockham_pass<4>(src, dst, M, Ns);
      Ns *= 4;
      rem /= 4;
    } else if (rem % 2 == 0) {
      stockham_pass<2>(src, dst, M, Ns);
      Ns *= 2;
      rem /= 2;
    } else if (rem % 3 == 0) {
      stockham_pass<3>(src, dst, M, Ns);
      Ns *= 3;
      rem /= 3;
    } else {
      stockham_pass<5>(src, dst, M, Ns);
      Ns *= 5;
      rem /= 5;
    }
    __syncthreads();
    cpx* t = src;
    src    = dst;
    dst    = t;
  }

  float st[4] = {0.f, 0.f, 0.f, 0.f};
  switch (d.qm) {
    case 2: tp_demap_store<2>(d, src, cls, mean, M, base, tab, gseq, llrs, st); break;
    case 4: tp_demap_store<4>(d, src, cls, mean, M, base, tab, gseq, llrs, st); break;
    case 6: tp_demap_store<6>(d, src, cls, mean, M, base, tab, gseq, llrs, st); break;
    default: tp_demap_store<8>(d, src, cls, mean, M, base, tab, gseq, llrs, st); break;
  }
  if (acc != nullptr) {
    block_sum2(st[0], st[1], scratch);
    block_sum2(st[2], st[3], scratch);
    if (threadIdx.x < 4) {
      atomicAdd(&acc[DEMOD_ACC_PER_TX * d.tx + 4 * l + threadIdx.x], st[threadIdx.x]);
    }
  }
}

/// Statistics of every transmission from the accumulators (which it resets for the next execute): per symbol
/// (pusch_demodulator_impl.cpp:406 on_provisional_stats) and for the transmission (:432 on_end_stats).
__global__ __launch_bounds__(64) void pusch_demod_stats_kernel(float* __restrict__ acc, float* __restrict__ stats,
                                                               int nof_tx)
{
  const int t = static_cast<int>(blockIdx.x * 64 + threadIdx.x);
  if (t >= nof_tx) {
    return;
  }
  float* a = acc + DEMOD_ACC_PER_TX * t;
  float* o = stats + DEMOD_STATS_PER_TX * t;
  for (int l = 0; l < 14; ++l) {
    symbol_stats(a, l, o);
  }
  total_stats(a, o);
  for (int i = 0; i < DEMOD_ACC_PER_TX; ++i) {
    a[i] = 0.f;
  }
}

} // namespace

void launch_pusch_demodulate(const demod_desc*       d_desc,
                             const mod_chunk*        d_chunks,
                             int                     nof_chunks,
                             int                     plan_threads,
                             const demap_pair_table* d_tables,
                             const uint32_t*         d_grids,
                             const uint32_t*         d_ch_est,
                             const float*            d_noise_var,
                             int8_t*                 d_llrs,
                             const uint32_t*         d_seq,
                             const uint16_t*         d_crbs,
                             float*                  d_acc,
                             hipStream_t             stream)
{
  if (nof_chunks <= 0) {
    return;
  }
  const int  threads = plan_threads;
  const auto launch  = [&](auto kernel, int t) {
    hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(nof_chunks)), dim3(static_cast<unsigned>(t)), 0, stream,
                       d_desc, d_chunks, d_tables, d_grids, d_ch_est, d_noise_var, d_llrs, d_seq, d_crbs, d_acc);
  };
  if (d_acc != nullptr) {
    launch(pusch_demodulate_kernel<true, DEMOD_THREADS>, DEMOD_THREADS);
  } else if (threads == 64) {
    launch(pusch_demodulate_kernel<false, 64>, 64);
  } else if (threads == 128) {
    launch(pusch_demodulate_kernel<false, 128>, 128);
  } else {
    launch(pusch_demodulate_kernel<false, DEMOD_THREADS>, DEMOD_THREADS);
  }
}


void launch_pusch_demodulate_tp(const demod_desc*       d_desc,
                                const demod_tp_job*     d_jobs,
                                int                     nof_jobs,
                                const demap_pair_table* d_tables,
                                const uint32_t*         d_grids,
                                const uint32_t*         d_ch_est,
                                const float*            d_noise_var,
                                int8_t*                 d_llrs,
                                const uint32_t*         d_seq,
                                const uint16_t*         d_crbs,
                                float*                  d_acc,
                                hipStream_t             stream)
{
  if (nof_jobs <= 0) {
    return;
  }
  hipLaunchKernelGGL(pusch_demodulate_tp_kernel, dim3(static_cast<unsigned>(nof_jobs)), dim3(TP_THREADS), 0, stream,
                     d_desc, d_jobs, d_tables, d_grids, d_ch_est, d_noise_var, d_llrs, d_seq, d_crbs, d_acc);
}

void launch_pusch_demod_stats(float* d_acc, float* d_stats, int nof_tx, hipStream_t stream)
{
  if (nof_tx <= 0) {
    return;
  }
  hipLaunchKernelGGL(pusch_demod_stats_kernel, dim3(static_cast<unsigned>((nof_tx + 63) / 64)), dim3(64), 0, stream,
                     d_acc, d_stats, nof_tx);
}

} // namespace srsgpu
