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
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "gold_device.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {

#ifdef CHEST_PROFILE
// Instrumented builds only (tools/chest_phase_profile.py): s_memtime per phase of the first CHEST_PROF_JOBS jobs.
constexpr int CHEST_PROF_JOBS  = 4096;
constexpr int CHEST_PROF_SLOTS = 12;
__device__ uint64_t g_chest_prof[CHEST_PROF_JOBS * CHEST_PROF_SLOTS];
#define CHEST_PROF(slot, value)                                                                                        \
  do {                                                                                                                 \
    if (lane == 0 && job < CHEST_PROF_JOBS) {                                                                          \
      g_chest_prof[job * CHEST_PROF_SLOTS + (slot)] = (value);                                                         \
    }                                                                                                                  \
  } while (0)
#else
#define CHEST_PROF(slot, value)                                                                                        \
  do {                                                                                                                 \
  } while (0)
#endif
#define CHEST_STAMP(slot) CHEST_PROF(slot, __builtin_amdgcn_s_memtime())

/// Minimum waves per SIMD the estimator is compiled for. 8 (a 64-VGPR cap) spilled 10 VGPRs to scratch; at 4-5 the
/// few-RB instantiations settle at 72-78 VGPRs (6-7 waves per SIMD) with no spill, and the headline bench gains
/// 1.4 % (137.8k -> 139.8k slots/s, estimator stage 37.4 -> 33.5 us per step; profiles/r4_chest_waves_ab.txt); 4 also
/// keeps the 1024-lane wideband instantiation (100 VGPRs) from spilling.
#define CHEST_WAVES_PER_EU 4

constexpr int CHEST_THREADS = 64;  // one wavefront per job (multi-wave workgroups for large allocations: T)
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

// Cross-lane reductions on DPP (VALU lane permutations: no LDS round trip, which __shfl_xor's ds_bpermute costs per
// step). Within a 16-lane row: quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror, after which every
// lane of the row holds the row's result (each step pairs lanes symmetrically, so all lanes compute identical bits).
// Across rows: row_bcast:15 into rows 1 and 3 (the 32-lane halves: lanes 31 / 63 hold them) and row_bcast:31 into
// rows 2 and 3 (lane 63 holds the wave's), read back with readlane.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float old, float v)
{
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROW_MASK, 0xf, false));
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int dpp_i(int old, int v)
{
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, 0xf, false);
}
constexpr int DPP_XOR1 = 0xb1, DPP_XOR2 = 0x4e, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
constexpr int DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143;

__device__ __forceinline__ float row_sum(float v)
{
  v += dpp_f<DPP_XOR1>(0.f, v);
  v += dpp_f<DPP_XOR2>(0.f, v);
  v += dpp_f<DPP_HALF_MIRROR>(0.f, v);
  v += dpp_f<DPP_MIRROR>(0.f, v);
  return v;
}

__device__ __forceinline__ float readlane_f(float v, int lane)
{
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

/// Sum over the wavefront (every lane gets the result).
__device__ __forceinline__ float wave_sum(float v)
{
  v = row_sum(v);
  v += dpp_f<DPP_BCAST15, 0xa>(0.f, v);
  v += dpp_f<DPP_BCAST31, 0xc>(0.f, v);
  return readlane_f(v, 63);
}

/// Sum over the workgroup of T lanes (every lane gets the result; all lanes must call it). T = 64: wave shuffles only.
template <int T>
__device__ __forceinline__ float block_sum(float v, float* red)
{
  v = wave_sum(v);
  if constexpr (T > 64) {
    __syncthreads();  // red may still be read by a previous reduction
    if ((threadIdx.x & 63u) == 0) {
      red[threadIdx.x >> 6] = v;
    }
    __syncthreads();
    v = 0.f;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
      v += red[w];
    }
  }
  return v;
}

/// Sum over an aligned group of TS lanes (TS = 16, 32 or 64, every lane of the group gets the result).
template <int TS>
__device__ __forceinline__ float sub_sum(float v)
{
  static_assert(TS == 16 || TS == 32 || TS == 64, "row, half-wave or wave");
  if constexpr (TS == 64) {
    return wave_sum(v);
  } else {
    v = row_sum(v);
    if constexpr (TS == 32) {
      v += dpp_f<DPP_BCAST15, 0xa>(0.f, v);
      const float lo = readlane_f(v, 31), hi = readlane_f(v, 63);
      v              = (threadIdx.x & 32u) ? hi : lo;
    }
    return v;
  }
}

/// Sum over one job's lanes: TS < 64 lanes of a wave that holds several jobs, or the whole workgroup.
template <int T, int TS>
__device__ __forceinline__ float job_sum(float v, float* red)
{
  if constexpr (TS < 64) {
    return sub_sum<TS>(v);
  } else {
    return block_sum<T>(v, red);
  }
}

/// job_sum of K values at once: one barrier pair for all of them in a multi-wave job (the per-value sums are the same
/// as K separate job_sum calls: each wave's total, then the waves in ascending order). red: K x T / 64 floats.
template <int T, int TS, int K>
__device__ __forceinline__ void job_sum_n(float (&v)[K], float* red)
{
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if constexpr (TS < 64) {
      v[k] = sub_sum<TS>(v[k]);
    } else {
      v[k] = wave_sum(v[k]);
    }
  }
  if constexpr (TS >= 64 && T > 64) {
    __syncthreads();  // red may still be read by a previous reduction
    if ((threadIdx.x & 63u) == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        red[k * (T / 64) + (threadIdx.x >> 6)] = v[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < T / 64; ++w) {
        t += red[k * (T / 64) + w];
      }
      v[k] = t;
    }
  }
}


/// Ordering of a job's LDS stages: a workgroup barrier; in a one-wave workgroup (T = 64, where the 32-lane halves may
/// run jobs with different stage sequences) a wave-level fence: a wave's LDS accesses complete in program order.
template <int T>
__device__ __forceinline__ void job_sync()
{
  if constexpr (T == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    __syncthreads();
  }
}

/// DM-RS QPSK symbol i of DM-RS symbol s from the staged sequence words (amplitude 1/sqrt(2)).
__device__ __forceinline__ cpx pilot(const uint32_t* seq, int W, int s, uint32_t n0, int i)
{
  const uint32_t n    = 2 * static_cast<uint32_t>(i) + (n0 & 31u);  // bit index relative to the first staged word
  const uint32_t word = seq[s * W + (n >> 5)];
  const uint32_t sh   = 31u - (n & 31u);  // even n: both bits in the same word
  const float    a    = 0.70710678f;
  return {((word >> sh) & 1u) ? -a : a, ((word >> (sh - 1)) & 1u) ? -a : a};
}

/// DM-RS value of pilot i (sequence position m) on DM-RS symbol s: the staged pseudo-random QPSK symbol, or the job's
/// low-PAPR sequence value (transform precoding: the same sequence on every DM-RS symbol).
__device__ __forceinline__ cpx dmrs_value(const chest_job& jb, const float2* __restrict__ lp, const uint32_t* seq,
                                          int W, int s, uint32_t n0, int m, int i);

/// compute_v_pilots on the lanes: with H lanes per band edge (H = 32, or TS / 2 when a wave holds several jobs), lanes
/// 0..nv-1 of the first H extrapolate the band start from E[VP .. VP+nv), lanes H..H+nv-1 the band end from
/// E[VP+N-nv .. VP+N): linear regression of |p| and the unwrapped arg over x = 0..nv-1, evaluated at x = -nv..-1
/// (start) or nv..2nv-1 (end). Lanes j >= nv carry zeros, so the sums and the prefix do not depend on H.
template <int H>
__device__ __forceinline__ void virtual_pilots(cpx* E, int N, int nv, int sub)
{
  const int   side = sub / H;
  const int   j    = sub % H;
  const bool  act  = j < nv;
  const cpx   b    = act ? E[CHEST_VP + (side ? N - nv : 0) + j] : cpx{1.f, 0.f};
  const float ab   = act ? sqrtf(b.x * b.x + b.y * b.y) : 0.f;
  const float a    = atan2f(b.y, b.x);
  // Unwrap: arg_j + 2 pi c_j with c_j = sum_{m <= j} rint((a_{m-1} - a_m) / 2 pi) (prefix sum within the half).
  const float twopi = 6.28318531f;
  // Lane j - 1: row_shr:1 inside a row, row_bcast:15 for a row's first lane (H = 32: lane 16 of each half).
  const float prev_row = dpp_f<0x111>(a, a);
  const float prev_bc  = dpp_f<DPP_BCAST15, 0xa>(a, a);
  const float prev     = ((sub & 15) == 0) ? prev_bc : prev_row;
  float       c        = (j > 0 && act) ? rintf((prev - a) / twopi) : 0.f;
  // Inclusive prefix sum within the H lanes: row_shr:1 / 2 / 4 / 8 (lanes shifted in from outside the row add 0),
  // then for H = 32 the first row's total into the second row (row_bcast:15).
  c += dpp_f<0x111>(0.f, c);
  c += dpp_f<0x112>(0.f, c);
  c += dpp_f<0x114>(0.f, c);
  c += dpp_f<0x118>(0.f, c);
  static_assert(H == 16 || H == 32, "one row or two rows per band edge");
  if constexpr (H == 32) {
    c += dpp_f<DPP_BCAST15, 0xa>(0.f, c);
  }
  const float ar        = act ? a + twopi * c : 0.f;
  const float n         = static_cast<float>(nv);
  const float mean_x    = static_cast<float>(nv * (nv - 1)) / 2.0f / n;
  const float norm_x_sq = static_cast<float>((nv - 1) * nv * (2 * nv - 1)) / 6.0f;
  const float mab       = sub_sum<H>(ab) / n;
  const float mar       = sub_sum<H>(ar) / n;
  const float dab       = sub_sum<H>(ab * static_cast<float>(j));
  const float dar       = sub_sum<H>(ar * static_cast<float>(j));
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

constexpr float CHEST_TWOPI = 6.283185307f;  // TWOPI (srsran/support/math_utils.h)

__device__ __forceinline__ cpx cmul(cpx a, cpx b)
{
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

/// std::polar(1.0F, theta) in float.
__device__ __forceinline__ cpx polar1(float theta)
{
  float sn, cs;
  sincosf(theta, &sn, &cs);
  return {cs, sn};
}

/// PRB of the allocation's rb-th allocated CRB relative to the first allocated CRB (the CRB list of a mask).
__device__ __forceinline__ int alloc_rb(const chest_job& jb, const uint16_t* __restrict__ crbs, int rb)
{
  return jb.crb_list == CHEST_CONTIGUOUS ? rb : static_cast<int>(crbs[jb.crb_list + static_cast<uint32_t>(rb)]);
}

/// Pilot subcarrier of pilot i relative to the first allocated subcarrier.
__device__ __forceinline__ uint32_t pilot_subcarrier(const chest_job& jb, const uint16_t* __restrict__ crbs, int i)
{
  const int rb = jb.pilots_per_rb == 6 ? i / 6 : i / 4;  // constant divisors: multiply-shift, not a division
  return static_cast<uint32_t>(alloc_rb(jb, crbs, rb) * 12 +
                               ((jb.pattern >> (4 * (i - rb * jb.pilots_per_rb))) & 15u));
}

/// DM-RS sequence position of pilot i relative to the first allocated CRB's first one: the sequence skips the
/// unallocated CRBs (dmrs_helper.cpp:64 dmrs_sequence_generate over rb_mask).
__device__ __forceinline__ int pilot_seq_index(const chest_job& jb, const uint16_t* __restrict__ crbs, int i)
{
  const int rb = jb.pilots_per_rb == 6 ? i / 6 : i / 4;
  return alloc_rb(jb, crbs, rb) * jb.pilots_per_rb + (i - rb * jb.pilots_per_rb);
}

__device__ __forceinline__ cpx dmrs_value(const chest_job& jb, const float2* __restrict__ lp, const uint32_t* seq,
                                          int W, int s, uint32_t n0, int m, int i)
{
  if (jb.lp_base != CHEST_CONTIGUOUS) {
    const float2 v = lp[jb.lp_base + static_cast<uint32_t>(i)];
    return {v.x, v.y};
  }
  return pilot(seq, W, s, n0, m);
}

/// One argmax step against the (value, index) DPP delivers (rows outside ROW_MASK compare with themselves): the larger
/// value, the lower index among equal values (srsvec::max_element keeps the first maximum).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ void argmax_step(float& v, int& idx)
{
  const float ov = dpp_f<CTRL, ROW_MASK>(v, v);
  const int   oi = dpp_i<CTRL, ROW_MASK>(idx, idx);
  if (ov > v || (ov == v && oi < idx)) {
    v   = ov;
    idx = oi;
  }
}

__device__ __forceinline__ void row_argmax(float& v, int& idx)
{
  argmax_step<DPP_XOR1>(v, idx);
  argmax_step<DPP_XOR2>(v, idx);
  argmax_step<DPP_HALF_MIRROR>(v, idx);
  argmax_step<DPP_MIRROR>(v, idx);
}

/// Maximum over the wavefront with the lowest index among equal values.
__device__ __forceinline__ void wave_argmax(float& v, int& idx)
{
  row_argmax(v, idx);
  argmax_step<DPP_BCAST15, 0xa>(v, idx);
  argmax_step<DPP_BCAST31, 0xc>(v, idx);
  v   = readlane_f(v, 63);
  idx = __builtin_amdgcn_readlane(idx, 63);
}

/// wave_argmax over an aligned group of TS = 16 or 32 lanes.
template <int TS>
__device__ __forceinline__ void sub_argmax(float& v, int& idx)
{
  static_assert(TS == 16 || TS == 32, "row or half-wave");
  row_argmax(v, idx);
  if constexpr (TS == 32) {
    argmax_step<DPP_BCAST15, 0xa>(v, idx);
    const bool hi = (threadIdx.x & 32u) != 0;
    const float v0 = readlane_f(v, 31), v1 = readlane_f(v, 63);
    const int   i0 = __builtin_amdgcn_readlane(idx, 31), i1 = __builtin_amdgcn_readlane(idx, 63);
    v              = hi ? v1 : v0;
    idx            = hi ? i1 : i0;
  }
}

/// wave_argmax over the workgroup of T lanes (lowest index among equal maxima; all lanes must call it).
template <int T>
__device__ __forceinline__ void block_argmax(float& v, int& idx, float* redf, int* redi)
{
  wave_argmax(v, idx);
  if constexpr (T > 64) {
    __syncthreads();
    if ((threadIdx.x & 63u) == 0) {
      redf[threadIdx.x >> 6] = v;
      redi[threadIdx.x >> 6] = idx;
    }
    __syncthreads();
    v   = redf[0];
    idx = redi[0];
#pragma unroll
    for (int w = 1; w < T / 64; ++w) {
      if (redf[w] > v || (redf[w] == v && redi[w] < idx)) {
        v   = redf[w];
        idx = redi[w];
      }
    }
  }
}

/// Argmax over one job's lanes (see job_sum).
template <int T, int TS>
__device__ __forceinline__ void job_argmax(float& v, int& idx, float* redf, int* redi)
{
  if constexpr (TS < 64) {
    sub_argmax<TS>(v, idx);
  } else {
    block_argmax<T>(v, idx, redf, redi);
  }
}

/// Two job_argmax reductions with one barrier pair in a multi-wave job (each result as job_argmax's: the waves'
/// maxima in ascending wave order). redf / redi: 2 x T / 64 entries.
template <int T, int TS>
__device__ __forceinline__ void job_argmax2(float& v0, int& i0, float& v1, int& i1, float* redf, int* redi)
{
  if constexpr (TS < 64) {
    sub_argmax<TS>(v0, i0);
    sub_argmax<TS>(v1, i1);
  } else {
    wave_argmax(v0, i0);
    wave_argmax(v1, i1);
    if constexpr (T > 64) {
      constexpr int NW = T / 64;
      __syncthreads();
      if ((threadIdx.x & 63u) == 0) {
        redf[threadIdx.x >> 6]      = v0;
        redi[threadIdx.x >> 6]      = i0;
        redf[NW + (threadIdx.x >> 6)] = v1;
        redi[NW + (threadIdx.x >> 6)] = i1;
      }
      __syncthreads();
      v0 = redf[0];
      i0 = redi[0];
      v1 = redf[NW];
      i1 = redi[NW];
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        if (redf[w] > v0 || (redf[w] == v0 && redi[w] < i0)) {
          v0 = redf[w];
          i0 = redi[w];
        }
        if (redf[NW + w] > v1 || (redf[NW + w] == v1 && redi[NW + w] < i1)) {
          v1 = redf[NW + w];
          i1 = redi[NW + w];
        }
      }
    }
  }
}

/// LDS of a job, carved from the plan-sized dynamic allocation (chest_geom): the staged sequence words, the filter
/// taps, the smoothed planes F and one region shared by the LSE stage (Y per DM-RS symbol + enlarged E per layer) and
/// the time-alignment stage (the DFT buffer X + the correlation), which run one after the other.
struct chest_lds {
  uint32_t* seq;   ///< [max_dmrs][max_words]
  float*    taps;  ///< [32]
  cpx*      F;     ///< [max_planes][max_gl][max_pilots]
  cpx*      Y;     ///< [max_dmrs][max_pilots]
  cpx*      E;     ///< [max_gl][max_pilots + 2 CHEST_VP]
  cpx*      X;     ///< [max_dft] (aliases Y / E)
  float*    corr;  ///< [max_dft]
};

__device__ __host__ inline size_t chest_region_bytes(const chest_geom& g)
{
  const size_t lse = (static_cast<size_t>(g.max_dmrs) * g.max_pilots +
                      static_cast<size_t>(g.max_gl) * (g.max_pilots + 2 * CHEST_VP)) * sizeof(cpx);
  const size_t ta  = static_cast<size_t>(g.max_dft) * (sizeof(cpx) + sizeof(float));
  return lse > ta ? lse : ta;
}

/// Dynamic LDS of one job (16-byte multiple: the jobs of a workgroup are laid out one after the other).
__device__ __host__ inline size_t chest_job_lds_bytes(const chest_geom& g)
{
  const size_t b = static_cast<size_t>(g.max_planes) * g.max_gl * g.max_pilots * sizeof(cpx) + chest_region_bytes(g) +
                   static_cast<size_t>(g.max_dmrs) * g.max_words * 4 + 32 * 4;
  return (b + 15) & ~static_cast<size_t>(15);
}

/// T lanes per workgroup, TS lanes per job: TS = T (one job per workgroup), or T = 64 and TS = 32 (two jobs per wave,
/// one per 32-lane half: a few-RB job's pilots fill half a wave, so a whole wave per job issued every instruction for
/// twice the lanes it used; the chest kernel is bound by VALU issue, profiles/r3_v2_sq_serial.log).
template <int T, int TS>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(CHEST_WAVES_PER_EU, 8))) void pusch_chest_kernel(
    const chest_job* __restrict__ jobs,
    int nof_jobs,
    chest_geom geom,
    const uint32_t* __restrict__ grids,
    uint32_t* __restrict__ ce,
    float* __restrict__ noise_var,
    float* __restrict__ metrics,
    const uint32_t* __restrict__ gseq,
    const uint16_t* __restrict__ crbs,
    const float2* __restrict__ lp,
    const srsgpu_copy_span* __restrict__ spans,
    int nof_spans)
{
  extern __shared__ __align__(16) unsigned char lds_raw[];
  __shared__ float redf[3 * (T / 64)];
  __shared__ int   redi[2 * (T / 64)];
  constexpr int JPW  = T / TS;  // jobs per workgroup
  // Workgroups past the jobs' copy the spans (srsgpu_pusch_chest_plan_execute_copy: grid rows the estimator does not
  // read, moved while it runs): the same number of workgroups per span, each a contiguous part of 16-byte vectors.
  const int job_blocks = (nof_jobs + JPW - 1) / JPW;
  if (static_cast<int>(blockIdx.x) >= job_blocks) {
    const uint32_t cb       = blockIdx.x - static_cast<uint32_t>(job_blocks);
    const uint32_t per_span = (gridDim.x - static_cast<uint32_t>(job_blocks)) / static_cast<uint32_t>(nof_spans);
    const srsgpu_copy_span sp = spans[cb / per_span];
    const uint4*           s4 = reinterpret_cast<const uint4*>(sp.src);
    uint4*                 d4 = reinterpret_cast<uint4*>(sp.dst);
    for (uint64_t i = (cb % per_span) * T + threadIdx.x; i < sp.bytes / 16u; i += static_cast<uint64_t>(per_span) * T) {
      d4[i] = s4[i];
    }
    return;
  }
  const int     slot = static_cast<int>(threadIdx.x) / TS;
  const int     job  = static_cast<int>(blockIdx.x) * JPW + slot;
  if (JPW > 1 && job >= nof_jobs) {
    return;  // an odd job count leaves the second half of the last wave without a job (no workgroup barriers here)
  }
  const int EN = geom.max_pilots + 2 * CHEST_VP;
  chest_lds L;
  L.F    = reinterpret_cast<cpx*>(lds_raw + static_cast<size_t>(slot) * chest_job_lds_bytes(geom));
  L.Y    = L.F + static_cast<size_t>(geom.max_planes) * geom.max_gl * geom.max_pilots;
  L.E    = L.Y + static_cast<size_t>(geom.max_dmrs) * geom.max_pilots;
  L.X    = L.Y;
  L.corr = reinterpret_cast<float*>(L.X + geom.max_dft);
  L.seq  = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(L.Y) + chest_region_bytes(geom));
  L.taps = reinterpret_cast<float*>(L.seq + geom.max_dmrs * geom.max_words);

  // The job descriptor staged in LDS once (one coalesced read) instead of dependent scalar loads of its fields
  // (A/B on MI355X: chest stage 32.6 -> 28.9 us per 16-slot step).
  __shared__ chest_job sjob[JPW];
  {
    static_assert(sizeof(chest_job) % 4 == 0, "word copy");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(jobs + job);
    uint32_t*       dst = reinterpret_cast<uint32_t*>(&sjob[slot]);
    for (int w = static_cast<int>(threadIdx.x) % TS; w < static_cast<int>(sizeof(chest_job) / 4); w += TS) {
      dst[w] = src[w];
    }
    job_sync<T>();
  }
  const chest_job& jb = sjob[slot];
  const int        lane  = static_cast<int>(threadIdx.x) % TS;  // lane within the job
  CHEST_STAMP(0);
  CHEST_PROF(10, __builtin_amdgcn_s_memrealtime());
  const int        N     = jb.nof_pilots;
  const int        GL    = jb.group_layers;
  const int        D     = jb.nof_dmrs;
  const int        Q     = jb.td_interp ? D : 1;
  const float      beta  = jb.beta;
  const uint32_t   n0    = 2 * jb.seq_offset;  // first sequence bit of the allocation
  const int        W     = geom.max_words;
  const int        NP    = geom.max_pilots;
  cpx* const       Fbase = L.F;

  // Stage: taps and the sequence words of every DM-RS symbol (the plan's resident words, gold_fill_kernel).
  if (lane < 32) {
    L.taps[lane] = jb.taps[lane];
  }
  const int nwords = static_cast<int>(((n0 & 31u) + 2u * static_cast<uint32_t>(jb.span_pilots) + 31u) >> 5);
  for (int s = 0; s < D; ++s) {
    for (int wl = lane; wl < nwords; wl += TS) {
      L.seq[s * W + wl] = gseq[jb.gseq_base + static_cast<uint32_t>(s * nwords + wl)];
    }
  }
  job_sync<T>();
  CHEST_STAMP(1);

  // Pass 1: LSE of every DM-RS symbol (received x conj(pilot)), EPRE.
  float epre_acc = 0.f;
  for (int i = lane; i < N; i += TS) {
    const uint32_t k = pilot_subcarrier(jb, crbs, i);
    const int      m = pilot_seq_index(jb, crbs, i);
    for (int s = 0; s < D; ++s) {
      const cpx y = bf16c(grids[jb.grid_base + jb.dmrs_symbols[s] * jb.nsc + k]);
      const cpx p = dmrs_value(jb, lp, L.seq, W, s, n0, m, i);
      L.Y[s * NP + i] = {y.x * p.x + y.y * p.y, y.y * p.x - y.x * p.y};
      epre_acc += y.x * y.x + y.y * y.y;
    }
  }
  job_sync<T>();
  CHEST_STAMP(2);

  // CFO from the first two DM-RS symbols (preprocess_pilots_and_estimate_cfo, :322): arg(sum lse_1 conj(lse_0)) over
  // the time between their starts; with compensation every DM-RS symbol is derotated by its start epoch.
  const bool has_cfo = D >= 2;
  float      cfo     = 0.f;
  if (has_cfo) {
    float ar = 0.f, ai = 0.f;
    for (int i = lane; i < N; i += TS) {
      const cpx a = L.Y[NP + i], b = L.Y[i];
      ar += a.x * b.x + a.y * b.y;
      ai += a.y * b.x - a.x * b.y;
    }
    float sums[2] = {ar, ai};
    job_sum_n<T, TS, 2>(sums, redf);
    ar = sums[0];
    ai = sums[1];
    cfo = atan2f(ai, ar) / CHEST_TWOPI / (jb.epochs[jb.dmrs_symbols[1]] - jb.epochs[jb.dmrs_symbols[0]]);
    if (jb.compensate_cfo) {
      for (int s = 0; s < D; ++s) {
        const cpx r = polar1(-CHEST_TWOPI * jb.epochs[jb.dmrs_symbols[s]] * cfo);
        for (int i = lane; i < N; i += TS) {
          L.Y[s * NP + i] = cmul(L.Y[s * NP + i], r);
        }
      }
      job_sync<T>();
    }
  }
  CHEST_STAMP(3);
  const bool rotate = has_cfo && jb.compensate_cfo;
  // Per-symbol CFO rotations e^{j 2 pi epoch_l cfo} of the noise residual, once per job instead of once per pilot.
  __shared__ cpx srot_all[JPW][14];
  cpx* const     srot = srot_all[slot];
  if (rotate) {
    if (lane < 14) {
      srot[lane] = polar1(CHEST_TWOPI * jb.epochs[lane] * cfo);
    }
    job_sync<T>();
  }

  // Planes: "average" combines the DM-RS symbols into one LSE scaled by 1 / (beta D); "interpolate" keeps one per
  // DM-RS symbol scaled by 1 / beta. Each is despread (two-layer groups), then smoothed in frequency into F.
  const float scale = jb.td_interp ? 1.0f / beta : 1.0f / beta / static_cast<float>(D);
  const int   nt    = jb.ntaps;
  const int   c     = nt / 2;
  for (int q = 0; q < Q; ++q) {
    cpx* const E0 = L.E;
    cpx* const E1 = L.E + EN;
    if (GL == 2) {
      for (int j = lane; j < N / 2; j += TS) {
        cpx a = L.Y[q * NP + 2 * j], b = L.Y[q * NP + 2 * j + 1];
        if (!jb.td_interp) {
          for (int s = 1; s < D; ++s) {
            a = {a.x + L.Y[s * NP + 2 * j].x, a.y + L.Y[s * NP + 2 * j].y};
            b = {b.x + L.Y[s * NP + 2 * j + 1].x, b.y + L.Y[s * NP + 2 * j + 1].y};
          }
        }
        const cpx h0 = {(a.x + b.x) * 0.5f * scale, (a.y + b.y) * 0.5f * scale};
        const cpx h1 = {(a.x - b.x) * 0.5f * scale, (a.y - b.y) * 0.5f * scale};
        E0[CHEST_VP + 2 * j] = E0[CHEST_VP + 2 * j + 1] = h0;
        E1[CHEST_VP + 2 * j] = E1[CHEST_VP + 2 * j + 1] = h1;
      }
    } else {
      for (int i = lane; i < N; i += TS) {
        cpx z = L.Y[q * NP + i];
        if (!jb.td_interp) {
          for (int s = 1; s < D; ++s) {
            z = {z.x + L.Y[s * NP + i].x, z.y + L.Y[s * NP + i].y};
          }
        }
        E0[CHEST_VP + i] = {z.x * scale, z.y * scale};
      }
    }
    job_sync<T>();
    for (int ly = 0; ly < GL; ++ly) {
      cpx* E = ly ? E1 : E0;
      cpx* F = Fbase + (q * GL + ly) * NP;
      if (jb.fd == CHEST_FD_FILTER) {
        const int nv = jb.nof_v_pilots;
        if (lane < 64) {  // the first wave (or the job's 2 x TS / 2 lanes) extrapolates both band edges
          virtual_pilots<(TS < 64 ? TS / 2 : 32)>(E, N, nv, lane);
        }
        job_sync<T>();
        for (int i = lane; i < N; i += TS) {
          // Taps j whose input CHEST_VP + i - c + j lies in the enlarged band [CHEST_VP - nv, CHEST_VP + N + nv), in
          // ascending order as the reference's convolution sums them (symmetric taps: correlation == convolution).
          const int j_lo = max(0, c - nv - i);
          const int j_hi = min(nt, N + nv + c - i);
          const cpx* Ei  = E + (CHEST_VP + i - c);
          cpx        acc = {0.f, 0.f};
          for (int j = j_lo; j < j_hi; ++j) {
            const float t = L.taps[j];
            acc.x += t * Ei[j].x;
            acc.y += t * Ei[j].y;
          }
          F[i] = acc;
        }
      } else if (jb.fd == CHEST_FD_MEAN) {
        float sx = 0.f, sy = 0.f;
        for (int i = lane; i < N; i += TS) {
          sx += E[CHEST_VP + i].x;
          sy += E[CHEST_VP + i].y;
        }
        float sums[2] = {sx, sy};
        job_sum_n<T, TS, 2>(sums, redf);
        sx = sums[0] / static_cast<float>(N);
        sy = sums[1] / static_cast<float>(N);
        for (int i = lane; i < N; i += TS) {
          F[i] = {sx, sy};
        }
      } else {
        for (int i = lane; i < N; i += TS) {
          F[i] = E[CHEST_VP + i];
        }
      }
    }
    job_sync<T>();
  }

  CHEST_STAMP(4);
  // RSRP of layer 0 over the planes, and the noise residual (group 0 only) against the time-averaged estimate
  // beta / Q sum_q F_q, re-rotated by the CFO when compensating (estimate_noise, :422).
  float rsrp_acc = 0.f, noise_acc = 0.f;
  for (int i = lane; i < N; i += TS) {
    cpx h = {0.f, 0.f};
    for (int q = 0; q < Q; ++q) {
      const cpx f0 = Fbase[(q * GL) * NP + i];
      rsrp_acc += f0.x * f0.x + f0.y * f0.y;
      cpx hq = f0;
      if (GL == 2) {  // layer 1 carries w_f = -1 on odd pilots
        const cpx  f1 = Fbase[(q * GL + 1) * NP + i];
        const bool od = (i & 1) != 0;
        hq            = {f0.x + (od ? -f1.x : f1.x), f0.y + (od ? -f1.y : f1.y)};
      }
      const float sq = beta / static_cast<float>(Q);
      h              = {hq.x * sq + h.x, hq.y * sq + h.y};
    }
    if (jb.group == 0) {
      const uint32_t k = pilot_subcarrier(jb, crbs, i);
      const int      m = pilot_seq_index(jb, crbs, i);
      for (int s = 0; s < D; ++s) {
        const cpx y = bf16c(grids[jb.grid_base + jb.dmrs_symbols[s] * jb.nsc + k]);
        cpx       q = cmul(h, dmrs_value(jb, lp, L.seq, W, s, n0, m, i));
        if (rotate) {
          q = cmul(q, srot[jb.dmrs_symbols[s]]);
        }
        const float ex = y.x - q.x, ey = y.y - q.y;
        noise_acc += ex * ex + ey * ey;
      }
    }
  }
  const float nof_pilots = static_cast<float>(N * D);
  float       sums3[3]   = {epre_acc, rsrp_acc, noise_acc};
  job_sum_n<T, TS, 3>(sums3, redf);
  const float epre      = sums3[0] / nof_pilots;
  const float rsrp      = sums3[1] * beta * beta * static_cast<float>(D) / static_cast<float>(Q) / nof_pilots;
  const float noise_sum = sums3[2];
  CHEST_STAMP(5);

  // Time alignment of the smoothed layer-0 planes (estimate_time_alignment, port_channel_estimator_helpers.cpp:246 ->
  // time_alignment_estimator_dft_impl): inverse DFT of size M through LDS (radix 2, decimation in frequency), |.|^2
  // summed over the planes at the searched bins, the peak within +-ta_max taps, quadratic refinement unless M is the
  // largest DFT size.
  if (jb.group == 0) {
    const int M   = jb.ta_dft;
    const int lgM = jb.ta_log2;
    job_sync<T>();  // Y / E are dead: the region becomes X / corr
    // Only the bins the search and the quadratic refinement read are needed: n in [0, m + 2) and [M - m - 2, M).
    const int m   = jb.ta_max;
    const int nb  = min(M, 2 * (m + 2));
    auto      bin = [&](int t) { return t < m + 2 ? t : M - nb + t; };
    for (int q = 0; q < Q; ++q) {
      // Natural-order input (the pilots at their positions, zeros elsewhere): decimation in frequency leaves the
      // output in bit-reversed order, read back only at the bins above.
      const cpx* Fq = Fbase + (q * GL) * NP;
      if (!jb.ta_positions) {
        for (int n = lane; n < M; n += TS) {
          L.X[n] = n < N ? Fq[n] : cpx{0.f, 0.f};
        }
      } else {
        for (int n = lane; n < M; n += TS) {
          L.X[n] = {0.f, 0.f};
        }
        job_sync<T>();
        const uint32_t k0 = pilot_subcarrier(jb, crbs, 0);
        for (int i = lane; i < N; i += TS) {
          L.X[pilot_subcarrier(jb, crbs, i) - k0] = Fq[i];
        }
      }
      job_sync<T>();
      CHEST_STAMP(8);
      // Radix-2 decimation in frequency, inverse sign, two stages per barrier: a lane takes the four elements
      // i0 + {0, h, 2h, 3h} through the stage of span 2h (twiddles e^{+j 2 pi j' / 4h}, j' = j, j + h) and the stage of
      // span h (e^{+j 2 pi j / 2h}) in registers.
      auto twiddle = [](int j, int span2) {  // e^{+j 2 pi j / span2} (revolutions)
        const float r = static_cast<float>(j) / static_cast<float>(span2);
        return cpx{__builtin_amdgcn_cosf(r), __builtin_amdgcn_sinf(r)};
      };
      int lh = lgM - 1;
      for (; lh >= 1; lh -= 2) {
        const int h = 1 << (lh - 1);
        for (int b = lane; b < M / 4; b += TS) {
          const int j  = b & (h - 1);
          const int i0 = ((b >> (lh - 1)) << (lh + 1)) + j;
          const cpx x0 = L.X[i0], x1 = L.X[i0 + h], x2 = L.X[i0 + 2 * h], x3 = L.X[i0 + 3 * h];
          const cpx y0 = {x0.x + x2.x, x0.y + x2.y};
          const cpx y2 = cmul({x0.x - x2.x, x0.y - x2.y}, twiddle(j, 4 * h));
          const cpx y1 = {x1.x + x3.x, x1.y + x3.y};
          const cpx y3 = cmul({x1.x - x3.x, x1.y - x3.y}, twiddle(j + h, 4 * h));
          const cpx w1 = twiddle(j, 2 * h);
          L.X[i0]         = {y0.x + y1.x, y0.y + y1.y};
          L.X[i0 + h]     = cmul({y0.x - y1.x, y0.y - y1.y}, w1);
          L.X[i0 + 2 * h] = {y2.x + y3.x, y2.y + y3.y};
          L.X[i0 + 3 * h] = cmul({y2.x - y3.x, y2.y - y3.y}, w1);
        }
        job_sync<T>();
      }
      if (lh == 0) {  // odd number of stages: the last one (span 1, unit twiddle) alone
        for (int b = lane; b < M / 2; b += TS) {
          const cpx a = L.X[2 * b], c = L.X[2 * b + 1];
          L.X[2 * b]     = {a.x + c.x, a.y + c.y};
          L.X[2 * b + 1] = {a.x - c.x, a.y - c.y};
        }
        job_sync<T>();
      }
      CHEST_STAMP(9);
      for (int t = lane; t < nb; t += TS) {
        const int   n = bin(t);
        const cpx   v = L.X[__brev(static_cast<uint32_t>(n)) >> (32 - lgM)];
        const float p = v.x * v.x + v.y * v.y;
        L.corr[n]     = q ? L.corr[n] + p : p;
      }
      job_sync<T>();
    }
    float     dv = -INFINITY, av = -INFINITY;
    int       di = 0x7fffffff, ai = 0x7fffffff;
    for (int n = lane; n < m; n += TS) {
      if (L.corr[n] > dv) {
        dv = L.corr[n];
        di = n;
      }
      if (L.corr[M - m + n] > av) {
        av = L.corr[M - m + n];
        ai = n;
      }
    }
    job_argmax2<T, TS>(dv, di, av, ai, redf, redi);
    const int idx  = (dv >= av) ? di : -(m - ai);
    float     frac = 0.f;
    if (M != 4096) {
      const int nt5 = (m > 2) ? 5 : 3;
      float     num, den, corr_k;
      auto      cv = [&](int i) { return L.corr[(idx + i - nt5 / 2) & (M - 1)]; };
      if (nt5 == 5) {
        num    = -0.4f * cv(0) + -0.2f * cv(1) + 0.0f * cv(2) + 0.2f * cv(3) + 0.4f * cv(4);
        den    = 0.571429f * cv(0) + -0.285714f * cv(1) + -0.571429f * cv(2) + -0.285714f * cv(3) + 0.571429f * cv(4);
        corr_k = 1.0f;
      } else {
        num    = -0.5f * cv(0) + 0.0f * cv(1) + 0.5f * cv(2);
        den    = 0.5f * cv(0) + -1.0f * cv(1) + 0.5f * cv(2);
        corr_k = 0.5f;
      }
      const float r = -corr_k * num / den;
      frac          = (isnan(r) || isinf(r) || fabsf(r) > 1.0f) ? 0.f : r;
    }
    // phy_time_unit::from_seconds of the float seconds: Tc units truncated at x10, then rounded half away.
    const float   ta_f = static_cast<float>((static_cast<double>(idx) + static_cast<double>(frac)) / jb.ta_fs);
    const double  t_c  = 1.0 / (480000.0 * 4096.0);
    const int64_t tc10 = static_cast<int64_t>(static_cast<double>(ta_f) / t_c * 10.0);
    const float   ta_s = static_cast<float>(static_cast<double>(tc10 / 10 + (tc10 % 10) / 5) * t_c);
    CHEST_STAMP(6);
    if (lane == 0) {
      const float nv = fmaxf(rsrp / 1e10f, noise_sum / (nof_pilots - 1.f));
      noise_var[jb.noise_slot] = nv;
      if (metrics != nullptr) {
        float* mt = metrics + CHEST_METRICS * jb.noise_slot;
        mt[0]     = rsrp;
        mt[1]     = epre;
        mt[2]     = nv;
        mt[3]     = (nv != 0.f) ? rsrp / beta / beta / nv : 1000.f;
        mt[4]     = ta_s;
        mt[5]     = has_cfo ? cfo * jb.scs_hz : __builtin_nanf("");
        mt[6]     = 0.f;
        mt[7]     = 0.f;
      }
    }
  }

  // Estimates of every RE of the allocation: linear frequency interpolation of the planes; "interpolate" then
  // interpolates in time between the planes around each symbol (host table); bf16, then the CFO rotation of each
  // symbol by its start epoch in bf16 like sc_prod on the channel_estimate (:128). The compact layout writes the
  // unrotated row of start_symbol and, with compensation, the CFO (float bits) in the first element of the next row.
  const int nre    = jb.nof_rb * 12;
  const int offset = jb.interp_offset;
  const int stride = jb.interp_stride;
  const int last   = offset + (N - 1) * stride;
  auto      freq   = [&](const cpx* F, int k) -> cpx {
    if (k <= offset) {
      return F[0];
    }
    if (k >= last) {
      return F[N - 1];
    }
    const int   i = stride == 2 ? (k - offset) >> 1 : (k - offset) / stride;  // k > offset here
    const float w = static_cast<float>((k - offset) - i * stride) / static_cast<float>(stride);
    const cpx   a = F[i], b = F[i + 1];
    return {(b.x - a.x) * w + a.x, (b.y - a.y) * w + a.y};
  };
  const bool rotate_out = rotate && !jb.compact_cfo;
  for (int k = lane; k < nre; k += TS) {
    // PRB k / 12 of the interpolated band is the (k / 12)-th allocated CRB (compute_hop maps the band PRB by PRB).
    const int kr = alloc_rb(jb, crbs, k / 12) * 12 + k % 12;
    for (int ly = 0; ly < GL; ++ly) {
      uint32_t* dst = ce + jb.ce_base + ly * jb.ce_layer_stride + static_cast<uint32_t>(kr);
      const cpx v0  = freq(Fbase + ly * NP, k);
      for (int r = 0; r < jb.nof_out_symbols; ++r) {
        const int l = jb.first_symbol + r;
        cpx       v = v0;
        if (jb.td_interp) {
          const cpx   a = freq(Fbase + (jb.td_q0[l] * GL + ly) * NP, k);
          const cpx   b = freq(Fbase + (jb.td_q1[l] * GL + ly) * NP, k);
          const float w = jb.td_w[l];
          v             = {a.x + (b.x - a.x) * w, a.y + (b.y - a.y) * w};
        }
        uint32_t u = to_bf16c(v);
        if (rotate_out) {
          // srot[l] is polar1(CHEST_TWOPI * epochs[l] * cfo), the expression the demodulator evaluates for the
          // compact layout, so both layouts round identically (one sincos per symbol instead of per estimate).
          const cpx h = bf16c(u);
          cpx       r;
          cmul_fused(h.x, h.y, srot[l].x, srot[l].y, r.x, r.y);
          u = to_bf16c(r);
        }
        dst[l * jb.nsc] = u;
      }
      if (jb.compact_cfo && k == 0) {
        dst[(jb.first_symbol + 1) * jb.nsc] = __float_as_uint(has_cfo ? cfo : 0.f);
      }
    }
  }
  CHEST_STAMP(7);
  CHEST_PROF(11, __builtin_amdgcn_s_memrealtime());
}

} // namespace

#ifdef CHEST_PROFILE
int debug_read_chest_profile(uint64_t* dst, size_t n)
{
  const size_t max = static_cast<size_t>(CHEST_PROF_JOBS) * CHEST_PROF_SLOTS;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_chest_prof), (n < max ? n : max) * sizeof(uint64_t)) == hipSuccess ? 0
                                                                                                                  : -1;
}
#endif

size_t pusch_chest_lds_bytes(const chest_geom& g)
{
  return chest_job_lds_bytes(g);
}

void launch_pusch_chest(const float2*   d_lp,
                        const uint16_t* d_crbs,
                        const chest_job* d_jobs,
                        int              nof_jobs,
                        const chest_geom& geom,
                        const uint32_t*  d_grids,
                        uint32_t*        d_ce,
                        float*           d_noise_var,
                        float*           d_metrics,
                        const uint32_t*  d_seq,
                        hipStream_t      stream,
                        const srsgpu_copy_span* d_spans,
                        int              nof_spans,
                        uint64_t         span_bytes)
{
  if (nof_jobs <= 0) {
    return;
  }
  const size_t lds = chest_job_lds_bytes(geom);
  // Copy workgroups: per span, enough for one 16-byte vector per lane of the largest span (a read from mapped host
  // memory is a PCIe round trip: the copy's rate is its requests in flight).
  const auto copy_blocks = [&](int threads) {
    if (nof_spans <= 0) {
      return 0;
    }
    const uint64_t per_span = std::max<uint64_t>(1, (span_bytes / 16u + threads - 1) / threads);
    return static_cast<int>(per_span * static_cast<uint64_t>(nof_spans));
  };
  // Two jobs per wave (32 lanes each) for the usual few-RB allocations (many jobs resident together); a job with
  // hundreds of pilots (a wideband allocation: few jobs, each a long serial chain on one wave) spreads over 4 or 16
  // waves (two jobs per wave against one: chest stage 51 -> 42 us per step, profiles/r3_chest_two_jobs_per_wave_ab.json).
  const auto launch = [&](auto kernel, int threads, int jpw) {
    hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>((nof_jobs + jpw - 1) / jpw + copy_blocks(threads))),
                       dim3(static_cast<unsigned>(threads)), static_cast<unsigned>(jpw * lds), stream, d_jobs, nof_jobs,
                       geom, d_grids, d_ce, d_noise_var, d_metrics, d_seq, d_crbs, d_lp, d_spans, nof_spans);
  };
  if (geom.max_pilots > 512) {
    launch(pusch_chest_kernel<1024, 1024>, 1024, 1);
  } else if (geom.max_pilots > 128) {
    launch(pusch_chest_kernel<256, 256>, 256, 1);
  } else if (geom.max_pilots <= 64 && 2 * lds <= 64 * 1024) {
    launch(pusch_chest_kernel<CHEST_THREADS, CHEST_THREADS / 2>, CHEST_THREADS, 2);
  } else {
    launch(pusch_chest_kernel<CHEST_THREADS, CHEST_THREADS>, CHEST_THREADS, 1);
  }
}

} // namespace srsgpu
