// PDSCH modulator on gfx950: scrambling + modulation mapping + layer mapping + wideband precoding + RE mapping into
// bf16 resource grids, for every PDSCH transmission of a batch of slots.
//
// Reference (behaviour, not code): lib/phy/upper/channel_processors/pdsch/pdsch_modulator_impl.cpp:107 (modulate),
// :30 (scramble), modulation_mapper_lut_impl.cpp:39 (constellations), support/resource_grid_mapper_impl.cpp:269 (RE
// order), generic_functions/precoding/channel_precoder_generic.cpp:51 (precoding), adt/bf16.h:39 (rounding).
//
// Work decomposition: a workgroup owns 8192 codeword bits (256 words) of one transmission. Its four waves first stage
// the scrambled words in LDS — codeword XOR the plan's precomputed scrambling sequence (filled once at plan creation
// by gold_fill_kernel, which evaluates the Gold sequence at any position by jumping the x2 LFSR state with
// precomputed GF(2) matrices and reading x1 from a table: the sequence depends only on c_init and the length, so the
// steady state reads one resident word per codeword word instead of recomputing the jumps) — then every lane takes one RE whose bits start in the chunk: it forms
// the L constellation points, precodes them for every port and stores one (re, im) bf16 pair per port. Consecutive
// lanes hold consecutive REs of a symbol, so the grid stores are coalesced 4-byte writes. HBM-bound: the codeword is
// read once (1 bit per bit) and every PDSCH RE of every port is written once (4 B).
//
// Floating point follows the reference exactly: every complex product term is rounded separately (no contraction),
// layer terms are summed in layer order and the result is rounded to bf16 half-to-even.
#include "gold_device.h"
#include "srsgpu_internal.h"

#pragma clang fp contract(off)

namespace srsgpu {
namespace {

constexpr int MOD_THREADS = 256;

/// Scrambled codeword word w (bits 32w..32w+31, MSB first) of a transmission: the plan's precomputed sequence word.
__device__ __forceinline__ uint32_t scrambled_word(const mod_desc& d,
                                                   const uint32_t* __restrict__ cw,
                                                   const uint32_t* __restrict__ seq,
                                                   uint32_t w)
{
  return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(cw) +
                                                              (d.cw_word_offset + w) * 4u)) ^
         *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(seq) + (d.seq_word_offset + w) * 4u);
}

/// Plan-time fill of the (de)scrambling sequences (launch_gold_fill): Gold sequence by GF(2) jumps.
__global__ __launch_bounds__(MOD_THREADS) void gold_fill_kernel(const uint32_t* __restrict__ c_inits,
                                                                 const uint32_t* __restrict__ offsets,
                                                                 const uint32_t* __restrict__ nwords,
                                                                 const uint32_t* __restrict__ wstart,
                                                                 uint32_t* __restrict__ seq,
                                                                 const uint32_t* __restrict__ x1,
                                                                 const uint32_t* __restrict__ x2_jump,
                                                                 const uint32_t* __restrict__ x2_lane)
{
  const uint32_t t = blockIdx.y;
  const uint32_t i = blockIdx.x * MOD_THREADS + threadIdx.x;
  if (i < nwords[t]) {
    const uint32_t w = (wstart != nullptr ? wstart[t] : 0u) + i;
    seq[offsets[t] + i] = gold_word(c_inits[t], w, w >> 6, x1, x2_jump, x2_lane);
  }
}

__device__ __forceinline__ uint32_t to_bf16_bits(float v)
{
  const uint32_t u = __float_as_uint(v);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

/// Constellation point of a Qm-bit index on the TS 38.211 section 5.1 integer grid (Gray mapping; the amplitude is in
/// the precoding weights): bit pairs (2j + 1, 2j) from the least significant pick the signs of the real and imaginary
/// parts after j + 1 levels (the reference's modulation_mapper_lut_impl.cpp tables hold the same points).
__device__ __forceinline__ float2 constellation_point(uint32_t idx, uint32_t qm)
{
  int re = 0, im = 0, off = -1;
  for (uint32_t j = 0; j < qm / 2; ++j) {
    re += off;
    im += off;
    off *= 2;
    re = ((idx >> (2 * j + 1)) & 1u) ? re : -re;
    im = ((idx >> (2 * j)) & 1u) ? im : -im;
  }
  return make_float2(static_cast<float>(re), static_cast<float>(im));
}

/// The chunk's REs: modulation, layer mapping, precoding and mapping. MAP: general allocation (the plan's RE ->
/// subcarrier map); PRG: per-PRG precoding weights (resource_grid_mapper_impl.cpp:218). points: the transmission's
/// 2^Qm constellation points, staged in LDS by the workgroup (one LDS read per layer and RE).
template <bool MAP, bool PRG>
__device__ __forceinline__ void modulate_res(const mod_desc& d,
                                             const mod_chunk& ch,
                                             const uint32_t*  bits,
                                             const float2*    points,
                                             const uint16_t* __restrict__ sc_map,
                                             const float* __restrict__ prg_w,
                                             uint32_t* __restrict__ grids)
{
  const uint32_t tid = threadIdx.x;
  const uint32_t qm = d.qm, L = d.L, P = d.P, Lq = L * qm;
  const uint32_t qmask = (1u << qm) - 1u;
  float          w[4][4][2];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      w[p][l][0] = d.w[p][l][0];
      w[p][l][1] = d.w[p][l][1];
    }
  }

  // OFDM symbol of the lane's current RE (allocation order: symbol-major, ascending subcarrier) and the first RE of
  // the next symbol: a lane's REs are MOD_THREADS apart, so the symbol search runs only when a lane crosses into a
  // later symbol.
  uint32_t l = 0, next = 0;
  for (uint32_t r = ch.re_begin + tid; r < ch.re_end; r += MOD_THREADS) {
    // The RE's L * Qm bits, left-aligned in 64 bits.
    const uint32_t o  = r * Lq - ch.word0 * 32u;
    const uint32_t wi = o >> 5;
    const uint64_t b  = ((static_cast<uint64_t>(bits[wi]) << 32) | bits[wi + 1]) << (o & 31u);

    if (r >= next) {
      l    = 0;
      next = 0xffffffffu;
#pragma unroll
      for (int j = 1; j < 15; ++j) {
        const uint32_t c = d.sym_cum[j];
        l += (c <= r) ? 1u : 0u;
        next = (c > r && c < next) ? c : next;
      }
    }
    const uint32_t k = r - d.sym_cum[l];
    uint32_t       sc;
    if constexpr (MAP) {
      // General allocation (CRB mask, reserved REs, PRG precoding): the plan's RE -> grid subcarrier map (grid_base
      // at CRB 0, so sc is the absolute subcarrier the PRG index below needs).
      sc = sc_map[d.sc_map + r];
    } else if ((d.dmrs_mask >> l) & 1u) {
      const uint32_t nd  = d.nd_dmrs;
      const uint32_t prb = k / nd;
      const uint32_t j   = k - prb * nd;
      sc                 = prb * 12u + static_cast<uint32_t>((d.dmrs_lut >> (4u * j)) & 15u);
    } else {
      sc = k;
    }
    const uint32_t e = d.grid_base + l * d.nsc + sc;
    // Per-PRG precoding: the weights of the PRG holding the RE's subcarrier.
    const float* wt = PRG ? prg_w + d.prg_w + (sc / d.prg_sc) * 32u : nullptr;

    // Constellation points of the layers.
    float xr[4], xi[4];
#pragma unroll
    for (int ly = 0; ly < 4; ++ly) {
      if (ly < static_cast<int>(L)) {
        const float2 x = points[static_cast<uint32_t>(b >> (64u - (ly + 1) * qm)) & qmask];
        xr[ly]         = x.x;
        xi[ly]         = x.y;
      }
    }

    // Precoding: port p gets sum over layers of x_l * w(p, l).
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p < static_cast<int>(P)) {
        float sr = 0.f, si = 0.f;
#pragma unroll
        for (int ly = 0; ly < 4; ++ly) {
          if (ly < static_cast<int>(L)) {
            const float wr = PRG ? wt[(p * 4 + ly) * 2] : w[p][ly][0];
            const float wi = PRG ? wt[(p * 4 + ly) * 2 + 1] : w[p][ly][1];
            const float pr = xr[ly] * wr - xi[ly] * wi;
            const float pi = xr[ly] * wi + xi[ly] * wr;
            sr             = (ly == 0) ? pr : sr + pr;
            si             = (ly == 0) ? pi : si + pi;
          }
        }
        // (an unsigned 32-bit byte offset from the grid's SGPR base: saddr stores)
        *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(grids) + (e + static_cast<uint32_t>(p) * d.port_stride) * 4u) =
            to_bf16_bits(sr) | (to_bf16_bits(si) << 16);
      }
    }
  }
}

__global__ __launch_bounds__(MOD_THREADS) void pdsch_modulate_kernel(const mod_desc* __restrict__ descs,
                                                                      const uint16_t* __restrict__ sc_map,
                                                                      const float* __restrict__ prg_w,
                                                                      const mod_chunk* __restrict__ chunks,
                                                                      const uint32_t* __restrict__ cw,
                                                                      uint32_t* __restrict__ grids,
                                                                      const uint32_t* __restrict__ seq)
{
  __shared__ uint32_t bits[MOD_CHUNK_WORDS + 1];
  __shared__ float2   points[256];
  const mod_chunk ch  = chunks[blockIdx.x];
  const mod_desc& d   = descs[ch.tx];
  const uint32_t  tid = threadIdx.x;
  const uint32_t  nwords = (d.nof_bits + 31u) >> 5;
  static_assert(MOD_THREADS >= 256, "one constellation point per lane");
  if (tid < (1u << d.qm)) {
    points[tid] = constellation_point(tid, d.qm);
  }

  // Stage the chunk's scrambled words (and the first word of the next chunk, for an RE straddling the boundary).
  for (uint32_t j = tid; j < MOD_CHUNK_WORDS; j += MOD_THREADS) {
    const uint32_t w = ch.word0 + j;
    bits[j]          = (w < nwords) ? scrambled_word(d, cw, seq, w) : 0u;
  }
  {
    if (tid == 0) {
      const uint32_t w2 = ch.word0 + MOD_CHUNK_WORDS;
      bits[MOD_CHUNK_WORDS] = (w2 < nwords) ? scrambled_word(d, cw, seq, w2) : 0u;
    }
  }

  __syncthreads();
  // One instantiation per allocation kind, chosen per workgroup (uniform): the contiguous wideband path keeps its
  // weights in registers and its subcarrier arithmetic; the general path reads the RE -> subcarrier map and, with
  // PRGs, the PRG's weights.
  if (d.sc_map == NO_SC_MAP) {
    modulate_res<false, false>(d, ch, bits, points, sc_map, prg_w, grids);
  } else if (d.prg_sc == 0) {
    modulate_res<true, false>(d, ch, bits, points, sc_map, prg_w, grids);
  } else {
    modulate_res<true, true>(d, ch, bits, points, sc_map, prg_w, grids);
  }
}

/// PDSCH DM-RS (dmrs_pdsch_processor_impl.cpp:56 sequence, :80 cover codes, :117 per-CDM-group precoding and
/// mapping): lane i owns DM-RS index i of the symbol in every CDM group. Same rounding as the modulator.
__global__ __launch_bounds__(MOD_THREADS) void pdsch_dmrs_kernel(const dmrs_job* __restrict__ jobs,
                                                                  uint32_t* __restrict__ grids,
                                                                  const uint32_t* __restrict__ gseq)
{
  const dmrs_job& jb     = jobs[blockIdx.x];
  const uint32_t  per_rb = jb.type2 ? 4u : 6u;
  const uint32_t  wfirst = (2 * jb.seq_offset) >> 5;
  // blockIdx.y: a wideband job's pilots are spread over several workgroups (one loop trip each).
  for (uint32_t i = threadIdx.x + blockIdx.y * blockDim.x; i < jb.nof_pilots; i += blockDim.x * gridDim.y) {
    const uint32_t n    = 2 * (jb.seq_offset + i);
    const uint32_t w    = n >> 5;
    const uint32_t word = gseq[jb.gseq_base + (w - wfirst)];  // the plan's resident sequence words
    const uint32_t sh   = 31u - (n & 31u);
    const float    re   = ((word >> sh) & 1u) ? -jb.amp : jb.amp;
    const float    im   = ((word >> (sh - 1)) & 1u) ? -jb.amp : jb.amp;
    const uint32_t rb   = i / per_rb, j = i - rb * per_rb;
    for (uint32_t g = 0; 2 * g < jb.L; ++g) {
      // Subcarrier of DM-RS j of the RB in CDM group g (type 1: 2j + g; type 2: 6 (j / 2) + 2g + j % 2).
      const uint32_t k = rb * 12u + (jb.type2 ? 6u * (j >> 1) + 2u * g + (j & 1u) : 2u * j + g);
      // Cover codes: w_f = (+1, -1) for odd ports on odd indices; w_t = -1 for ports >= 4 when l' = 1 (none here:
      // at most four layers, ports 0..3).
      const float s1 = (i & 1u) ? -1.f : 1.f;
      const uint32_t q0 = 2 * g, q1 = 2 * g + 1;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (p < static_cast<int>(jb.P)) {
          const float wr0 = jb.w[p][q0][0], wi0 = jb.w[p][q0][1];
          float       sr  = re * wr0 - im * wi0;
          float       si  = re * wi0 + im * wr0;
          if (q1 < jb.L) {
            const float a = re * s1, b = im * s1;
            const float wr1 = jb.w[p][q1][0], wi1 = jb.w[p][q1][1];
            sr = sr + (a * wr1 - b * wi1);
            si = si + (a * wi1 + b * wr1);
          }
          grids[jb.grid_base + static_cast<uint32_t>(p) * jb.port_stride + k] =
              to_bf16_bits(sr) | (to_bf16_bits(si) << 16);
        }
      }
    }
  }
}

} // namespace

void launch_pdsch_dmrs(const dmrs_job* d_jobs,
                       int             nof_jobs,
                       int             max_pilots,
                       uint32_t*       d_grids,
                       const uint32_t* d_seq,
                       hipStream_t     stream)
{
  if (nof_jobs <= 0) {
    return;
  }
  // One wave per job for few-RB allocations (a 4-5 RB job has 24-30 pilots: a 256-lane workgroup left 7 of 8 lanes
  // idle), 256 lanes and more workgroups per job for wideband ones.
  const int      threads = max_pilots <= 64 ? 64 : MOD_THREADS;
  const unsigned ny      = static_cast<unsigned>((max_pilots + threads - 1) / threads);
  hipLaunchKernelGGL(pdsch_dmrs_kernel, dim3(static_cast<unsigned>(nof_jobs), ny > 0 ? ny : 1u),
                     dim3(static_cast<unsigned>(threads)), 0,
                     stream, d_jobs, d_grids, d_seq);
}

void launch_pdsch_modulate(const mod_desc*  d_desc,
                           const uint16_t*  d_sc_map,
                           const float*     d_prg_w,
                           const mod_chunk* d_chunks,
                           int              nof_chunks,
                           const uint32_t*  d_codewords,
                           uint32_t*        d_grids,
                           const uint32_t*  d_seq,
                           hipStream_t      stream)
{
  if (nof_chunks <= 0) {
    return;
  }
  hipLaunchKernelGGL(pdsch_modulate_kernel, dim3(static_cast<unsigned>(nof_chunks)), dim3(MOD_THREADS), 0, stream,
                     d_desc, d_sc_map, d_prg_w, d_chunks, d_codewords, d_grids, d_seq);
}

void launch_gold_fill(const uint32_t* d_c_inits,
                      const uint32_t* d_offsets,
                      const uint32_t* d_nwords,
                      const uint32_t* d_wstart,
                      int             nof_tx,
                      uint32_t        max_nwords,
                      uint32_t*       d_seq,
                      const uint32_t* d_x1,
                      const uint32_t* d_x2_jump,
                      const uint32_t* d_x2_lane,
                      hipStream_t     stream)
{
  if (nof_tx <= 0 || max_nwords == 0) {
    return;
  }
  const dim3 grid((max_nwords + MOD_THREADS - 1) / MOD_THREADS, static_cast<unsigned>(nof_tx));
  hipLaunchKernelGGL(gold_fill_kernel, grid, dim3(MOD_THREADS), 0, stream, d_c_inits, d_offsets, d_nwords, d_wstart,
                     d_seq, d_x1, d_x2_jump, d_x2_lane);
}

} // namespace srsgpu
