// Batched LDPC decoder for 5G NR (TS 38.212 BG1/BG2), layered normalised min-sum on 8-bit LLRs, for gfx950.
//
// Drop-in semantics of srsran::ldpc_decoder::decode (reference lib/phy/upper/channel_coding/ldpc/
// ldpc_decoder_impl.cpp:60): same trimming of the input, same soft-bit clamp (:152), same layer schedule, same
// check-node arithmetic (ldpc_decoder_avx2.cpp:69/:111/:165/:205, or ldpc_decoder_generic.cpp for MODE 0), same CRC
// early stop after every full iteration (:133) and the same hard-decision output. Results are bit-exact with the
// reference on identical inputs (tests/test_ldpc_decoder_gpu.py).
//
// Mapping to CDNA4:
//  * one workgroup decodes one codeblock; lane z (0 <= z < Z) owns lifted check row z of every layer, so a layer is
//    Z independent check-node updates (a circulant permutation guarantees no two lanes touch the same soft bit);
//  * the soft bits of the whole codeblock live in LDS (68 x 384 B for BG1); column c of the lifted graph sits at
//    c * 384, so every column offset is a ds_read/ds_write immediate;
//  * the check-to-variable messages never leave the VGPRs: per layer a lane keeps the scaled minimum, second minimum,
//    argmin and one sign bit per edge (one 32-bit word, two for the 19-edge core rows of BG1) - the messages are
//    rebuilt from them exactly;
//  * the base-graph structure (edges per layer, columns) is unrolled at compile time; only the lifting shifts are
//    read at run time (wave-uniform loads).
#include "common.h"
#include "ldpc_base_graphs.h"
#include "srsgpu_internal.h"
#include "ldpc_decoder_common.h"

namespace srsgpu {
namespace {
using namespace ldpc_dec;

constexpr int LDPC_DEC_MIN_WAVES = 4;

#ifdef LDPC_DEC_PROFILE
// Instrumented build only (SRSGPU_EXTRA_FLAGS=-DLDPC_DEC_PROFILE): per-codeblock s_memtime stamps of the decoder
// phases, read back with srsgpu_debug_decoder_profile (tools/decoder_phase_profile.py).
__device__ uint64_t g_dec_prof[LDPC_DEC_PROF_CBS * LDPC_DEC_PROF_SLOTS];
#define DEC_PROF(slot, value)                                                                                          \
  do {                                                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < LDPC_DEC_PROF_CBS) {                                                          \
      g_dec_prof[blockIdx.x * LDPC_DEC_PROF_SLOTS + (slot)] = (value);                                                 \
    }                                                                                                                  \
  } while (0)
#else
#define DEC_PROF(slot, value)                                                                                          \
  do {                                                                                                                 \
  } while (0)
#endif
#define DEC_STAMP(slot) DEC_PROF(slot, __builtin_amdgcn_s_memtime())

/// One lifted check row of layer m: variable-to-check messages, min-sum analysis, check-to-variable messages and the
/// soft-bit update (ldpc_decoder_impl.cpp:195, :255, :240).
template <int BG, int MODE, int m>
__device__ __forceinline__ void row_update(int8_t* __restrict__ soft,
                                           const_u32_ptr sh,  // lifting shifts of this Z
                                           int           z,
                                           int           Z,
                                           uint32_t      sf16,
                                           float         sf,
                                           uint32_t&     st,
                                           uint32_t&     st_hi)
{
  using G            = bg_t<BG>;
  constexpr int e0   = G::rs(m);
  constexpr int deg  = G::rs(m + 1) - e0;
  const int     om1  = static_cast<int>(st & 127u);
  const int     om2  = static_cast<int>((st >> 7) & 127u);
  const int     oidx = static_cast<int>((st >> 14) & 31u);
  int           v2c[deg];
  uint32_t      k1 = KEY_INIT, k2 = KEY_INIT;  // two smallest keys
  uint32_t      sx = 0;                        // sign parity in bit 31
  // Sign bits of edges >= SIGNS_LO of the (at most four) high-degree core rows share one word, 6 bits per row.
  constexpr int HI_SHIFT = 6 * (m & 3);

  static_for<deg>([&](auto E) {
    constexpr int e   = decltype(E)::value;
    constexpr int col = G::col(e0 + e);
    // Rotated position (z + s) mod Z with one unsigned min: z + s - Z wraps above z + s when z + s < Z.
    const uint32_t p0 = static_cast<uint32_t>(z) + sh[e0 + e];
    const uint32_t p1 = p0 - static_cast<uint32_t>(Z);
    const int      p  = static_cast<int>(p0 < p1 ? p0 : p1);
    const int      sb = soft[col * SOFT_COL_STRIDE + p];
    // Previous check-to-variable message of this edge, rebuilt from the compressed state (n = 0 or -1: its sign).
    int n;
    if constexpr (e < SIGNS_LO) {
      n = static_cast<int>(st << (12 - e)) >> 31;
    } else {
      n = static_cast<int>(st_hi << (31 - (HI_SHIFT + e - SIGNS_LO))) >> 31;
    }
    const int om = (oidx == e) ? om2 : om1;
    const int c  = (om ^ n) - n;
    // v2c = soft - c2v saturated to +/-LLR_MAX; infinite soft bits stay infinite (ldpc_decoder_avx2.cpp:69): they
    // get |v2c| >= 392, never a minimum, and saturate back to infinity in the update.
    const int fin = clamp_i(sb, -LLR_MAX, LLR_MAX);
    const int v   = clamp_i(sb - c, -LLR_MAX, LLR_MAX) + ((sb - fin) << 9);
    v2c[e]        = v;
    // Two smallest magnitudes and argmin (ldpc_decoder_avx2.cpp:111) on keys |v| << 5 | e; sign parity by XOR.
    const uint32_t key = (static_cast<uint32_t>(v < 0 ? -v : v) << 5) | static_cast<uint32_t>(e);
    k2                 = umed3(key, k1, k2);
    k1                 = key < k1 ? key : k1;
    sx ^= static_cast<uint32_t>(v);
  });

  const int idx = static_cast<int>(k1 & 31u);
  const int s1  = scale_mag<MODE>(static_cast<int>(k1 >> 5), sf16, sf);
  const int s2  = scale_mag<MODE>(static_cast<int>(k2 >> 5), sf16, sf);
  uint32_t  nst = static_cast<uint32_t>(s1) | (static_cast<uint32_t>(s2) << 7) | (static_cast<uint32_t>(idx) << 14);
  uint32_t  nhi = 0;

  static_for<deg>([&](auto E) {
    constexpr int e   = decltype(E)::value;
    constexpr int col = G::col(e0 + e);
    const int     v   = v2c[e];
    // c2v sign = product of the other edges' signs (ldpc_decoder_avx2.cpp:165).
    const int n   = static_cast<int>(sx ^ static_cast<uint32_t>(v)) >> 31;
    const int mag = (idx == e) ? s2 : s1;
    const int c   = (mag ^ n) - n;
    // Promotion sum (log_likelihood_ratio.cpp:75, ldpc_decoder_avx2.cpp:205): |sum| > LLR_MAX becomes +/-infinity.
    const int      sb = clamp_i(c + v, -SOFT_INF, SOFT_INF);
    const uint32_t p0 = static_cast<uint32_t>(z) + sh[e0 + e];
    const uint32_t p1 = p0 - static_cast<uint32_t>(Z);
    soft[col * SOFT_COL_STRIDE + static_cast<int>(p0 < p1 ? p0 : p1)] = static_cast<int8_t>(sb);
    if constexpr (e < SIGNS_LO) {
      nst |= static_cast<uint32_t>(n) & (1u << (19 + e));
    } else {
      nhi |= static_cast<uint32_t>(n) & (1u << (HI_SHIFT + e - SIGNS_LO));
    }
  });
  st = nst;
  if constexpr (deg > SIGNS_LO) {
    static_assert(m < 4 && deg - SIGNS_LO <= 6, "only the core rows may exceed SIGNS_LO edges");
    st_hi = (st_hi & ~(0x3fu << HI_SHIFT)) | nhi;
  }
}

/// Hard decisions of the K*Z systematic bits, packed MSB first (log_likelihood_ratio.cpp:350 hard_decision).
__device__ __forceinline__ void write_hard_bits(const int8_t* __restrict__ soft,
                                                uint8_t* __restrict__ out,
                                                int      nbits,
                                                int      Z,
                                                uint32_t magic)
{
  const int nbytes = (nbits + 7) / 8;
  for (int b = threadIdx.x; b < nbytes; b += blockDim.x) {
    uint32_t byte = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = 8 * b + k;
      if (i < nbits) {
        const int col = static_cast<int>(__umulhi(static_cast<uint32_t>(i), magic));
        const int l   = i - col * Z;
        byte |= static_cast<uint32_t>(soft[col * SOFT_COL_STRIDE + l] <= 0) << (7 - k);
      }
    }
    out[b] = static_cast<uint8_t>(byte);
  }
}

template <int BG, int MODE>
__global__ __launch_bounds__(384, LDPC_DEC_MIN_WAVES) void ldpc_decode_kernel(const dec_desc* __restrict__ descs,
                                                          const int8_t* __restrict__ llrs,
                                                          uint8_t* __restrict__ out,
                                                          int32_t* __restrict__ results,
                                                          const uint32_t* __restrict__ shift_table,
                                                          const uint32_t* __restrict__ crc_tables,
                                                          uint8_t* __restrict__ cb_crc_ok,
                                                          int8_t* const* __restrict__ llr_cbs)
{
  using G = bg_t<BG>;
  // Static LDS: its base is a link-time constant, so every soft-bit access is (lane offset + immediate).
  __shared__ __attribute__((aligned(16))) int8_t smem[G::NF * SOFT_COL_STRIDE + SCRATCH_BYTES];
  int8_t*   soft    = smem;
  int*      scratch = reinterpret_cast<int*>(smem + G::NF * SOFT_COL_STRIDE);

  DEC_STAMP(0);
  DEC_PROF(29, __builtin_amdgcn_s_memrealtime());
  const dec_desc d      = descs[blockIdx.x];
  // HARQ context (pusch_decoder_impl.cpp:300): a codeblock whose CRC already passed is not decoded again.
  if (cb_crc_ok != nullptr && cb_crc_ok[d.cb_index] != 0) {
    if (threadIdx.x == 0) {
      results[d.cb_index] = 0;
    }
    return;
  }
  const int      Z      = d.Z;
  const auto     sh     = (const_u32_ptr)(uintptr_t)(shift_table + static_cast<uint32_t>(d.zpos) * G::NE);
  // Warm the scalar cache with this Z's shift row while the LLRs load: the layers read it with s_load, and cold
  // misses there would stall every layer of the first iteration. The loads are ordinary (compiler-tracked) scalar loads
  // consumed only after the LLR stage (scalar_touch, ldpc_decoder_common.h).
  // (Kernel arguments are pinned in SGPRs first: a later kernarg s_load would wait for the warm-up loads.)
  asm volatile("" ::"s"(llrs), "s"(out), "s"(results), "s"(crc_tables), "s"(cb_crc_ok), "s"(blockDim.x));
  constexpr int SH_LINES = (G::NE * 4 - 4) / 64 + 2;
  uint32_t      pf[SH_LINES];
  static_for<SH_LINES>([&](auto L) {
    constexpr int l = decltype(L)::value;
    scalar_touch<(l * 64 < G::NE * 4 - 4) ? l * 64 : G::NE * 4 - 4>(pf[l], sh);
  });
  const int      z      = threadIdx.x;
  const bool     active = z < Z;
  const int      wave   = threadIdx.x / WAVE;
  const int      nwaves = blockDim.x / WAVE;
  const int      lane   = threadIdx.x % WAVE;

  // ---- Load the LLRs into the soft-bit image (ldpc_decoder_impl.cpp:152) and find the last non-zero LLR (:94). ----
  // 16-byte loads from the aligned span covering the LLRs, all of a lane's loads in flight at once, then a byte
  // scatter into the column-major image. A vector inside one lifted column of the clamped region (the common case)
  // takes the short path: one address, a clamp per byte, a whole-vector non-zero test. Boundary vectors (head and
  // tail of the span, column crossings, the unclamped tail of the input) go byte by byte.
  // The input: at its offset in the batch buffer, or wherever llr_cbs[cb] points (a persistent HARQ arena slot).
  const int8_t*  llr   = (llr_cbs != nullptr) ? llr_cbs[d.cb_index] : llrs + d.llr_offset;
  const int      n_llr = static_cast<int>(d.nof_llr);
  const uint32_t ncols = __umulhi(static_cast<uint32_t>(n_llr), d.div_magic);  // whole lifted columns of input
  const uint32_t full  = ncols * static_cast<uint32_t>(Z);
  int            last  = -1;
  const bool     use_crc = d.crc_table != NO_CRC_TABLE;
  const int      nsig    = d.nof_significant;
  {
    const uint32_t head = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(llr)) & 15u;
    const uint4*   vecs = reinterpret_cast<const uint4*>(llr - head);
    const int      nvec = static_cast<int>((head + static_cast<uint32_t>(n_llr) + 15u) >> 4);
    // 5 x 16 B per lane covers a whole BG1 codeblock at Z = 384 with 384 lanes (and at every smaller Z).
    constexpr int BATCH  = 5;
    int           last_w = -1;  // last short-path vector with a non-zero byte, and its bytes
    uint4         last_v = make_uint4(0u, 0u, 0u, 0u);
    for (int w0 = threadIdx.x; w0 < nvec; w0 += BATCH * blockDim.x) {
      uint4 val[BATCH];
#pragma unroll
      for (int j = 0; j < BATCH; ++j) {
        const int w = w0 + j * blockDim.x;
        val[j]      = (w < nvec) ? vecs[w] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int j = 0; j < BATCH; ++j) {
        const int w = w0 + j * blockDim.x;
        if (w >= nvec) {
          continue;
        }
        const uint32_t i0 = static_cast<uint32_t>(16 * w) - head;  // LLR index of byte 0 (wraps for the head)
        const uint32_t c0 = __umulhi(i0, d.div_magic);
        const uint32_t l0 = i0 - c0 * static_cast<uint32_t>(Z);
        const bool     short_path = (16u * static_cast<uint32_t>(w) >= head) && (i0 + 16u <= full) &&
                                (l0 + 16u <= static_cast<uint32_t>(Z));
        if (short_path) {
          int8_t* dst = soft + (c0 + 2) * SOFT_COL_STRIDE + l0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t word = (q == 0) ? val[j].x : (q == 1) ? val[j].y : (q == 2) ? val[j].z : val[j].w;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              dst[4 * q + k] = static_cast<int8_t>(clamp_i(static_cast<int8_t>(word >> (8 * k)), -64, 64));
            }
          }
          if ((val[j].x | val[j].y | val[j].z | val[j].w) != 0u) {
            last_w = w;
            last_v = val[j];
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t word = (q == 0) ? val[j].x : (q == 1) ? val[j].y : (q == 2) ? val[j].z : val[j].w;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t i = i0 + static_cast<uint32_t>(4 * q + k);
              if (i < static_cast<uint32_t>(n_llr)) {
                int v = static_cast<int8_t>(word >> (8 * k));
                last  = (v != 0) ? static_cast<int>(i) : last;
                // Soft clamp of the whole lifted columns (:152); the tail keeps its LLRs, infinities as
                // +/-SOFT_INF.
                v                 = (i < full) ? clamp_i(v, -64, 64) : clamp_i(v, -SOFT_INF, SOFT_INF);
                const uint32_t cq = __umulhi(i, d.div_magic);
                soft[(cq + 2) * SOFT_COL_STRIDE + (i - cq * static_cast<uint32_t>(Z))] = static_cast<int8_t>(v);
              }
            }
          }
        }
      }
    }
    if (last_w >= 0) {
      // Highest non-zero byte of the last non-zero short-path vector.
      const uint32_t words[4] = {last_v.x, last_v.y, last_v.z, last_v.w};
      int            hb       = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        hb = (words[q] != 0u) ? 4 * q + (31 - __clz(static_cast<int>(words[q]))) / 8 : hb;
      }
      const int i = 16 * last_w - static_cast<int>(head) + hb;
      last        = i > last ? i : last;
    }
  }
  // Zero the punctured columns 0, 1 and every position beyond the input (the image is read up to K + nof_layers
  // columns).
  if (active) {
    soft[0 * SOFT_COL_STRIDE + z] = 0;
    soft[1 * SOFT_COL_STRIDE + z] = 0;
    int c = 2 + static_cast<int>(ncols);
    if (static_cast<uint32_t>(n_llr) > full) {
      if (z >= n_llr - static_cast<int>(full)) {
        soft[c * SOFT_COL_STRIDE + z] = 0;
      }
      ++c;
    }
    for (; c < G::NF; ++c) {
      soft[c * SOFT_COL_STRIDE + z] = 0;
    }
  }
  last = wave_max(last);
  if (lane == 0) {
    scratch[wave] = last;
  }
  __syncthreads();
  // Consume the scalar-cache warm-up loads (they landed long ago; the compiler places the wait).
  static_for<SH_LINES>([&](auto L) { keep_sgpr(pf[decltype(L)::value]); });
  int input_size = scratch[0];
  for (int w = 1; w < nwaves; ++w) {
    input_size = scratch[w] > input_size ? scratch[w] : input_size;
  }
  input_size += 1;

  const int  msg_len = G::K * Z;
  uint8_t*   cb_out  = out + d.out_offset;
  if (input_size < msg_len) {
    // Not enough LLRs: no decoding; when the CRC is not the decoder's (no CRC, or checked by the caller after the
    // last iteration: no early stop, pusch_codeblock_decoder passes no calculator) the output is all ones
    // (ldpc_decoder_impl.cpp:95).
    if (!use_crc || (d.flags & DEC_FLAG_EARLY_STOP) == 0) {
      for (int b = threadIdx.x; b < (msg_len + 7) / 8; b += blockDim.x) {
        cb_out[b] = 0xff;
      }
    }
    if (threadIdx.x == 0) {
      results[d.cb_index] = -1;
    }
    return;
  }
  int cb_len = input_size + 2 * Z;
  cb_len     = cb_len > msg_len + 4 * Z ? cb_len : msg_len + 4 * Z;
  const int nof_layers =
      __builtin_amdgcn_readfirstlane(static_cast<int>(__umulhi(static_cast<uint32_t>(cb_len + Z - 1), d.div_magic)) -
                                     G::K);

  const uint32_t  sf16      = d.sf16;
  const float     sf        = d.sf;

  uint32_t st[G::M];
  uint32_t st_hi = 0;
#pragma unroll
  for (int m = 0; m < G::M; ++m) {
    st[m] = 0;
  }
  __syncthreads();


  const uint32_t* crc_table = crc_tables + (use_crc ? d.crc_table : 0u);
  const int max_iter = d.max_iter;
  DEC_STAMP(1);
  DEC_PROF(31, static_cast<uint64_t>(nof_layers));
  for (int it = 0; it < max_iter; ++it) {
    // Opaque per-iteration copies: stop the compiler from hoisting per-layer predicates and per-column addresses out
    // of the iteration loop (they would pin ~70 registers for values that cost one instruction to recompute).
    int nl = nof_layers, zz = z, ZZ = Z;
    asm volatile("" : "+s"(nl));
    asm volatile("" : "+v"(zz));
    asm volatile("" : "+s"(ZZ));
    static_for<G::M>([&](auto Mi) {
      constexpr int m = decltype(Mi)::value;
      if (m < nl) {
        if (active) {
          row_update<BG, MODE, m>(soft, sh, zz, ZZ, sf16, sf, st[m], st_hi);
        }
        __syncthreads();
      }
    });
    DEC_STAMP(2 + 2 * (it & 7));

    // With early stopping the CRC is checked after every iteration (ldpc_decoder_impl.cpp:133); without it, once after
    // the last iteration (pusch_codeblock_decoder.cpp:53: decode without CRC, then check the CRC of the output).
    if (use_crc && ((d.flags & DEC_FLAG_EARLY_STOP) != 0 || it == max_iter - 1)) {
      // Success: every systematic soft bit non-zero (early stop only) and CRC remainder zero. The CRC of
      // the hard decisions is the XOR of per-bit contributions x^(order + L - 1 - i) mod g(x) (crc_table).
      uint32_t acc  = 0;
      uint32_t zero = 0;
      if (active) {
        // Unconditional table loads (index clamped, value masked): no divergent branch between them, so they are
        // all in flight at once.
        uint32_t       i        = static_cast<uint32_t>(zz);
        const uint32_t last_bit = static_cast<uint32_t>(nsig) - 1u;
        static_for<G::K>([&](auto Ci) {
          constexpr int  c  = decltype(Ci)::value;
          const int      sb = soft[c * SOFT_COL_STRIDE + zz];
          const uint32_t t  = crc_table[i < last_bit ? i : last_bit];
          zero |= static_cast<uint32_t>(sb == 0);
          acc ^= (sb <= 0 && i <= last_bit) ? t : 0u;
          i += static_cast<uint32_t>(ZZ);
        });
      }
      acc  = wave_xor(acc);
      zero = (__ballot(zero != 0) != 0) ? 1u : 0u;
      int* red = scratch + 8 + 16 * (it & 1);
      if (lane == 0) {
        red[2 * wave]     = static_cast<int>(acc);
        red[2 * wave + 1] = static_cast<int>(zero);
      }
      __syncthreads();
      uint32_t tacc = 0, tzero = 0;
      for (int w = 0; w < nwaves; ++w) {
        tacc ^= static_cast<uint32_t>(red[2 * w]);
        tzero |= static_cast<uint32_t>(red[2 * w + 1]);
      }
      const bool early = (d.flags & DEC_FLAG_EARLY_STOP) != 0;
      DEC_STAMP(3 + 2 * (it & 7));
      if ((tzero == 0 || !early) && tacc == 0) {
        write_hard_bits(soft, cb_out, msg_len, Z, d.div_magic);
        DEC_STAMP(28);
        DEC_PROF(30, __builtin_amdgcn_s_memrealtime());
        if (threadIdx.x == 0) {
          results[d.cb_index] = it + 1;
          if (cb_crc_ok != nullptr) {
            cb_crc_ok[d.cb_index] = 1;
          }
        }
        return;
      }
    }
  }
  write_hard_bits(soft, cb_out, msg_len, Z, d.div_magic);
  DEC_STAMP(28);
  DEC_PROF(30, __builtin_amdgcn_s_memrealtime());
  if (threadIdx.x == 0) {
    results[d.cb_index] = -1;
  }
}

} // namespace

#ifdef LDPC_DEC_PROFILE
int debug_read_decoder_profile(uint64_t* dst, size_t n)
{
  const size_t max = static_cast<size_t>(LDPC_DEC_PROF_CBS) * LDPC_DEC_PROF_SLOTS;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_dec_prof), (n < max ? n : max) * sizeof(uint64_t)) == hipSuccess ? 0
                                                                                                              : -1;
}
#endif

void launch_ldpc_decode(int             bg,
                        int             mode,
                        const dec_desc* d_desc,
                        int             nof_cbs,
                        int             block_threads,
                        const int8_t*   d_llrs,
                        uint8_t*        d_out,
                        int32_t*        d_results,
                        const uint32_t* d_shifts,
                        const uint32_t* d_crc_tables,
                        uint8_t*        d_cb_crc_ok,
                        hipStream_t     stream,
                        int8_t* const*  d_llr_cbs)
{
  if (nof_cbs <= 0) {
    return;
  }
  const size_t lds = 0;
  dim3         grid(nof_cbs), block(block_threads);
  if (bg == 1) {
    if (mode == 1) {
      ldpc_decode_kernel<1, 1><<<grid, block, lds, stream>>>(d_desc, d_llrs, d_out, d_results, d_shifts, d_crc_tables, d_cb_crc_ok, d_llr_cbs);
    } else {
      ldpc_decode_kernel<1, 0><<<grid, block, lds, stream>>>(d_desc, d_llrs, d_out, d_results, d_shifts, d_crc_tables, d_cb_crc_ok, d_llr_cbs);
    }
  } else {
    if (mode == 1) {
      ldpc_decode_kernel<2, 1><<<grid, block, lds, stream>>>(d_desc, d_llrs, d_out, d_results, d_shifts, d_crc_tables, d_cb_crc_ok, d_llr_cbs);
    } else {
      ldpc_decode_kernel<2, 0><<<grid, block, lds, stream>>>(d_desc, d_llrs, d_out, d_results, d_shifts, d_crc_tables, d_cb_crc_ok, d_llr_cbs);
    }
  }
}

} // namespace srsgpu
