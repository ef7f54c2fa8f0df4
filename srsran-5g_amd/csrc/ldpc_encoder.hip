// PDSCH channel encoding for 5G NR on gfx950: transport-block CRC, codeblock assembly with CB CRC24B, LDPC encoding
// (TS 38.212 §5.3.2, BG1/BG2) and rate matching with bit interleaving (§5.4.2), batched over every codeblock of a slot.
//
// Drop-in semantics of srsran::pdsch_encoder_impl::encode (reference lib/phy/upper/channel_processors/pdsch/
// pdsch_encoder_impl.cpp:28): ldpc_segmenter_tx_impl::read_codeblock (ldpc_segmenter_tx_impl.cpp:144), the LDPC
// encoder (ldpc_encoder_generic.cpp) and ldpc_rate_matcher_impl::rate_match (ldpc_rate_matcher_impl.cpp:95). The
// codeword is produced packed MSB first (the bit_buffer / hw_accelerator_pdsch_enc packed layout); the reference
// unpacks it one bit per byte, which the host binding does for comparisons.
//
// Mapping to CDNA4: one workgroup per codeblock. Codeblocks with Z % 32 == 0 and byte-aligned data (the common case)
// take the packed kernel (pdsch_encode_packed_kernel: 32 lifted rows per lane-word, funnel-shift rotations, windowed
// rate matching); the others the byte kernel, where the codeblock's bits live one per byte in LDS (column c at
// c * 384, as in the decoder) and lane z computes row z of every lifted parity equation. Both produce the
// rate-matched output 32 bits per lane and write whole words (atomicOr only for the two words a codeblock shares
// with its neighbours).
#include "common.h"
#include "crc_device.h"
#include "ldpc_base_graphs.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {

#ifdef ENC_PROFILE
// Instrumented builds only (tools/encoder_phase_profile.py): s_memtime per phase of the first ENC_PROF_CBS codeblocks.
constexpr int ENC_PROF_CBS   = 8192;
constexpr int ENC_PROF_SLOTS = 16;
__device__ uint64_t g_enc_prof[ENC_PROF_CBS * ENC_PROF_SLOTS];
#define ENC_PROF(slot, value)                                                                                          \
  do {                                                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < ENC_PROF_CBS) {                                                               \
      g_enc_prof[blockIdx.x * ENC_PROF_SLOTS + (slot)] = (value);                                                      \
    }                                                                                                                  \
  } while (0)
#else
#define ENC_PROF(slot, value)                                                                                          \
  do {                                                                                                                 \
  } while (0)
#endif
#define ENC_STAMP(slot) ENC_PROF(slot, __builtin_amdgcn_s_memtime())

template <int BG>
struct ebg;
template <>
struct ebg<1> {
  static constexpr int M  = kBG1_M;
  static constexpr int NF = kBG1_N_FULL;
  static constexpr int K  = kBG1_K;
  static constexpr int NE = kBG1_NUM_EDGES;
  static constexpr int rs(int m) { return kBG1_ROW_START[m]; }
  static constexpr int col(int e) { return kBG1_COL[e]; }
};
template <>
struct ebg<2> {
  static constexpr int M  = kBG2_M;
  static constexpr int NF = kBG2_N_FULL;
  static constexpr int K  = kBG2_K;
  static constexpr int NE = kBG2_NUM_EDGES;
  static constexpr int rs(int m) { return kBG2_ROW_START[m]; }
  static constexpr int col(int e) { return kBG2_COL[e]; }
};

constexpr int S = SOFT_COL_STRIDE;

/// Largest degree of the four core rows.
template <int BG>
constexpr int core_max_degree()
{
  int d = 0;
  for (int m = 0; m < 4; ++m) {
    d = (ebg<BG>::rs(m + 1) - ebg<BG>::rs(m) > d) ? ebg<BG>::rs(m + 1) - ebg<BG>::rs(m) : d;
  }
  return d;
}

__device__ __forceinline__ int rot(int z, int s, int Z)
{
  const uint32_t p0 = static_cast<uint32_t>(z + s);
  const uint32_t p1 = p0 - static_cast<uint32_t>(Z);
  return static_cast<int>(p0 < p1 ? p0 : p1);
}

/// CRC of every transport block (TS 38.212 §5.1): one 256-lane workgroup per TB slice (crc_device.h), each XORing its
/// slice's contribution into the TB's (zeroed) CRC word.
__global__ __launch_bounds__(256) void tb_crc_kernel(const tb_crc_desc* __restrict__ descs,
                                                     const tb_crc_slice* __restrict__ slices,
                                                     const uint8_t* __restrict__ tbs,
                                                     uint32_t* __restrict__ crcs,
                                                     const uint32_t* __restrict__ crc_tables)
{
  __shared__ uint32_t table[256];
  __shared__ uint32_t part[256];
  const tb_crc_slice sl = slices[blockIdx.x];
  const tb_crc_desc  d  = descs[sl.tb];
  // Chunked byte-table CRC moved by the per-bit contribution table when the plan could cache one for this length,
  // else the byte table with pairwise GF(2) combination.
  uint32_t crc;
  if (d.table != NO_CRC_TABLE) {
    crc_byte_lut(table, static_cast<int>(d.order), d.poly);
    const uint8_t* tb = tbs + d.byte_offset;
    crc = block_crc_chunks<16>([tb](int i) { return tb[i]; }, static_cast<int>(d.nbytes), crc_tables + d.table,
                               static_cast<int>(d.order), d.poly, table, part, static_cast<int>(sl.begin),
                               static_cast<int>(sl.end));
  } else {  // one slice: the whole TB
    crc = block_crc_bytes(tbs + d.byte_offset, static_cast<int>(d.nbytes), static_cast<int>(d.order), d.poly, table,
                          part);
  }
  if (threadIdx.x == 0) {
    atomicXor(&crcs[sl.tb], crc);
  }
}

template <int BG, int QM>
__device__ __forceinline__ void rate_match_words(const enc_desc& d, const uint8_t* __restrict__ bits, int Z,
                                                 uint32_t* __restrict__ out_words)
{
  // Output bit t of the codeblock: symbol i = t / Qm, bit j = t % Qm carries e[j * R + i] (interleaver, :150);
  // e[n] is the circular-buffer bit at valid position (v0 + n) mod V, fillers skipped (select_bits, :104).
  const int      E = static_cast<int>(d.E), R = E / QM;
  const int      V = static_cast<int>(d.Ncb) - d.filler;
  const int      ninfo = (ebg<BG>::K - 2) * Z - d.filler;
  const uint32_t g0    = d.out_bit_offset;
  const uint32_t w0 = g0 / 32u, w1 = (g0 + static_cast<uint32_t>(E) - 1u) / 32u;
  for (uint32_t w = w0 + threadIdx.x; w <= w1; w += blockDim.x) {
    uint32_t word = 0;
    bool     full = true;
    for (int b = 0; b < 32; ++b) {
      const int t = static_cast<int>(w * 32u + static_cast<uint32_t>(b) - g0);
      if (t < 0 || t >= E) {
        full = false;
        continue;
      }
      const int i = t / QM, j = t - i * QM;
      int       v = static_cast<int>(d.v0) + j * R + i;
      while (v >= V) {
        v -= V;
      }
      const int k   = (v < ninfo ? v : v + d.filler) + 2 * Z;  // shortened position -> full codeblock position
      const int col = static_cast<int>(__umulhi(static_cast<uint32_t>(k), d.div_magic));
      const int l   = k - col * Z;
      // Byte (g / 8) of the packed stream, bit 7 - g % 8, inside a little-endian 32-bit word.
      word |= static_cast<uint32_t>(bits[col * S + l]) << ((b & ~7) + 7 - (b & 7));
    }
    if (full) {
      out_words[w] = word;
    } else if (word != 0) {
      atomicOr(&out_words[w], word);
    }
  }
}

template <int BG>
__global__ __launch_bounds__(384) void pdsch_encode_kernel(const enc_desc* __restrict__ descs,
                                                           const uint8_t* __restrict__ tbs,
                                                           const uint32_t* __restrict__ tb_crcs,
                                                           uint32_t* __restrict__ out_words,
                                                           const uint16_t* __restrict__ shift_table,
                                                           const core_plan* __restrict__ core_plans,
                                                           const uint32_t* __restrict__ crc_tables)
{
  using G = ebg<BG>;
  __shared__ __attribute__((aligned(16))) uint8_t bits[G::NF * S];
  __shared__ uint8_t  lam[4 * S];
  __shared__ uint16_t sh[G::NE];
  __shared__ uint32_t red[8];
  __shared__ uint32_t lut[256];
  __shared__ uint8_t  msg[G::K * 384 / 8];  // packed message bytes (byte path): input of the CB CRC

  const enc_desc d  = descs[blockIdx.x];
  const int      Z  = d.Z;
  const int      K  = G::K;
  const int      KZ = K * Z;
  for (int e = threadIdx.x; e < G::NE; e += blockDim.x) {
    sh[e] = shift_table[static_cast<uint32_t>(d.zpos) * G::NE + e];
  }
  // ---- Codeblock message (ldpc_segmenter_tx_impl.cpp:144): TB(+TB CRC) bits, zero padding, CB CRC, fillers. ----
  const uint8_t* tb      = tbs + d.tb_byte_offset;
  const uint32_t tb_crc  = tb_crcs[d.tb_index];
  const int      ndata   = d.nof_data;
  // Byte path: TS 38.214 TB sizes make every codeblock's data byte-aligned ((TBS + 24) is a multiple of 8 C), so the
  // message is whole TB / TB CRC bytes; they are also kept packed for the CB CRC.
  const bool byte_path = ((d.tb_bit_offset | static_cast<uint32_t>(ndata) | d.tb_bits | d.tb_crc_len) & 7u) == 0 &&
                         (d.crc_table == NO_CRC_TABLE || (d.used & 7u) == 0);
  int first_bit = 0;  // bits below are written by the byte path
  if (byte_path) {
    const int nmsg = (d.crc_table != NO_CRC_TABLE) ? static_cast<int>(d.used) / 8 : ndata / 8;
    for (int q = threadIdx.x; q < nmsg; q += blockDim.x) {
      uint32_t byte = 0;
      if (8 * q < ndata) {
        const uint32_t p = d.tb_bit_offset + 8u * static_cast<uint32_t>(q);
        byte = (p < d.tb_bits) ? tb[p >> 3] : (tb_crc >> (d.tb_crc_len - 8u - (p - d.tb_bits))) & 0xffu;
      }
      msg[q]       = static_cast<uint8_t>(byte);
      const int i0 = 8 * q;
      int       col = static_cast<int>(__umulhi(static_cast<uint32_t>(i0), d.div_magic));
      int       l   = i0 - col * Z;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bits[col * S + l] = static_cast<uint8_t>((byte >> (7 - k)) & 1u);
        if (++l == Z) {
          l = 0;
          ++col;
        }
      }
    }
    first_bit = 8 * nmsg;
  }
  for (int i = first_bit + static_cast<int>(threadIdx.x); i < KZ; i += blockDim.x) {
    uint32_t bit = 0;
    if (i < ndata) {
      const uint32_t p = d.tb_bit_offset + static_cast<uint32_t>(i);
      bit              = (p < d.tb_bits) ? (tb[p >> 3] >> (7u - (p & 7u))) & 1u
                                         : (tb_crc >> (d.tb_crc_len - 1u - (p - d.tb_bits))) & 1u;
    }
    const int col = static_cast<int>(__umulhi(static_cast<uint32_t>(i), d.div_magic));
    bits[col * S + (i - col * Z)] = static_cast<uint8_t>(bit);
  }
  if (byte_path && d.crc_table != NO_CRC_TABLE) {
    crc_byte_lut(lut, 24, 0x1800063u);  // CRC24B; ends with a barrier (msg and bits complete)
  }
  __syncthreads();
  // ---- Codeblock CRC24B over the first `used` bits. ----
  if (d.crc_table != NO_CRC_TABLE) {
    const uint32_t* P = crc_tables + d.crc_table;
    uint32_t        crc;
    if (byte_path) {
      crc = block_crc_chunks<16>([](int q) { return msg[q]; }, static_cast<int>(d.used) / 8, P, 24, 0x1800063u,
                                 lut, red);
    } else {  // XOR of per-bit contributions (table per length)
      uint32_t acc = 0;
      for (int i = threadIdx.x; i < d.used; i += blockDim.x) {
        const int col = static_cast<int>(__umulhi(static_cast<uint32_t>(i), d.div_magic));
        acc ^= bits[col * S + (i - col * Z)] ? P[i] : 0u;
      }
      acc = wave_xor(acc);
      if ((threadIdx.x % WAVE) == 0) {
        red[threadIdx.x / WAVE] = acc;
      }
      __syncthreads();
      crc = 0;
      for (int w = 0; w < static_cast<int>(blockDim.x / WAVE); ++w) {
        crc ^= red[w];
      }
    }
    for (int k = threadIdx.x; k < 24; k += blockDim.x) {
      const int i   = d.used + k;
      const int col = static_cast<int>(__umulhi(static_cast<uint32_t>(i), d.div_magic));
      bits[col * S + (i - col * Z)] = static_cast<uint8_t>((crc >> (23 - k)) & 1u);
    }
    __syncthreads();
  }
  const int  z      = threadIdx.x;
  const bool active = z < Z;
  // ---- Core parity (rows 0..3, double-diagonal): lambda_m = sum of the rotated information nodes. ----
  if (active) {
    static_for<4>([&](auto Mi) {
      constexpr int m  = decltype(Mi)::value;
      constexpr int e0 = G::rs(m), deg = G::rs(m + 1) - e0;
      uint32_t      acc = 0;
      static_for<deg>([&](auto Ei) {
        constexpr int e   = e0 + decltype(Ei)::value;
        constexpr int col = G::col(e);
        if constexpr (col < G::K) {
          acc ^= bits[col * S + rot(z, sh[e], Z)];
        }
      });
      lam[m * S + z] = static_cast<uint8_t>(acc);
    });
  }
  __syncthreads();
  const core_plan* __restrict__ cp = core_plans + d.zpos;
  if (active) {
    // P^x p0 = lambda_0 + lambda_1 + lambda_2 + lambda_3
    bits[K * S + rot(z, cp->x, Z)] = lam[z] ^ lam[S + z] ^ lam[2 * S + z] ^ lam[3 * S + z];
  }
  __syncthreads();
  for (int step = 0; step < 3; ++step) {
    if (active) {
      const int u   = cp->unk[step];
      const int row = cp->row[step];
      uint32_t  acc = lam[row * S + z];
      for (int j = 0; j < 4; ++j) {
        const int s = cp->sh[step][j];
        if (j != u && s >= 0) {
          acc ^= bits[(K + j) * S + rot(z, s, Z)];
        }
      }
      bits[(K + u) * S + rot(z, cp->sh[step][u], Z)] = static_cast<uint8_t>(acc);
    }
    __syncthreads();
  }
  // ---- Extension parity (identity extension): p_{K+m} = sum over the row's nodes of the high-rate region. ----
  if (active) {
    const int n_ext = d.n_ext;
    static_for<G::M - 4>([&](auto Mi) {
      constexpr int m  = 4 + decltype(Mi)::value;
      constexpr int e0 = G::rs(m), deg = G::rs(m + 1) - e0;
      if (m - 4 < n_ext) {
        uint32_t acc = 0;
        static_for<deg>([&](auto Ei) {
          constexpr int e   = e0 + decltype(Ei)::value;
          constexpr int col = G::col(e);
          if constexpr (col < G::K + 4) {
            acc ^= bits[col * S + rot(z, sh[e], Z)];
          }
        });
        bits[(K + m) * S + z] = static_cast<uint8_t>(acc);
      }
    });
  }
  __syncthreads();
  // ---- Rate matching + interleaving + packing. ----
  switch (d.Qm) {
    case 1: rate_match_words<BG, 1>(d, bits, Z, out_words); break;
    case 2: rate_match_words<BG, 2>(d, bits, Z, out_words); break;
    case 4: rate_match_words<BG, 4>(d, bits, Z, out_words); break;
    case 6: rate_match_words<BG, 6>(d, bits, Z, out_words); break;
    default: rate_match_words<BG, 8>(d, bits, Z, out_words); break;
  }
}

// ---------------------------------------------------------------------------------------------------------------------
// Packed encoder (Z a multiple of 32, byte-aligned codeblock data: every codeblock of TS 38.214 TB sizes with
// Z >= 32 of the form 2^j * {1, 3, 5, 7, 9, 11}): the codeblock lives in LDS as LSB-first bit words, column c word k
// holding bits 32k..32k+31 of node c, so full-codeblock position p is bit p & 31 of word p >> 5. A lifted rotation
// by s of a column is a funnel shift of two of its words (Z % 32 == 0 makes the rotation word-granular plus a bit
// offset), so one lane computes 32 rows of a lifted parity equation per instruction sequence, and the rate matcher
// reads 32 consecutive circular-buffer bits per window instead of one byte per bit.
// ---------------------------------------------------------------------------------------------------------------------

constexpr int PK_THREADS = 128;

/// Bits X[(32 k + t + o) mod Z], t = 0..31, of a packed Z-bit column X (W = Z / 32 words), 0 <= o < Z.
__device__ __forceinline__ uint32_t col_window(const uint32_t* x, int k, int o, int W)
{
  int a = k + (o >> 5);
  a     = a >= W ? a - W : a;
  int b = a + 1;
  b     = b >= W ? b - W : b;
  return __builtin_amdgcn_alignbit(x[b], x[a], static_cast<uint32_t>(o & 31));
}

/// Reverses the bit order inside every byte (LSB-first word <-> MSB-first byte stream in a little-endian word).
__device__ __forceinline__ uint32_t bytes_bitrev(uint32_t x)
{
  return __builtin_bitreverse32(__builtin_bswap32(x));
}

struct pk_rm {
  const uint32_t* cw;  ///< Packed full codeblock (LDS).
  uint32_t        v0, V, ninfo, filler, Z2;

  /// Full-codeblock position of circular-buffer valid position v (fillers skipped, first 2Z punctured).
  __device__ __forceinline__ uint32_t pos(uint32_t v) const { return v + Z2 + (v < ninfo ? 0u : filler); }
  __device__ __forceinline__ uint32_t bit_at(uint32_t v) const
  {
    const uint32_t k = pos(v);
    return (cw[k >> 5] >> (k & 31u)) & 1u;
  }
  __device__ __forceinline__ uint32_t wrap(uint32_t n) const
  {
    uint32_t v = v0 + n;
    while (v >= V) {
      v -= V;
    }
    return v;
  }
  /// e[n .. n + L - 1] (rate-matcher selection output, ldpc_rate_matcher_impl.cpp:104) as LSB-first bits.
  template <int L>
  __device__ __forceinline__ uint32_t window(uint32_t n) const
  {
    const uint32_t v = wrap(n);
    if (v + L <= V && (v >= ninfo || v + L <= ninfo)) {  // one contiguous run of the codeblock
      const uint32_t k = pos(v);
      return __builtin_amdgcn_alignbit(cw[(k >> 5) + 1u], cw[k >> 5], k & 31u);
    }
    uint32_t r = 0;
    uint32_t u = v;
    for (int t = 0; t < L; ++t) {
      r |= bit_at(u) << t;
      u = (u + 1u == V) ? 0u : u + 1u;
    }
    return r;
  }
};

/// Spreads the low 32/QM bits of x to bit positions 0, QM, 2 QM, ... (QM in {1, 2, 4, 8}).
template <int QM>
__device__ __forceinline__ uint32_t spread_bits(uint32_t x)
{
  if constexpr (QM == 1) {
    return x;
  } else if constexpr (QM == 2) {
    x &= 0xffffu;
    x = (x | (x << 8)) & 0x00ff00ffu;
    x = (x | (x << 4)) & 0x0f0f0f0fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
  } else if constexpr (QM == 4) {
    x &= 0xffu;
    x = (x | (x << 12)) & 0x000f000fu;
    x = (x | (x << 6)) & 0x03030303u;
    return (x | (x << 3)) & 0x11111111u;
  } else {
    x &= 0xfu;
    x = (x | (x << 14)) & 0x00030003u;
    return (x | (x << 7)) & 0x01010101u;
  }
}

/// Rate matching + bit interleaving (ldpc_rate_matcher_impl.cpp:95/:150) of the packed codeblock into packed output
/// words: stream bit t = Qm i + j carries e[j R + i]. Words wholly inside the codeblock with symbol-aligned bits
/// (Qm in {1, 2, 4, 8}, g0 % Qm == 0) take one e window per bit row j; the rest (the two boundary words, Qm = 6,
/// unaligned offsets) are assembled bit by bit.
/// Exchanges the bits of a selected by mask m << k with the bits of b selected by m (one delta swap).
__device__ __forceinline__ void delta_swap(uint32_t& a, uint32_t& b, int k, uint32_t m)
{
  const uint32_t t = ((a >> k) ^ b) & m;
  b ^= t;
  a ^= t << k;
}

/// 256QAM groups (ldpc_rate_matcher_impl.cpp:150 interleaving, Qm = 8): 32 consecutive modulation symbols i0 .. i0 + 31
/// from one 32-bit circular-buffer window per bit row j (r_j bit s = e[j R + i0 + s]), transposed as four 8 x 8 bit
/// blocks by three rounds of delta swaps (rows fed in reverse, so each symbol's byte comes out MSB first) into the 8
/// output words of the group: 8 windows and ~70 VALU for 8 words instead of 8 windows and ~20 VALU per word.
__device__ __forceinline__ void rate_match_group8(const pk_rm& rm, int R, int i0, uint32_t* __restrict__ out)
{
  uint32_t r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    r[j] = rm.window<32>(static_cast<uint32_t>((7 - j) * R + i0));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    delta_swap(r[j], r[j + 4], 4, 0x0f0f0f0fu);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if ((j & 2) == 0) {
      delta_swap(r[j], r[j + 2], 2, 0x33333333u);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    delta_swap(r[j], r[j + 1], 1, 0x55555555u);
  }
  // Now byte c of r[j] is symbol 8 c + j: output word t = symbols 4 t .. 4 t + 3 = byte t / 2 of r[4 (t & 1) + q].
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int      c  = t >> 1;
    const uint32_t* q = r + 4 * (t & 1);
    const uint32_t lo = __builtin_amdgcn_perm(q[1], q[0], 0x0c0c0400u + 0x0101u * static_cast<uint32_t>(c));
    const uint32_t hi = __builtin_amdgcn_perm(q[3], q[2], 0x04000c0cu + 0x01010000u * static_cast<uint32_t>(c));
    out[t]            = lo | hi;
  }
}

template <int QM>
__device__ __forceinline__ void rate_match_packed(const enc_desc& d, const pk_rm& rm, uint32_t* __restrict__ out_words)
{
  const int      E  = static_cast<int>(d.E), R = E / QM;
  const uint32_t g0 = d.out_bit_offset;
  const uint32_t w1 = (g0 + static_cast<uint32_t>(E) - 1u) / 32u;
  uint32_t       w0 = g0 / 32u;
  constexpr bool pow2   = (QM == 1 || QM == 2 || QM == 4 || QM == 8);
  const bool     align  = pow2 && (g0 % QM) == 0;
  if constexpr (QM == 8) {
    if ((g0 & 31u) == 0u) {
      // Whole 32-symbol groups by transposition; the remaining words below.
      const int ng = R / 32;
      for (int g = threadIdx.x; g < ng; g += blockDim.x) {
        rate_match_group8(rm, R, 32 * g, out_words + w0 + 8u * static_cast<uint32_t>(g));
      }
      w0 += 8u * static_cast<uint32_t>(ng);
    }
  }
  for (uint32_t w = w0 + threadIdx.x; w <= w1; w += blockDim.x) {
    const int t0   = static_cast<int>(w * 32u - g0);
    const bool full = t0 >= 0 && t0 + 32 <= E;
    uint32_t  lin  = 0;  // bit b = stream bit t0 + b
    if constexpr (pow2) {
      if (full && align) {
        constexpr int SP = 32 / QM;
        const int     i0 = t0 / QM;
#pragma unroll
        for (int j = 0; j < QM; ++j) {
          lin |= spread_bits<QM>(rm.window<SP>(static_cast<uint32_t>(j * R + i0))) << j;
        }
        out_words[w] = bytes_bitrev(lin);
        continue;
      }
    }
    for (int b = 0; b < 32; ++b) {
      const int t = t0 + b;
      if (t >= 0 && t < E) {
        const int i = t / QM, j = t - i * QM;
        lin |= rm.bit_at(rm.wrap(static_cast<uint32_t>(j * R + i))) << b;
      }
    }
    const uint32_t word = bytes_bitrev(lin);
    if (full) {
      out_words[w] = word;
    } else if (word != 0) {
      atomicOr(&out_words[w], word);
    }
  }
}

template <int BG>
__global__ __launch_bounds__(PK_THREADS) void pdsch_encode_packed_kernel(const enc_desc* __restrict__ descs,
                                                                         const uint8_t* __restrict__ tbs,
                                                                         const uint32_t* __restrict__ tb_crcs,
                                                                         const tb_crc_desc* __restrict__ tb_descs,
                                                                         uint32_t* __restrict__ out_words,
                                                                         const uint16_t* __restrict__ shift_table,
                                                                         const core_plan* __restrict__ core_plans,
                                                                         const uint32_t* __restrict__ crc_tables,
                                                                         const uint32_t* __restrict__ crc_slice)
{
  using G = ebg<BG>;
  constexpr int WMAX = 384 / 32;
  __shared__ uint32_t cw[G::NF * WMAX + 1];        // packed codeblock, node c at c * W
  __shared__ uint32_t lam[4 * WMAX];               // core row sums
  __shared__ __attribute__((aligned(4))) uint8_t msg[G::K * 384 / 8];  // message bytes, MSB first
  __shared__ uint32_t edge[G::NE];                 // column << 16 | lifted shift of every base-graph edge
  __shared__ uint16_t row_start[G::M + 1];
  __shared__ uint32_t red[PK_THREADS / WAVE];
  __shared__ uint32_t t4b[CRC_SLICE_WORDS];        // CB CRC24B slice-by-4 tables
  __shared__ uint32_t t4t[CRC_SLICE_WORDS];        // TB CRC (24A or 16) slice-by-4 tables (the carrier only)

  ENC_STAMP(0);
  ENC_PROF(9, __builtin_amdgcn_s_memrealtime());
  const enc_desc d   = descs[blockIdx.x];
  const int      Z   = d.Z;
  const int      W   = Z / 32;
  const int      K   = G::K;
  const int      nkb = K * Z / 8;  // message bytes
  const int      tid = static_cast<int>(threadIdx.x);
  const uint8_t* tb  = tbs + d.tb_byte_offset;
  const int      nd8 = d.nof_data / 8;
  // Every global load that depends only on the descriptor is issued up front (edge table, message bytes, the CB CRC's
  // chunk power, the TB CRC word), so their latencies overlap instead of adding up.
  constexpr int NEL = (G::NE + PK_THREADS - 1) / PK_THREADS;
  uint32_t      ev[NEL];
#pragma unroll
  for (int r = 0; r < NEL; ++r) {
    const int e = tid + r * PK_THREADS < G::NE ? tid + r * PK_THREADS : G::NE - 1;
    ev[r]       = (static_cast<uint32_t>(G::col(e)) << 16) | shift_table[static_cast<uint32_t>(d.zpos) * G::NE + e];
  }
  // All of a lane's message bytes are loaded before any is stored (the address is clamped into the TB so the loads
  // are unconditional).
  constexpr int  MB    = (G::K * 384 / 8 + PK_THREADS - 1) / PK_THREADS;
  const uint32_t tb_hi = d.tb_bits >= 8u ? (d.tb_bits - 8u) >> 3 : 0u;
  uint32_t       byte[MB];
#pragma unroll
  for (int r = 0; r < MB; ++r) {
    const int      q  = tid + r * PK_THREADS;
    const uint32_t p  = d.tb_bit_offset + 8u * static_cast<uint32_t>(q);
    const uint32_t pb = p >> 3;
    byte[r]           = (q < nd8) ? tb[pb < tb_hi ? pb : tb_hi] : 0u;
  }
  constexpr int CB_CS    = 8;
  const bool    has_cbc  = d.crc_table != NO_CRC_TABLE;
  const int     cb_bytes = static_cast<int>(d.used) / 8;
  const bool    pre_m    = has_cbc && tid < (cb_bytes + CB_CS - 1) / CB_CS;
  const uint32_t m0      = pre_m ? crc_chunk_power<CB_CS>(tid, cb_bytes, crc_tables + d.crc_table, 24) : 0u;
  uint32_t       tb_crc  = (tb_descs == nullptr) ? tb_crcs[d.tb_index] : 0u;  // from tb_crc_kernel
  // Inline TB CRC (every TB of the plan has a contribution table): the workgroup of the codeblock that carries the TB
  // CRC computes it, the others never need it (no separate tb_crc_kernel launch and dependency). TBs of at most
  // 2 x 16 bytes per lane with 4-byte aligned offset and size (every multi-UE slot TB): each lane's two 16-byte chunks
  // and their powers are loaded here with everything else, and the two chunk chains run interleaved below.
  const bool  carrier = tb_descs != nullptr && d.tb_bit_offset + d.nof_data > d.tb_bits;
  // The TB's CRC parameters straight from the codeblock descriptor (as tb_descs[d.tb_index] holds them): no dependent
  // descriptor load before the TB's own loads.
  tb_crc_desc tcd{};
  tcd.byte_offset = d.tb_byte_offset;
  tcd.nbytes      = d.tb_bits / 8u;
  tcd.order       = d.tb_crc_len;
  tcd.poly        = (d.tb_crc_len == 24) ? 0x1864cfbu : 0x11021u;
  tcd.table       = d.tb_crc_table;
  constexpr int TCS   = 16;
  const bool    tfast = carrier && tcd.nbytes <= 2u * TCS * PK_THREADS && ((tcd.byte_offset | tcd.nbytes) & 3u) == 0u;
  uint32_t      tw[2][TCS / 4];
  uint32_t      tm[2] = {0u, 0u};
  if (tfast) {
    const uint32_t* tbw = reinterpret_cast<const uint32_t*>(tbs + tcd.byte_offset);
    const int       nw  = static_cast<int>(tcd.nbytes / 4u);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = tid + h * PK_THREADS;
#pragma unroll
      for (int q = 0; q < TCS / 4; ++q) {
        const int w = c * (TCS / 4) + q;
        tw[h][q]    = (w < nw) ? tbw[w] : 0u;
      }
      if (c * TCS < static_cast<int>(tcd.nbytes)) {
        tm[h] = crc_chunk_power<TCS>(c, static_cast<int>(tcd.nbytes), crc_tables + tcd.table,
                                     static_cast<int>(tcd.order));
      }
    }
  }
  // Slice-by-4 CRC tables from the context (L2-resident, 8 words per lane; the barriers below publish them).
  constexpr int TW = CRC_SLICE_WORDS / PK_THREADS;
  if (has_cbc) {
    const uint32_t* src = crc_slice + CRC_SLICE_24B * CRC_SLICE_WORDS;
    uint32_t        t[TW];
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      t[q] = src[tid + q * PK_THREADS];
    }
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      t4b[tid + q * PK_THREADS] = t[q];
    }
  }
  if (carrier) {
    const uint32_t* src = crc_slice + (tcd.order == 24 ? CRC_SLICE_24A : CRC_SLICE_16) * CRC_SLICE_WORDS;
    uint32_t        t[TW];
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      t[q] = src[tid + q * PK_THREADS];
    }
#pragma unroll
    for (int q = 0; q < TW; ++q) {
      t4t[tid + q * PK_THREADS] = t[q];
    }
  }
#pragma unroll
  for (int r = 0; r < NEL; ++r) {
    if (tid + r * PK_THREADS < G::NE) {
      edge[tid + r * PK_THREADS] = ev[r];
    }
  }
  for (int m = tid; m <= G::M; m += PK_THREADS) {
    row_start[m] = static_cast<uint16_t>(G::rs(m));
  }
  // ---- Message bytes (ldpc_segmenter_tx_impl.cpp:144): TB(+TB CRC) bytes, zero padding / CRC slot / fillers. ----
  if (tfast) {
    __syncthreads();  // t4t complete
    const int order  = static_cast<int>(tcd.order);
    const int nb     = static_cast<int>(tcd.nbytes);
    uint32_t  rem[2] = {0u, 0u};
    // Whole 4-byte words (the TB size is a multiple of 4 here): one slice-by-4 step each, the two chunks interleaved.
#pragma unroll
    for (int q = 0; q < TCS / 4; ++q) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = tid + h * PK_THREADS;
        if (c * TCS + 4 * q < nb) {
          rem[h] = crc_step4(rem[h], __builtin_bswap32(tw[h][q]), order, t4t);
        }
      }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if ((tid + h * PK_THREADS) * TCS < nb) {
        acc ^= gf2_mulmod(rem[h], tm[h], order, tcd.poly);
      }
    }
    acc = wave_xor(acc);
    if ((tid % WAVE) == 0) {
      red[tid / WAVE] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < PK_THREADS / WAVE; ++w) {
      tb_crc ^= red[w];
    }
  } else if (carrier) {
    __syncthreads();  // t4t complete
    const uint8_t* tbp = tbs + tcd.byte_offset;
    tb_crc = block_crc_slice4<16>([tbp](int i) { return tbp[i]; }, static_cast<int>(tcd.nbytes),
                                  crc_tables + tcd.table, static_cast<int>(tcd.order), tcd.poly, t4t, red);
  }
  ENC_STAMP(1);
#pragma unroll
  for (int r = 0; r < MB; ++r) {
    const int q = tid + r * PK_THREADS;
    if (q < nkb) {
      const uint32_t p = d.tb_bit_offset + 8u * static_cast<uint32_t>(q);
      uint32_t       b = byte[r];
      if (q < nd8 && p >= d.tb_bits) {
        b = (tb_crc >> (d.tb_crc_len - 8u - (p - d.tb_bits))) & 0xffu;
      }
      msg[q] = static_cast<uint8_t>(b);
    }
  }
  ENC_STAMP(2);
  if (has_cbc) {
    __syncthreads();  // msg and lut_b complete
    const uint32_t crc = block_crc_slice4<CB_CS>([](int q) { return msg[q]; }, cb_bytes, crc_tables + d.crc_table, 24,
                                                 0x1800063u, t4b, red, pre_m, m0);
    if (tid < 3) {
      msg[d.used / 8 + tid] = static_cast<uint8_t>(crc >> (16 - 8 * tid));
    }
  }
  __syncthreads();
  ENC_STAMP(3);
  // ---- Message words: node c word k = message bits 32 (c W + k) .. + 31. ----
  const uint32_t* msg32 = reinterpret_cast<const uint32_t*>(msg);
  for (int q = tid; q < K * W; q += PK_THREADS) {
    cw[q] = bytes_bitrev(msg32[q]);
  }
  if (tid < 4 * WMAX) {
    lam[tid] = 0u;
  }
  __syncthreads();
  ENC_STAMP(4);
  // ---- Core rows 0..3: lambda_m = sum of the rotated information nodes (32 rows per task). Each (row, word) is
  // split into CH edge chunks over the workgroup's lanes (every window load of a chunk in flight at once); the partial
  // sums are XORed into lam (zeroed with the message) by LDS atomics. ----
  {
    const int CH     = (W <= 10) ? 3 : 2;  // 4 W CH <= PK_THREADS
    const int ntask  = 4 * W * CH;
    if (tid < ntask) {
      const int m     = tid / (W * CH);
      const int rem   = tid - m * W * CH;
      const int ch    = rem / W;
      const int k     = rem - ch * W;
      const int rs    = row_start[m];
      const int deg   = row_start[m + 1] - rs;
      const int per   = (deg + CH - 1) / CH;
      const int e_beg = rs + ch * per;
      const int e_end = min(e_beg + per, rs + deg);
      constexpr int MAXCH = (core_max_degree<BG>() + 1) / 2;  // a core row's edges over at least two chunks
      uint32_t acc = 0;
#pragma unroll
      for (int q = 0; q < MAXCH; ++q) {
        const int e = e_beg + q;
        if (e < e_end) {
          const uint32_t ce = edge[e];
          const int      c  = static_cast<int>(ce >> 16);
          if (c < K) {
            acc ^= col_window(cw + c * W, k, static_cast<int>(ce & 0xffffu), W);
          }
        }
      }
      if (acc != 0u) {
        atomicXor(&lam[m * WMAX + k], acc);
      }
    }
  }
  __syncthreads();
  ENC_STAMP(5);
  // The four core parity nodes are W <= 12 words each, solved one after the other: the first wave alone runs the four
  // dependent steps, ordered by wave-level LDS fences instead of workgroup barriers (window offsets precomputed mod Z
  // per (BG, Z) in the core plan).
  if (tid < WAVE) {
    const core_plan cp = core_plans[d.zpos];
    // P^x p0 = lambda_0 + ... + lambda_3  ->  p0[l] = sum lambda[(l - x) mod Z].
    if (tid < W) {
      const int k   = tid;
      const int o   = cp.o0;
      cw[K * W + k] = col_window(lam, k, o, W) ^ col_window(lam + WMAX, k, o, W) ^
                      col_window(lam + 2 * WMAX, k, o, W) ^ col_window(lam + 3 * WMAX, k, o, W);
    }
    // p_u[(z + s_u) mod Z] = lambda_row[z] + sum_{j != u} p_j[(z + s_j) mod Z]  (same steps as the byte kernel).
#pragma unroll
    for (int step = 0; step < 3; ++step) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (tid < W) {
        const int k   = tid;
        uint32_t  acc = col_window(lam + cp.row[step] * WMAX, k, cp.orow[step], W);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int oj = cp.oj[step][j];
          if (oj >= 0) {
            acc ^= col_window(cw + (K + j) * W, k, oj, W);
          }
        }
        cw[(K + cp.unk[step]) * W + k] = acc;
      }
    }
  }
  __syncthreads();
  ENC_STAMP(6);
  // ---- Extension parity (identity extension), every needed row in parallel. ----
  const int n_ext = d.n_ext;
  for (int task = tid; task < n_ext * W; task += PK_THREADS) {
    const int r = task / W, k = task - r * W;
    uint32_t  acc = 0;
    for (int e = row_start[4 + r]; e < row_start[5 + r] - 1; ++e) {  // the row's last edge is its own (identity) node
      const uint32_t ce = edge[e];
      acc ^= col_window(cw + (ce >> 16) * W, k, static_cast<int>(ce & 0xffffu), W);
    }
    cw[(K + 4 + r) * W + k] = acc;
  }
  __syncthreads();
  ENC_STAMP(7);
  // ---- Rate matching + interleaving + packing. ----
  const pk_rm rm{cw, d.v0, d.Ncb - d.filler, static_cast<uint32_t>((K - 2) * Z - d.filler), d.filler,
                 static_cast<uint32_t>(2 * Z)};
  switch (d.Qm) {
    case 1: rate_match_packed<1>(d, rm, out_words); break;
    case 2: rate_match_packed<2>(d, rm, out_words); break;
    case 4: rate_match_packed<4>(d, rm, out_words); break;
    case 6: rate_match_packed<6>(d, rm, out_words); break;
    default: rate_match_packed<8>(d, rm, out_words); break;
  }
  ENC_STAMP(8);
  ENC_PROF(10, __builtin_amdgcn_s_memrealtime());
}

} // namespace

#ifdef ENC_PROFILE
int debug_read_encoder_profile(uint64_t* dst, size_t n)
{
  const size_t max = static_cast<size_t>(ENC_PROF_CBS) * ENC_PROF_SLOTS;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_enc_prof), (n < max ? n : max) * sizeof(uint64_t)) == hipSuccess ? 0
                                                                                                                : -1;
}
#endif

void launch_pdsch_encode_packed(int              bg,
                                const enc_desc*  d_desc,
                                int              nof_cbs,
                                const uint8_t*   d_tbs,
                                const uint32_t*  d_tb_crcs,
                                const tb_crc_desc* d_tb_inline,
                                uint32_t*        d_out_words,
                                const uint16_t*  d_shifts,
                                const core_plan* d_core_plans,
                                const uint32_t*  d_crc_tables,
                                const uint32_t*  d_crc_slice,
                                hipStream_t      s)
{
  if (nof_cbs <= 0) {
    return;
  }
  if (bg == 1) {
    pdsch_encode_packed_kernel<1><<<nof_cbs, PK_THREADS, 0, s>>>(d_desc, d_tbs, d_tb_crcs, d_tb_inline, d_out_words,
                                                                  d_shifts, d_core_plans, d_crc_tables, d_crc_slice);
  } else {
    pdsch_encode_packed_kernel<2><<<nof_cbs, PK_THREADS, 0, s>>>(d_desc, d_tbs, d_tb_crcs, d_tb_inline, d_out_words,
                                                                  d_shifts, d_core_plans, d_crc_tables, d_crc_slice);
  }
}

void launch_tb_crc(const tb_crc_desc*  d_desc,
                   const tb_crc_slice* d_slices,
                   int                 nof_slices,
                   const uint8_t*      d_tbs,
                   uint32_t*           d_crcs,
                   const uint32_t*     d_crc_tables,
                   hipStream_t         s)
{
  if (nof_slices > 0) {
    tb_crc_kernel<<<nof_slices, 256, 0, s>>>(d_desc, d_slices, d_tbs, d_crcs, d_crc_tables);
  }
}

void launch_pdsch_encode(int              bg,
                         const enc_desc*  d_desc,
                         int              nof_cbs,
                         int              block_threads,
                         const uint8_t*   d_tbs,
                         const uint32_t*  d_tb_crcs,
                         uint32_t*        d_out_words,
                         const uint16_t*  d_shifts,
                         const core_plan* d_core_plans,
                         const uint32_t*  d_crc_tables,
                         hipStream_t      s)
{
  if (nof_cbs <= 0) {
    return;
  }
  if (bg == 1) {
    pdsch_encode_kernel<1><<<nof_cbs, block_threads, 0, s>>>(d_desc, d_tbs, d_tb_crcs, d_out_words, d_shifts,
                                                              d_core_plans, d_crc_tables);
  } else {
    pdsch_encode_kernel<2><<<nof_cbs, block_threads, 0, s>>>(d_desc, d_tbs, d_tb_crcs, d_out_words, d_shifts,
                                                              d_core_plans, d_crc_tables);
  }
}

} // namespace srsgpu
