// Block-wide CRC of a byte string on gfx950 (TS 38.212 §5.1, crc_calculator_generic_impl.cpp:64 calculate_byte:
// zero initial remainder, MSB first). Each of the 256 lanes computes the CRC of a contiguous chunk with a byte table,
// then chunks are combined pairwise: CRC(A|B) = CRC(A) * x^(8|B|) + CRC(B) mod g. The message is conceptually
// front-padded with zero bytes to a multiple of the chunk size (leading zeros do not change a zero-initialised CRC).
#pragma once

#include "common.h"

namespace srsgpu {

/// a(x) * b(x) mod g(x) over GF(2) for polynomials of degree < order (g includes the x^order term).
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b, uint32_t g, int order)
{
  const uint32_t high = 1u << order;
  uint32_t       r    = 0;
  for (int i = order - 1; i >= 0; --i) {
    r <<= 1;
    if (r & high) {
      r ^= g;
    }
    if ((b >> i) & 1u) {
      r ^= a;
    }
  }
  return r;
}

/// CRC (order 8..24, g including x^order) of data[0..n) computed by the first 256 lanes of the workgroup (any larger
/// lanes only take part in the barriers). `table` and `part` are 256-entry LDS scratch arrays. Returns the CRC in every
/// lane. Must be called by all lanes.
__device__ inline uint32_t block_crc_bytes(const uint8_t* data, int n, int order, uint32_t g, uint32_t* table,
                                           uint32_t* part)
{
  const uint32_t mask = (1u << order) - 1u;
  const bool     in   = threadIdx.x < 256u;
  if (in) {
    uint32_t r = static_cast<uint32_t>(threadIdx.x) << (order - 8);
    for (int k = 0; k < 8; ++k) {
      r <<= 1;
      if (r & (1u << order)) {
        r ^= g;
      }
    }
    table[threadIdx.x] = r & mask;
  }
  __syncthreads();
  const int cs  = (n + 255) / 256;
  const int pad = cs * 256 - n;
  uint32_t  rem = 0;
  for (int p = threadIdx.x * cs; in && p < (threadIdx.x + 1) * cs; ++p) {
    const int i = p - pad;
    if (i >= 0) {
      rem = ((rem << 8) ^ table[((rem >> (order - 8)) ^ data[i]) & 0xffu]) & mask;
    }
  }
  if (in) {
    part[threadIdx.x] = rem;
  }
  __syncthreads();
  uint32_t f = 1u;  // x^(8 cs) mod g by square-and-multiply
  {
    uint32_t base = 2u;
    uint32_t e    = 8u * static_cast<uint32_t>(cs);
    while (e) {
      if (e & 1u) {
        f = gf2_mulmod(f, base, g, order);
      }
      base = gf2_mulmod(base, base, g, order);
      e >>= 1;
    }
  }
  for (int step = 1; step < 256; step <<= 1) {
    if (in && (threadIdx.x % (2 * step)) == 0) {
      part[threadIdx.x] = gf2_mulmod(part[threadIdx.x], f, g, order) ^ part[threadIdx.x + step];
    }
    f = gf2_mulmod(f, f, g, order);
    __syncthreads();
  }
  const uint32_t crc = part[0];
  __syncthreads();
  return crc;
}

/// CRC of data[0..nbytes) from the per-bit contribution table P of the message length L = 8 * nbytes
/// (P[i] = x^(order + L - 1 - i) mod g, 16-byte aligned): the CRC is the XOR of P[i] over the set message bits. Each
/// lane takes whole bytes and reads their 8 contributions as two 16-byte vectors (no dependent chain, no GF(2)
/// products). `red` is LDS scratch of one word per wave. Returns the CRC in every lane; all lanes must call it.
__device__ inline uint32_t block_crc_table(const uint8_t* data, int nbytes, const uint32_t* P, uint32_t* red)
{
  uint32_t acc = 0;
  for (int j = threadIdx.x; j < nbytes; j += blockDim.x) {
    const uint32_t byte = data[j];
    const uint4*   p4   = reinterpret_cast<const uint4*>(P + 8 * j);
    const uint4    a    = p4[0];
    const uint4    b    = p4[1];
    acc ^= (byte & 0x80u) ? a.x : 0u;
    acc ^= (byte & 0x40u) ? a.y : 0u;
    acc ^= (byte & 0x20u) ? a.z : 0u;
    acc ^= (byte & 0x10u) ? a.w : 0u;
    acc ^= (byte & 0x08u) ? b.x : 0u;
    acc ^= (byte & 0x04u) ? b.y : 0u;
    acc ^= (byte & 0x02u) ? b.z : 0u;
    acc ^= (byte & 0x01u) ? b.w : 0u;
  }
  acc = wave_xor(acc);
  if ((threadIdx.x % WAVE) == 0) {
    red[threadIdx.x / WAVE] = acc;
  }
  __syncthreads();
  uint32_t crc = 0;
  for (int w = 0; w < static_cast<int>(blockDim.x / WAVE); ++w) {
    crc ^= red[w];
  }
  __syncthreads();
  return crc;
}

/// Byte table of a CRC (order 8..24, g including x^order) in LDS: lut[t] = t(x) x^order mod g, the remainder update
/// of one byte. Every lane of the workgroup must call it (it ends with a barrier).
__device__ inline void crc_byte_lut(uint32_t* lut, int order, uint32_t g)
{
  const uint32_t mask = (1u << order) - 1u;
  for (uint32_t t = threadIdx.x; t < 256u; t += blockDim.x) {
    uint32_t r = t << (order - 8);
    for (int k = 0; k < 8; ++k) {
      r <<= 1;
      if (r & (1u << order)) {
        r ^= g;
      }
    }
    lut[t] = r & mask;
  }
  __syncthreads();
}

/// r(x) M(x) mod g(x) for r, M of degree < order (g including x^order): shift-and-add, no memory.
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t r, uint32_t M, int order, uint32_t g)
{
  uint32_t acc = 0;
#pragma unroll
  for (int b = 23; b >= 0; --b) {  // M < 2^order: the iterations above order - 1 leave acc at 0
    acc = (acc << 1) ^ (((acc >> (order - 1)) & 1u) ? g : 0u);
    acc ^= ((M >> b) & 1u) ? r : 0u;
  }
  return acc;
}

/// CRC of data[0..nbytes) (global or LDS) by chunks: every lane runs the byte-table CRC over CS-byte chunks, then
/// moves each chunk remainder r to the end of the message: r(x) x^(8 (nbytes - end)) mod g, with the power read from
/// the per-bit contribution table P of the message length L = 8 nbytes (P[j] = x^(order + L - 1 - j) mod g, so the
/// power is P[8 end + order - 1]; below x^order it is the monomial itself) and the product formed by shift-and-add in
/// registers: one table load per chunk instead of one per remainder bit (those uncoalesced loads made the kernels
/// texture-addresser bound). `lut` from crc_byte_lut; `red` one word per wave of LDS scratch. All lanes must call it;
/// returns the CRC in every lane.
/// [begin, end) (begin a multiple of CS; default the whole message) restricts the sum to that byte range's chunks: their
/// contribution to the CRC of the whole nbytes-byte message (the CRC is linear, so slices XOR together).
/// One 4-byte step of the slice-by-4 CRC (order 16 or 24): r' = (r x^32 + m x^order) mod g, m = the next four message
/// bytes MSB first; T = the four byte tables T_k[v] = v x^(order + 8 k) mod g (4 x 256 words, context table
/// CRC_SLICE_WORDS staged in LDS): four independent lookups instead of a chain of four.
__device__ __forceinline__ uint32_t crc_step4(uint32_t r, uint32_t m, int order, const uint32_t* T)
{
  const uint32_t u = (r << (32 - order)) ^ m;
  return T[u & 0xffu] ^ T[256u + ((u >> 8) & 0xffu)] ^ T[512u + ((u >> 16) & 0xffu)] ^ T[768u + (u >> 24)];
}

/// block_crc_chunks with the slice-by-4 tables T (T_0 is the byte table): whole 4-byte words of a chunk in one step
/// each, a trailing partial word byte by byte. Same results.
template <int CS, typename Data>
__device__ inline uint32_t block_crc_slice4(Data data, int nbytes, const uint32_t* P, int order, uint32_t g,
                                            const uint32_t* T, uint32_t* red, bool have_m0 = false, uint32_t m0 = 0)
{
  static_assert(CS % 4 == 0, "whole words per chunk");
  const uint32_t mask = (1u << order) - 1u;
  const int      L    = 8 * nbytes;
  const int      nch  = (nbytes + CS - 1) / CS;
  const int      c0   = static_cast<int>(threadIdx.x);
  uint32_t       acc  = 0;
  for (int c = c0; c < nch; c += blockDim.x) {
    const int      b0 = c * CS;
    const int      b1 = min(b0 + CS, nbytes);
    const int      j  = 8 * b1 + order - 1;
    const uint32_t M  = (have_m0 && c == c0) ? m0 : ((j < L) ? P[j] : (1u << (order + L - 1 - j)));
    uint32_t       byte[CS];
#pragma unroll
    for (int k = 0; k < CS; ++k) {
      byte[k] = (b0 + k < b1) ? static_cast<uint32_t>(data(b0 + k)) : 0u;
    }
    uint32_t rem = 0;
#pragma unroll
    for (int w = 0; w < CS / 4; ++w) {
      const int k = 4 * w;
      if (b0 + k + 4 <= b1) {
        rem = crc_step4(rem, (byte[k] << 24) | (byte[k + 1] << 16) | (byte[k + 2] << 8) | byte[k + 3], order, T);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (b0 + k + q < b1) {
            rem = ((rem << 8) ^ T[((rem >> (order - 8)) ^ byte[k + q]) & 0xffu]) & mask;
          }
        }
      }
    }
    acc ^= gf2_mulmod(rem, M, order, g);
  }
  acc = wave_xor(acc);
  if ((threadIdx.x % WAVE) == 0) {
    red[threadIdx.x / WAVE] = acc;
  }
  __syncthreads();
  uint32_t crc = 0;
  for (int w = 0; w < static_cast<int>((blockDim.x + WAVE - 1) / WAVE); ++w) {
    crc ^= red[w];
  }
  __syncthreads();
  return crc;
}

/// The power M of chunk c of an nbytes-byte message (see block_crc_chunks), for a caller that issues the table load
/// early (c < number of chunks).
template <int CS>
__device__ __forceinline__ uint32_t crc_chunk_power(int c, int nbytes, const uint32_t* P, int order)
{
  const int L  = 8 * nbytes;
  const int b1 = min((c + 1) * CS, nbytes);
  const int j  = 8 * b1 + order - 1;
  return (j < L) ? P[j] : (1u << (order + L - 1 - j));
}

template <int CS, typename Data>
__device__ inline uint32_t block_crc_chunks(Data data, int nbytes, const uint32_t* P, int order, uint32_t g,
                                            const uint32_t* lut, uint32_t* red, int begin = 0, int end = -1,
                                            bool have_m0 = false, uint32_t m0 = 0)
{
  const uint32_t mask = (1u << order) - 1u;
  const int      L    = 8 * nbytes;
  const int      nch  = ((end < 0 ? nbytes : end) + CS - 1) / CS;
  const int      c0   = begin / CS + static_cast<int>(threadIdx.x);
  uint32_t       acc  = 0;
  for (int c = c0; c < nch; c += blockDim.x) {
    const int b0  = c * CS;
    const int b1  = min(b0 + CS, nbytes);
    const int j   = 8 * b1 + order - 1;
    // Issued before the chunk's serial chain; m0 = the lane's first power, loaded by the caller (crc_chunk_power).
    const uint32_t M = (have_m0 && c == c0) ? m0 : ((j < L) ? P[j] : (1u << (order + L - 1 - j)));
    // The chunk's bytes are all loaded before the table chain starts (a rolled loop waited for each load in turn).
    uint32_t byte[CS];
#pragma unroll
    for (int k = 0; k < CS; ++k) {
      byte[k] = (b0 + k < b1) ? static_cast<uint32_t>(data(b0 + k)) : 0u;
    }
    uint32_t rem = 0;
#pragma unroll
    for (int k = 0; k < CS; ++k) {
      if (b0 + k < b1) {
        rem = ((rem << 8) ^ lut[((rem >> (order - 8)) ^ byte[k]) & 0xffu]) & mask;
      }
    }
    acc ^= gf2_mulmod(rem, M, order, g);
  }
  acc = wave_xor(acc);
  if ((threadIdx.x % WAVE) == 0) {
    red[threadIdx.x / WAVE] = acc;
  }
  __syncthreads();
  uint32_t crc = 0;
  for (int w = 0; w < static_cast<int>((blockDim.x + WAVE - 1) / WAVE); ++w) {
    crc ^= red[w];
  }
  __syncthreads();
  return crc;
}

} // namespace srsgpu
