// Transport-block stage of the PUSCH decoder on gfx950: concatenation of the decoded codeblocks into the transport
// block and the TB CRC24A check, with the reference's HARQ bookkeeping.
//
// Drop-in semantics of pusch_decoder_impl::join_and_notify / concatenate_codeblocks (reference
// lib/phy/upper/channel_processors/pusch/pusch_decoder_impl.cpp:386 and :438): with one codeblock the TB CRC is the
// codeblock CRC and the TB is copied only when it passed; with several codeblocks the TB is assembled (each codeblock
// contributes min(free TB bits, data bits), the last one also carries the 24-bit TB checksum) only when every codeblock
// CRC passed, then CRC24A(TB) is compared with the checksum; a mismatch resets every codeblock CRC flag (:423).
#include "common.h"
#include "crc_device.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {

/// p / d with the magic m = ceil(2^32 / d): the high product never undershoots and overshoots by at most one once
/// p * d >= 2^32 (TB bits up to ~1.3 M x codeblock bits up to 8448), so one correction makes it exact for every p.
__device__ __forceinline__ uint32_t cb_index(uint32_t p, uint32_t d, uint32_t m)
{
  const uint32_t q = __umulhi(p, m);
  return (q * d > p) ? q - 1u : q;
}

/// tb[b] = src(b) for b < bytes, coalesced over the workgroup with 8 loads per lane in flight before the stores (a
/// rolled byte loop waited for each load in turn: ~36 round trips per lane for a 37 KB TB).
template <typename Src>
__device__ __forceinline__ void copy_batched(uint8_t* tb, uint32_t bytes, Src src)
{
  constexpr uint32_t BB = 8;
  for (uint32_t b0 = threadIdx.x; b0 < bytes; b0 += BB * blockDim.x) {
    uint8_t v[BB];
#pragma unroll
    for (uint32_t k = 0; k < BB; ++k) {
      const uint32_t b = b0 + k * blockDim.x;
      v[k]             = b < bytes ? src(b) : uint8_t{0};
    }
#pragma unroll
    for (uint32_t k = 0; k < BB; ++k) {
      const uint32_t b = b0 + k * blockDim.x;
      if (b < bytes) {
        tb[b] = v[k];
      }
    }
  }
}

__global__ __launch_bounds__(1024) void pusch_tb_kernel(const tb_dec_desc* __restrict__ descs,
                                                       uint8_t* __restrict__ cb_crc_ok,
                                                       const uint8_t* __restrict__ cb_msgs,
                                                       uint8_t* __restrict__ tbs,
                                                       uint8_t* __restrict__ tb_crc_ok,
                                                       const uint32_t* __restrict__ crc_tables)
{
  __shared__ uint32_t table[256];
  __shared__ uint32_t part[256];
  const tb_dec_desc d     = descs[blockIdx.x];
  uint8_t*          tb    = tbs + d.tb_offset;
  const uint8_t*    msgs  = cb_msgs + static_cast<size_t>(d.first_cb) * CB_MSG_STRIDE;
  const uint32_t    bytes = d.tbs_bits / 8u;
  // Codeblock CRC flags: loaded first, combined (workgroup AND) only after the speculative TB CRC below.
  int ok = 1;
  for (uint32_t c = threadIdx.x; c < d.nof_cbs; c += blockDim.x) {
    ok &= cb_crc_ok[d.first_cb + c] != 0;
  }
  // TS 38.214 TB sizes make the codeblock data byte-aligned when C > 1 ((TBS + 24) is a multiple of 8 C): then the TB
  // CRC runs straight on the codeblock messages, before (and whatever) the flags say, so that its loads and table
  // chain overlap the flag loads. A TB that does not pass its codeblock CRCs discards it.
  const bool crc_from_msgs = d.nof_cbs > 1 && d.crc_table != NO_CRC_TABLE && (d.cb_data_bits & 7u) == 0;
  uint32_t   crc           = 0;
  if (crc_from_msgs) {
    crc_byte_lut(table, 24, 0x1864cfbu);
    const uint32_t cb_bytes = d.cb_data_bits / 8u;
    const uint32_t magic    = d.data_magic;
    crc = block_crc_chunks<16>(
        [msgs, cb_bytes, magic](int i) {
          const uint32_t cb = __umulhi(8u * static_cast<uint32_t>(i), magic);
          return msgs[cb * CB_MSG_STRIDE + (static_cast<uint32_t>(i) - cb * cb_bytes)];
        },
        static_cast<int>(bytes), crc_tables + d.crc_table, 24, 0x1864cfbu, table, part);
  }
  if (!__syncthreads_and(ok)) {
    if (threadIdx.x == 0) {
      tb_crc_ok[d.tb_index] = 0;
    }
    return;
  }
  if (d.nof_cbs == 1) {
    copy_batched(tb, bytes, [msgs](uint32_t b) { return msgs[b]; });
    if (threadIdx.x == 0) {
      tb_crc_ok[d.tb_index] = 1;
    }
    return;
  }
  // TB bit p comes from codeblock p / cb_data_bits, message bit p % cb_data_bits.
  if ((d.cb_data_bits & 7u) == 0) {
    const uint32_t cb_bytes = d.cb_data_bits / 8u;
    const uint32_t bits     = d.cb_data_bits;
    const uint32_t magic    = d.data_magic;
    copy_batched(tb, bytes, [msgs, cb_bytes, bits, magic](uint32_t b) {
      const uint32_t cb = cb_index(8u * b, bits, magic);
      return msgs[cb * CB_MSG_STRIDE + (b - cb * cb_bytes)];
    });
  }
  for (uint32_t b = threadIdx.x; (d.cb_data_bits & 7u) != 0 && b < bytes; b += blockDim.x) {
    uint32_t byte = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t p  = 8u * b + static_cast<uint32_t>(k);
      const uint32_t cb = cb_index(p, d.cb_data_bits, d.data_magic);
      const uint32_t q  = p - cb * d.cb_data_bits;
      const uint8_t* m  = msgs + cb * CB_MSG_STRIDE;
      byte |= ((static_cast<uint32_t>(m[q >> 3]) >> (7u - (q & 7u))) & 1u) << (7 - k);
    }
    tb[b] = static_cast<uint8_t>(byte);
  }
  if (!crc_from_msgs) {
    __syncthreads();  // the CRC reads the TB back
    if (d.crc_table != NO_CRC_TABLE) {
      crc_byte_lut(table, 24, 0x1864cfbu);
      crc = block_crc_chunks<16>([tb](int i) { return tb[i]; }, static_cast<int>(bytes), crc_tables + d.crc_table,
                                 24, 0x1864cfbu, table, part);
    } else {
      crc = block_crc_bytes(tb, static_cast<int>(bytes), 24, 0x1864cfbu, table, part);
    }
  }
  // Checksum: the 24 bits that follow the last codeblock's TB bits (concatenate_codeblocks, :465).
  const uint32_t last_q = d.tbs_bits - (d.nof_cbs - 1u) * d.cb_data_bits;
  const uint8_t* lm     = msgs + (d.nof_cbs - 1u) * CB_MSG_STRIDE;
  // The 24 bits span at most 4 message bytes: four independent loads, then one 32-bit window shift.
  const uint32_t q0 = last_q >> 3;
  const uint32_t w  = (static_cast<uint32_t>(lm[q0]) << 24) | (static_cast<uint32_t>(lm[q0 + 1]) << 16) |
                     (static_cast<uint32_t>(lm[q0 + 2]) << 8) | static_cast<uint32_t>(lm[q0 + 3]);
  const uint32_t chk = (w >> (8u - (last_q & 7u))) & 0xffffffu;
  const bool crc_ok = (crc == chk);
  if (!crc_ok) {
    for (uint32_t c = threadIdx.x; c < d.nof_cbs; c += blockDim.x) {
      cb_crc_ok[d.first_cb + c] = 0;
    }
  }
  if (threadIdx.x == 0) {
    tb_crc_ok[d.tb_index] = crc_ok ? 1 : 0;
  }
}

/// Large segmented TBs over several workgroups (launch_pusch_tb_sliced): workgroup w owns the TB byte range of
/// slices[w] (TB_SLICE_BYTES, chunk-aligned). It checks the TB's codeblock flags, XORs its range's contribution to the
/// TB CRC (block_crc_chunks over [begin, end) of the codeblock messages: the CRC is linear) into acc[tb] and copies its
/// range into the TB when every flag passed; the TB's last workgroup to finish (counter cnt[tb]) compares the sum with
/// the checksum, writes the TB flag, clears the codeblock flags on a mismatch and resets acc / cnt for the next
/// execute (self-cleaning: graph replays on one stream need no memset). One TB of a single-workgroup launch takes ~15 us
/// on a 37 KB TB (its byte copy and CRC chain on one CU); here the slices run in parallel.
__global__ __launch_bounds__(256) void pusch_tb_slice_kernel(const tb_dec_desc* __restrict__ descs,
                                                            const tb_slice* __restrict__ slices,
                                                            uint8_t* __restrict__ cb_crc_ok,
                                                            const uint8_t* __restrict__ cb_msgs,
                                                            uint8_t* __restrict__ tbs,
                                                            uint8_t* __restrict__ tb_crc_ok,
                                                            const uint32_t* __restrict__ crc_tables,
                                                            uint32_t* __restrict__ acc,
                                                            uint32_t* __restrict__ cnt)
{
  __shared__ uint32_t table[256];
  __shared__ uint32_t part[4];
  __shared__ int      last;
  const tb_slice    sl    = slices[blockIdx.x];
  const tb_dec_desc d     = descs[sl.tb];
  uint8_t*          tb    = tbs + d.tb_offset;
  const uint8_t*    msgs  = cb_msgs + static_cast<size_t>(d.first_cb) * CB_MSG_STRIDE;
  const uint32_t    bytes = d.tbs_bits / 8u;
  int ok = 1;
  for (uint32_t c = threadIdx.x; c < d.nof_cbs; c += blockDim.x) {
    ok &= cb_crc_ok[d.first_cb + c] != 0;
  }
  const bool     all_ok   = __syncthreads_and(ok) != 0;
  const uint32_t cb_bytes = d.cb_data_bits / 8u;
  const uint32_t magic    = d.data_magic;
  if (all_ok) {
    crc_byte_lut(table, 24, 0x1864cfbu);
    const uint32_t part_crc = block_crc_chunks<16>(
        [msgs, cb_bytes, magic](int i) {
          const uint32_t cb = __umulhi(8u * static_cast<uint32_t>(i), magic);
          return msgs[cb * CB_MSG_STRIDE + (static_cast<uint32_t>(i) - cb * cb_bytes)];
        },
        static_cast<int>(bytes), crc_tables + d.crc_table, 24, 0x1864cfbu, table, part, static_cast<int>(sl.begin),
        static_cast<int>(sl.end));
    const uint32_t bits = d.cb_data_bits;
    copy_batched(tb + sl.begin, sl.end - sl.begin, [msgs, cb_bytes, bits, magic, sl](uint32_t r) {
      const uint32_t b  = sl.begin + r;
      const uint32_t cb = cb_index(8u * b, bits, magic);
      return msgs[cb * CB_MSG_STRIDE + (b - cb * cb_bytes)];
    });
    if (threadIdx.x == 0) {
      atomicXor(&acc[sl.tb], part_crc);
    }
  }
  if (threadIdx.x == 0) {
    __threadfence();
    last = (atomicAdd(&cnt[sl.tb], 1u) == sl.nof_slices - 1u) ? 1 : 0;
  }
  __syncthreads();
  if (last == 0) {
    return;
  }
  // The TB's last workgroup: every other slice's contribution is in acc[tb].
  __threadfence();
  bool crc_ok = false;
  if (all_ok) {
    const uint32_t crc    = atomicOr(&acc[sl.tb], 0u);
    const uint32_t last_q = d.tbs_bits - (d.nof_cbs - 1u) * d.cb_data_bits;
    const uint8_t* lm     = msgs + (d.nof_cbs - 1u) * CB_MSG_STRIDE;
    const uint32_t q0     = last_q >> 3;
    const uint32_t w      = (static_cast<uint32_t>(lm[q0]) << 24) | (static_cast<uint32_t>(lm[q0 + 1]) << 16) |
                       (static_cast<uint32_t>(lm[q0 + 2]) << 8) | static_cast<uint32_t>(lm[q0 + 3]);
    crc_ok = crc == ((w >> (8u - (last_q & 7u))) & 0xffffffu);
    if (!crc_ok) {
      for (uint32_t c = threadIdx.x; c < d.nof_cbs; c += blockDim.x) {
        cb_crc_ok[d.first_cb + c] = 0;
      }
    }
  }
  if (threadIdx.x == 0) {
    tb_crc_ok[d.tb_index] = crc_ok ? 1 : 0;
    acc[sl.tb]            = 0u;
    cnt[sl.tb]            = 0u;
  }
}

} // namespace

void launch_pusch_tb(const tb_dec_desc* d_desc,
                     int                nof_tbs,
                     int                threads,
                     uint8_t*           d_cb_crc_ok,
                     const uint8_t*     d_cb_msgs,
                     uint8_t*           d_tbs,
                     uint8_t*           d_tb_crc_ok,
                     const uint32_t*    d_crc_tables,
                     hipStream_t        stream)
{
  if (nof_tbs > 0) {
    pusch_tb_kernel<<<nof_tbs, threads, 0, stream>>>(d_desc, d_cb_crc_ok, d_cb_msgs, d_tbs, d_tb_crc_ok, d_crc_tables);
  }
}

void launch_pusch_tb_sliced(const tb_dec_desc* d_desc,
                            const tb_slice*    d_slices,
                            int                nof_slices,
                            uint8_t*           d_cb_crc_ok,
                            const uint8_t*     d_cb_msgs,
                            uint8_t*           d_tbs,
                            uint8_t*           d_tb_crc_ok,
                            const uint32_t*    d_crc_tables,
                            uint32_t*          d_acc,
                            uint32_t*          d_cnt,
                            hipStream_t        stream)
{
  if (nof_slices > 0) {
    pusch_tb_slice_kernel<<<nof_slices, 256, 0, stream>>>(d_desc, d_slices, d_cb_crc_ok, d_cb_msgs, d_tbs, d_tb_crc_ok,
                                                          d_crc_tables, d_acc, d_cnt);
  }
}

} // namespace srsgpu
