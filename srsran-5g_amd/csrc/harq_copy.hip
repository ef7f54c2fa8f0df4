// HARQ soft-buffer transfers between a persistent per-codeblock arena and a slot batch's contiguous HARQ buffer
// (srsgpu_harq_copy, include/srsgpu_phy.h). The reference keeps each codeblock's soft bits in the rx buffer pool,
// addressed by its absolute codeblock identifier (rx_buffer.h:65 get_absolute_codeblock_id, :72
// get_codeblock_soft_bits), across slots; a batched PUSCH decoder plan addresses them contiguously per transport
// block. One workgroup per codeblock, 16-byte vector copies (every offset and length is a multiple of 16 for the LDPC
// lengths N = 64 Z / 48 Z at even Z; a byte loop otherwise). HBM-bound: 2 bytes moved per soft bit.
// Also srsgpu_copy_spans: a list of copies as one launch (the slot batches' rx grids, read in place from mapped host
// memory into their HBM grid slots).
#include "srsgpu_internal.h"
#include "capi_internal.h"
#include <algorithm>

namespace {

/// MULTI: the job's arena is arenas[j.arena] (several sectors' rx buffer pools in one launch).
template <bool MULTI>
__global__ void __launch_bounds__(256) harq_copy_kernel(int8_t* __restrict__ arena,
                                                        int8_t* const* __restrict__ arenas,
                                                        uint32_t arena_stride,
                                                        int8_t* __restrict__ batch,
                                                        const srsgpu_harq_copy_job* __restrict__ jobs,
                                                        int to_arena)
{
  const srsgpu_harq_copy_job j = jobs[blockIdx.x];
  int8_t*       base = MULTI ? arenas[j.arena] : arena;
  int8_t*       a    = base + static_cast<size_t>(j.slot) * arena_stride;
  int8_t*       b   = batch + j.batch_offset;
  const int8_t* src = to_arena ? b : a;
  int8_t*       dst = to_arena ? a : b;
  const bool    vec = ((j.batch_offset | j.bytes | arena_stride) & 15u) == 0;
  if (vec) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4*       d4 = reinterpret_cast<uint4*>(dst);
    for (uint32_t i = threadIdx.x; i < j.bytes / 16u; i += blockDim.x) {
      d4[i] = s4[i];
    }
  } else {
    for (uint32_t i = threadIdx.x; i < j.bytes; i += blockDim.x) {
      dst[i] = src[i];
    }
  }
}

/// Span copies: blockIdx.y = span, the x blocks stride over it in 16-byte words (the entry point checks alignment).
__global__ void __launch_bounds__(256) copy_spans_kernel(const srsgpu_copy_span* __restrict__ spans)
{
  const srsgpu_copy_span sp = spans[blockIdx.y];
  const uint4*           s4 = reinterpret_cast<const uint4*>(sp.src);
  uint4*                 d4 = reinterpret_cast<uint4*>(sp.dst);
  const uint64_t         n  = sp.bytes / 16u;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    d4[i] = s4[i];
  }
}

/// Span merges: as copy_spans_kernel, but a 32-bit source word replaces the destination's only when it differs from
/// `sentinel` (the words a producer left unwritten in a sentinel-filled grid).
__global__ void __launch_bounds__(256) merge_spans_kernel(const srsgpu_copy_span* __restrict__ spans, uint32_t sentinel)
{
  const srsgpu_copy_span sp = spans[blockIdx.y];
  const uint4*           s4 = reinterpret_cast<const uint4*>(sp.src);
  uint4*                 d4 = reinterpret_cast<uint4*>(sp.dst);
  const uint64_t         n  = sp.bytes / 16u;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint4    v    = s4[i];
    const uint32_t keep = (v.x != sentinel ? 1u : 0u) | (v.y != sentinel ? 2u : 0u) | (v.z != sentinel ? 4u : 0u) |
                          (v.w != sentinel ? 8u : 0u);
    if (keep == 15u) {
      d4[i] = v;
    } else if (keep != 0u) {
      uint4 o = d4[i];
      o.x     = (keep & 1u) ? v.x : o.x;
      o.y     = (keep & 2u) ? v.y : o.y;
      o.z     = (keep & 4u) ? v.z : o.z;
      o.w     = (keep & 8u) ? v.w : o.w;
      d4[i]   = o;
    }
  }
}

} // namespace

extern "C" int srsgpu_merge_spans(const srsgpu_copy_span* d_spans,
                                  uint32_t                nof_spans,
                                  uint64_t                max_bytes,
                                  uint32_t                sentinel,
                                  void*                   stream)
{
  if ((d_spans == nullptr && nof_spans > 0) || (max_bytes & 15u) != 0) {
    return srsgpu::fail(SRSGPU_ERR_INVALID_ARG, "srsgpu_merge_spans: invalid argument (max_bytes a multiple of 16)");
  }
  if (nof_spans == 0 || max_bytes == 0) {
    return SRSGPU_OK;
  }
  const uint64_t blocks = std::min<uint64_t>(256, (max_bytes / 16u + 255u) / 256u);
  merge_spans_kernel<<<dim3(static_cast<unsigned>(blocks), nof_spans), 256, 0, static_cast<hipStream_t>(stream)>>>(
      d_spans, sentinel);
  const hipError_t err = hipGetLastError();
  return err == hipSuccess ? SRSGPU_OK : srsgpu::fail(SRSGPU_ERR_HIP, "srsgpu_merge_spans: %s", hipGetErrorString(err));
}

extern "C" int srsgpu_copy_spans(const srsgpu_copy_span* d_spans, uint32_t nof_spans, uint64_t max_bytes, void* stream)
{
  if ((d_spans == nullptr && nof_spans > 0) || (max_bytes & 15u) != 0) {
    return srsgpu::fail(SRSGPU_ERR_INVALID_ARG, "srsgpu_copy_spans: invalid argument (max_bytes a multiple of 16)");
  }
  if (nof_spans == 0 || max_bytes == 0) {
    return SRSGPU_OK;
  }
  // Enough workgroups per span that a host-memory source keeps many reads in flight (about 4 KB per workgroup pass).
  const uint64_t blocks = std::min<uint64_t>(256, (max_bytes / 16u + 255u) / 256u);
  copy_spans_kernel<<<dim3(static_cast<unsigned>(blocks), nof_spans), 256, 0, static_cast<hipStream_t>(stream)>>>(
      d_spans);
  const hipError_t err = hipGetLastError();
  return err == hipSuccess ? SRSGPU_OK : srsgpu::fail(SRSGPU_ERR_HIP, "srsgpu_copy_spans: %s", hipGetErrorString(err));
}

extern "C" int srsgpu_harq_copy(srsgpu_context*             ctx,
                                int                         direction,
                                int8_t*                     d_arena,
                                uint32_t                    arena_stride,
                                int8_t*                     d_batch,
                                const srsgpu_harq_copy_job* d_jobs,
                                uint32_t                    nof_jobs,
                                void*                       stream)
{
  if (ctx == nullptr || d_arena == nullptr || d_batch == nullptr || (d_jobs == nullptr && nof_jobs > 0) ||
      (direction != SRSGPU_HARQ_TO_BATCH && direction != SRSGPU_HARQ_TO_ARENA)) {
    return srsgpu::fail(SRSGPU_ERR_INVALID_ARG, "srsgpu_harq_copy: invalid argument");
  }
  if (nof_jobs == 0) {
    return SRSGPU_OK;
  }
  harq_copy_kernel<false><<<nof_jobs, 256, 0, static_cast<hipStream_t>(stream)>>>(
      d_arena, nullptr, arena_stride, d_batch, d_jobs, direction == SRSGPU_HARQ_TO_ARENA ? 1 : 0);
  if (hipGetLastError() != hipSuccess) {
    return srsgpu::fail(SRSGPU_ERR_HIP, "srsgpu_harq_copy: launch failed");
  }
  return SRSGPU_OK;
}

extern "C" int srsgpu_harq_copy_arenas(srsgpu_context*             ctx,
                                       int                         direction,
                                       int8_t* const*              d_arenas,
                                       uint32_t                    arena_stride,
                                       int8_t*                     d_batch,
                                       const srsgpu_harq_copy_job* d_jobs,
                                       uint32_t                    nof_jobs,
                                       void*                       stream)
{
  if (ctx == nullptr || d_arenas == nullptr || d_batch == nullptr || (d_jobs == nullptr && nof_jobs > 0) ||
      (direction != SRSGPU_HARQ_TO_BATCH && direction != SRSGPU_HARQ_TO_ARENA)) {
    return srsgpu::fail(SRSGPU_ERR_INVALID_ARG, "srsgpu_harq_copy_arenas: invalid argument");
  }
  if (nof_jobs == 0) {
    return SRSGPU_OK;
  }
  harq_copy_kernel<true><<<nof_jobs, 256, 0, static_cast<hipStream_t>(stream)>>>(
      nullptr, d_arenas, arena_stride, d_batch, d_jobs, direction == SRSGPU_HARQ_TO_ARENA ? 1 : 0);
  if (hipGetLastError() != hipSuccess) {
    return srsgpu::fail(SRSGPU_ERR_HIP, "srsgpu_harq_copy_arenas: launch failed");
  }
  return SRSGPU_OK;
}
