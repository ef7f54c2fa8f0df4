// Reference-side binding (the file a srsRAN maintainer adds, e.g. as lib/phy/upper/channel_coding/ldpc/
// ldpc_decoder_gpu.cpp): an srsran::ldpc_decoder implemented over the srsgpu C ABI, so that
// create_ldpc_decoder_factory_sw("gpu") and every caller of ldpc_decoder::decode() (pusch_codeblock_decoder.cpp:45)
// run the MI355X kernels unchanged. Per codeblock: the LLRs and the previous output go through pinned staging buffers
// with asynchronous copies on the instance's own stream, and the decode runs a plan cached per codeblock configuration
// (no allocation, no device-wide synchronisation in steady state). oracle/build_hal.sh links this file with the
// reference's own pusch_codeblock_decoder and tests/test_hal_gpu.py runs it on the GPU.
#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/upper/channel_coding/crc_calculator.h"
#include "srsran/phy/upper/channel_coding/channel_coding_factories.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h"
#include "srsgpu_phy.h"
#include <hip/hip_runtime.h>
#include <cstring>
#include <list>
#include <stdexcept>
#include <vector>

namespace srsran {

/// LDPC decoder running on an MI355X through libsrsgpu_phy.so. One instance per worker thread (like the SW decoders);
/// device and pinned buffers are sized for the largest codeblock once.
class ldpc_decoder_gpu : public ldpc_decoder
{
public:
  explicit ldpc_decoder_gpu(srsgpu_context* ctx_, bool generic_arithmetic = false) :
    ctx(ctx_), impl(generic_arithmetic ? SRSGPU_LDPC_IMPL_GENERIC : SRSGPU_LDPC_IMPL_SIMD)
  {
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d_llr, MAX_LLRS) != hipSuccess || hipMalloc(&d_out, MAX_OUT) != hipSuccess ||
        hipMalloc(&d_iters, sizeof(int32_t)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&h_llr), MAX_LLRS) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&h_out), MAX_OUT) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&h_iters), sizeof(int32_t)) != hipSuccess) {
      throw std::runtime_error("ldpc_decoder_gpu: HIP allocation failed");
    }
  }

  ~ldpc_decoder_gpu() override
  {
    for (auto& e : cache) {
      srsgpu_ldpc_decoder_plan_destroy(e.plan);
    }
    (void)hipFree(d_llr);
    (void)hipFree(d_out);
    (void)hipFree(d_iters);
    (void)hipHostFree(h_llr);
    (void)hipHostFree(h_out);
    (void)hipHostFree(h_iters);
    (void)hipStreamDestroy(stream);
  }

  std::optional<unsigned> decode(bit_buffer&                      output,
                                 span<const log_likelihood_ratio> input,
                                 crc_calculator*                  crc,
                                 const configuration&             cfg) override
  {
    srsgpu_ldpc_decoder_config c;
    std::memset(&c, 0, sizeof(c));
    c.base_graph      = (cfg.block_conf.tb_common.base_graph == ldpc_base_graph_type::BG1) ? 1 : 2;
    c.crc_poly        = (crc != nullptr) ? static_cast<uint8_t>(crc->get_generator_poly()) : SRSGPU_CRC_NONE;
    c.lifting_size    = static_cast<uint16_t>(cfg.block_conf.tb_common.lifting_size);
    c.nof_filler_bits = static_cast<uint16_t>(cfg.block_conf.cb_specific.nof_filler_bits);
    c.nof_crc_bits    = static_cast<uint8_t>(cfg.block_conf.cb_specific.nof_crc_bits);
    c.max_iterations  = static_cast<uint8_t>(cfg.algorithm_conf.max_iterations);
    c.scaling_factor  = cfg.algorithm_conf.scaling_factor;
    c.nof_llrs        = static_cast<uint32_t>(input.size());
    if (input.size() > MAX_LLRS) {
      throw std::runtime_error("ldpc_decoder_gpu: input longer than a codeblock");
    }
    srsgpu_ldpc_decoder_plan* plan = plan_for(c);
    // The output keeps its previous content when the decoder does not run (ldpc_decoder_impl.cpp:100).
    span<uint8_t> packed = output.get_buffer();
    std::memcpy(h_out, packed.data(), packed.size());
    std::memcpy(h_llr, input.data(), input.size());
    (void)hipMemcpyAsync(d_out, h_out, packed.size(), hipMemcpyHostToDevice, stream);
    (void)hipMemcpyAsync(d_llr, h_llr, input.size(), hipMemcpyHostToDevice, stream);
    if (srsgpu_ldpc_decoder_plan_execute(plan, d_llr, d_out, d_iters, stream) != SRSGPU_OK) {
      throw std::runtime_error(srsgpu_last_error());
    }
    (void)hipMemcpyAsync(h_out, d_out, packed.size(), hipMemcpyDeviceToHost, stream);
    (void)hipMemcpyAsync(h_iters, d_iters, sizeof(int32_t), hipMemcpyDeviceToHost, stream);
    if (hipStreamSynchronize(stream) != hipSuccess) {
      throw std::runtime_error("ldpc_decoder_gpu: stream synchronisation failed");
    }
    std::memcpy(packed.data(), h_out, packed.size());
    if (*h_iters < 0) {
      return std::nullopt;
    }
    return static_cast<unsigned>(*h_iters);
  }

private:
  static constexpr size_t   MAX_LLRS        = 66 * 384;
  static constexpr size_t   MAX_OUT         = (22 * 384 + 7) / 8;
  static constexpr unsigned PLAN_CACHE_SIZE = 32;

  struct cached_plan {
    srsgpu_ldpc_decoder_config key;
    srsgpu_ldpc_decoder_plan*  plan;
  };

  /// The single-codeblock plan of a configuration, from the cache (most recently used first) or created.
  srsgpu_ldpc_decoder_plan* plan_for(const srsgpu_ldpc_decoder_config& key)
  {
    for (auto it = cache.begin(); it != cache.end(); ++it) {
      if (std::memcmp(&it->key, &key, sizeof(key)) == 0) {
        cache.splice(cache.begin(), cache, it);
        return cache.front().plan;
      }
    }
    srsgpu_ldpc_decoder_plan* plan = nullptr;
    if (srsgpu_ldpc_decoder_plan_create(ctx, impl, &key, 1, &plan) != SRSGPU_OK) {
      throw std::runtime_error(srsgpu_last_error());
    }
    cache.push_front({key, plan});
    if (cache.size() > PLAN_CACHE_SIZE) {
      srsgpu_ldpc_decoder_plan_destroy(cache.back().plan);
      cache.pop_back();
    }
    return plan;
  }

  srsgpu_context*        ctx;
  int                    impl;
  hipStream_t            stream  = nullptr;
  int8_t*                d_llr   = nullptr;
  uint8_t*               d_out   = nullptr;
  int32_t*               d_iters = nullptr;
  int8_t*                h_llr   = nullptr;
  uint8_t*               h_out   = nullptr;
  int32_t*               h_iters = nullptr;
  std::list<cached_plan> cache;
};

/// Factory, the counterpart of create_ldpc_decoder_factory_sw() (channel_coding_factories.h).
class ldpc_decoder_factory_gpu : public ldpc_decoder_factory
{
public:
  explicit ldpc_decoder_factory_gpu(int device)
  {
    if (srsgpu_context_create(device, &ctx) != SRSGPU_OK) {
      throw std::runtime_error(srsgpu_last_error());
    }
  }
  ~ldpc_decoder_factory_gpu() override { srsgpu_context_destroy(ctx); }
  std::unique_ptr<ldpc_decoder> create() override { return std::make_unique<ldpc_decoder_gpu>(ctx); }

private:
  srsgpu_context* ctx = nullptr;
};

std::shared_ptr<ldpc_decoder_factory> create_ldpc_decoder_factory_gpu(int device)
{
  return std::make_shared<ldpc_decoder_factory_gpu>(device);
}

} // namespace srsran
