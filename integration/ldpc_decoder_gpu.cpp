// Reference-side binding (the file a srsRAN maintainer adds, e.g. as lib/phy/upper/channel_coding/ldpc/
// ldpc_decoder_gpu.cpp): an srsran::ldpc_decoder implemented over the srsgpu C ABI, so that
// create_ldpc_decoder_factory_sw("gpu") and every caller of ldpc_decoder::decode() (pusch_codeblock_decoder.cpp:45)
// run the MI355X kernels unchanged. Per codeblock: the LLRs and the previous output go through pinned staging buffers
// with asynchronous copies on the instance's own stream, and the decode runs a plan cached per codeblock configuration
// (no allocation, no device-wide synchronisation in steady state). Every HIP call is checked (a failure throws). The
// srsgpu context is shared by the factory and every decoder it creates (integration/gpu_context.h). oracle/build_hal.sh
// links this file with the reference's own pusch_codeblock_decoder and tests/test_hal_gpu.py runs it on the GPU.
#include "gpu_context.h"
#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/upper/channel_coding/crc_calculator.h"
#include "srsran/phy/upper/channel_coding/channel_coding_factories.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h"
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
  explicit ldpc_decoder_gpu(std::shared_ptr<srsgpu_context> owner_, bool generic_arithmetic = false) :
    owner(std::move(owner_)), ctx(owner.get()), impl(generic_arithmetic ? SRSGPU_LDPC_IMPL_GENERIC : SRSGPU_LDPC_IMPL_SIMD)
  {
    check(hipSetDevice(srsgpu_context_device(ctx)), "device");
    check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream");
    check(hipMalloc(&d_llr, MAX_LLRS), "LLR buffer");
    check(hipMalloc(&d_out, MAX_OUT), "output buffer");
    check(hipMalloc(&d_iters, sizeof(int32_t)), "iteration counter");
    check(hipHostMalloc(reinterpret_cast<void**>(&h_llr), MAX_LLRS), "pinned LLRs");
    check(hipHostMalloc(reinterpret_cast<void**>(&h_out), MAX_OUT), "pinned output");
    check(hipHostMalloc(reinterpret_cast<void**>(&h_iters), sizeof(int32_t)), "pinned iteration counter");
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
    gpu::device_scope dev_scope(ctx, "ldpc_decoder_gpu");
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
    check(hipMemcpyAsync(d_out, h_out, packed.size(), hipMemcpyHostToDevice, stream), "output upload");
    check(hipMemcpyAsync(d_llr, h_llr, input.size(), hipMemcpyHostToDevice, stream), "LLR upload");
    gpu::srsgpu_check(srsgpu_ldpc_decoder_plan_execute(plan, d_llr, d_out, d_iters, stream), "ldpc_decoder_gpu");
    check(hipMemcpyAsync(h_out, d_out, packed.size(), hipMemcpyDeviceToHost, stream), "output download");
    check(hipMemcpyAsync(h_iters, d_iters, sizeof(int32_t), hipMemcpyDeviceToHost, stream), "iteration download");
    check(hipStreamSynchronize(stream), "synchronise");
    std::memcpy(packed.data(), h_out, packed.size());
    if (*h_iters < 0) {
      return std::nullopt;
    }
    return static_cast<unsigned>(*h_iters);
  }

private:
  static void check(hipError_t e, const char* what) { gpu::hip_check(e, "ldpc_decoder_gpu", what); }

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
    gpu::srsgpu_check(srsgpu_ldpc_decoder_plan_create(ctx, impl, &key, 1, &plan), "ldpc_decoder_gpu");
    cache.push_front({key, plan});
    if (cache.size() > PLAN_CACHE_SIZE) {
      srsgpu_ldpc_decoder_plan_destroy(cache.back().plan);
      cache.pop_back();
    }
    return plan;
  }

  std::shared_ptr<srsgpu_context> owner;
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
  explicit ldpc_decoder_factory_gpu(int device) : ctx(gpu::shared_context(device)) {}
  std::unique_ptr<ldpc_decoder> create() override { return std::make_unique<ldpc_decoder_gpu>(ctx); }

private:
  std::shared_ptr<srsgpu_context> ctx;
};

std::shared_ptr<ldpc_decoder_factory> create_ldpc_decoder_factory_gpu(int device)
{
  return std::make_shared<ldpc_decoder_factory_gpu>(device);
}

} // namespace srsran
