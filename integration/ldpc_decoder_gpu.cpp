// Reference-side binding (the file a srsRAN maintainer adds, e.g. as lib/phy/upper/channel_coding/ldpc/
// ldpc_decoder_gpu.cpp): an srsran::ldpc_decoder implemented over the srsgpu C ABI, so that
// create_ldpc_decoder_factory_sw("gpu") and every caller of ldpc_decoder::decode() (pusch_codeblock_decoder.cpp:45)
// run the MI355X kernels unchanged. tests/test_integration_compile.py compiles this file against the reference
// headers (compile-only; not part of the product build).
#include "srsran/adt/bit_buffer.h"
#include "srsran/phy/upper/channel_coding/crc_calculator.h"
#include "srsran/phy/upper/channel_coding/channel_coding_factories.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h"
#include "srsgpu_phy.h"
#include <hip/hip_runtime.h>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace srsran {

/// LDPC decoder running on an MI355X through libsrsgpu_phy.so. One instance per worker thread (like the SW decoders);
/// device buffers are sized for the largest codeblock once.
class ldpc_decoder_gpu : public ldpc_decoder
{
public:
  explicit ldpc_decoder_gpu(srsgpu_context* ctx_, bool generic_arithmetic = false) :
    ctx(ctx_), impl(generic_arithmetic ? SRSGPU_LDPC_IMPL_GENERIC : SRSGPU_LDPC_IMPL_SIMD)
  {
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d_llr, 66 * 384) != hipSuccess || hipMalloc(&d_out, (22 * 384 + 7) / 8) != hipSuccess ||
        hipMalloc(&d_iters, sizeof(int32_t)) != hipSuccess) {
      throw std::runtime_error("ldpc_decoder_gpu: HIP allocation failed");
    }
  }

  ~ldpc_decoder_gpu() override
  {
    (void)hipFree(d_llr);
    (void)hipFree(d_out);
    (void)hipFree(d_iters);
    (void)hipStreamDestroy(stream);
  }

  std::optional<unsigned> decode(bit_buffer&                      output,
                                 span<const log_likelihood_ratio> input,
                                 crc_calculator*                  crc,
                                 const configuration&             cfg) override
  {
    srsgpu_ldpc_decoder_config c = {};
    c.base_graph      = (cfg.block_conf.tb_common.base_graph == ldpc_base_graph_type::BG1) ? 1 : 2;
    c.crc_poly        = (crc != nullptr) ? static_cast<uint8_t>(crc->get_generator_poly()) : SRSGPU_CRC_NONE;
    c.lifting_size    = static_cast<uint16_t>(cfg.block_conf.tb_common.lifting_size);
    c.nof_filler_bits = static_cast<uint16_t>(cfg.block_conf.cb_specific.nof_filler_bits);
    c.nof_crc_bits    = static_cast<uint8_t>(cfg.block_conf.cb_specific.nof_crc_bits);
    c.max_iterations  = static_cast<uint8_t>(cfg.algorithm_conf.max_iterations);
    c.scaling_factor  = cfg.algorithm_conf.scaling_factor;
    c.nof_llrs        = static_cast<uint32_t>(input.size());
    // The output keeps its previous content when the decoder does not run (ldpc_decoder_impl.cpp:100).
    span<uint8_t> packed = output.get_buffer();
    (void)hipMemcpyAsync(d_out, packed.data(), packed.size(), hipMemcpyHostToDevice, stream);
    (void)hipMemcpyAsync(d_llr, input.data(), input.size(), hipMemcpyHostToDevice, stream);
    if (srsgpu_ldpc_decode(ctx, impl, &c, 1, d_llr, d_out, d_iters, stream) != SRSGPU_OK) {
      throw std::runtime_error(srsgpu_last_error());
    }
    int32_t iters = -1;
    (void)hipMemcpyAsync(packed.data(), d_out, packed.size(), hipMemcpyDeviceToHost, stream);
    (void)hipMemcpyAsync(&iters, d_iters, sizeof(iters), hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    if (iters < 0) {
      return std::nullopt;
    }
    return static_cast<unsigned>(iters);
  }

private:
  srsgpu_context* ctx;
  int             impl;
  hipStream_t     stream  = nullptr;
  int8_t*         d_llr   = nullptr;
  uint8_t*        d_out   = nullptr;
  int32_t*        d_iters = nullptr;
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
  std::unique_ptr<ldpc_decoder> create() override { return std::make_unique<ldpc_decoder_gpu>(ctx); }

private:
  srsgpu_context* ctx = nullptr;
};

std::shared_ptr<ldpc_decoder_factory> create_ldpc_decoder_factory_gpu(int device)
{
  return std::make_shared<ldpc_decoder_factory_gpu>(device);
}

} // namespace srsran
