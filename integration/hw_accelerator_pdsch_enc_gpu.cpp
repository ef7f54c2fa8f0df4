// Reference-side binding: srsran::hal::hw_accelerator_pdsch_enc (include/srsran/hal/phy/upper/channel_processors/
// hw_accelerator_pdsch_enc.h:85-104) over the srsgpu C ABI in transport-block mode (cb_mode = false: the accelerator
// attaches the TB CRC and the CB CRCs, segments, LDPC-encodes and rate-matches), so that the reference's own
// pdsch_encoder_hw_impl (lib/phy/upper/channel_processors/pdsch/pdsch_encoder_hw_impl.cpp) encodes on an MI355X.
//
// The HAL configuration carries the segmentation result (E of the short / long segments) rather than the number of
// layers and channel symbols the srsgpu plan segments from; they follow from it: G = Ea * short + Eb * long, and the
// long segments hold NL * Qm more bits than the short ones (TS 38.212 5.4.2.1), so NL = (Eb - Ea) / Qm (any layer
// count reproduces the segmentation when every segment is short). Plans are cached per configuration. The srsgpu context
// is shared by the factory and every accelerator it creates (integration/gpu_context.h): accelerators outlive it.
#include "gpu_context.h"
#include "hw_accelerator_pusch_dec_gpu.h"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <list>
#include <string>
#include <stdexcept>
#include <vector>

namespace srsran {
namespace hal {

namespace {

constexpr unsigned PLAN_CACHE_SIZE = 64;
constexpr unsigned MAX_TB_BYTES    = 1277992 / 8 + 4;
constexpr unsigned MAX_CW_BYTES    = 2 * 1024 * 1024;

constexpr const char* WHO = "hw_accelerator_pdsch_enc_gpu";

void hip_check(hipError_t e, const char* what)
{
  gpu::hip_check(e, WHO, what);
}

} // namespace

class hw_accelerator_pdsch_enc_gpu : public hw_accelerator_pdsch_enc
{
public:
  explicit hw_accelerator_pdsch_enc_gpu(std::shared_ptr<srsgpu_context> owner_) :
    owner(std::move(owner_)), ctx(owner.get())
  {
    hip_check(hipSetDevice(srsgpu_context_device(ctx)), "device");
    hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream");
    hip_check(hipMalloc(&d_tb, MAX_TB_BYTES), "TB buffer");
    hip_check(hipMalloc(&d_cw, MAX_CW_BYTES), "codeword buffer");
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&h_tb), MAX_TB_BYTES), "pinned TB");
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&h_cw), MAX_CW_BYTES), "pinned codeword");
  }

  ~hw_accelerator_pdsch_enc_gpu() override
  {
    for (auto& e : cache) {
      srsgpu_pdsch_encoder_plan_destroy(e.plan);
    }
    (void)hipFree(d_tb);
    (void)hipFree(d_cw);
    (void)hipHostFree(h_tb);
    (void)hipHostFree(h_cw);
    (void)hipStreamDestroy(stream);
  }

  void reserve_queue() override { encoded = false; }
  void free_queue() override {}

  void configure_operation(const hw_pdsch_encoder_configuration& config, unsigned /*cb_index*/) override
  {
    cfg = config;
  }

  bool is_cb_mode_supported() const override { return false; }

  unsigned get_max_supported_buff_size() const override { return MAX_CW_BYTES; }

  bool enqueue_operation(span<const uint8_t> data, span<const uint8_t> /*aux_data*/, unsigned /*cb_index*/) override
  {
    // Configuration errors are not back-pressure: pdsch_encoder_hw_impl retries a false enqueue forever, and an
    // exception would unwind through a processor task that is not exception-safe (std::terminate). The TB is accepted
    // and its codeword comes out zero (one bad grant, not a dead gNB); the error is logged once per accelerator.
    error.clear();
    if (cfg.cb_mode) {
      error = "codeblock mode is not supported (is_cb_mode_supported())";
    } else if (data.size() > MAX_TB_BYTES || data.size() * 8 != cfg.nof_tb_bits) {
      error = "TB of " + std::to_string(data.size()) + " bytes does not match the configured " +
              std::to_string(cfg.nof_tb_bits) + " bits";
    } else {
      std::memcpy(h_tb, data.data(), data.size());
      tb_bytes = static_cast<unsigned>(data.size());
    }
    encoded = false;
    return true;
  }

  /// data: the codeword, one bit per byte (do_unpack) or packed; aux_data: the packed codeword.
  bool dequeue_operation(span<uint8_t> data, span<uint8_t> aux_data, unsigned /*cb_index*/) override
  {
    gpu::device_scope dev(ctx, WHO);
    const unsigned qm     = static_cast<unsigned>(cfg.modulation);
    const unsigned nshort = cfg.nof_short_segments;
    const unsigned G      = cfg.cw_length_a * nshort + cfg.cw_length_b * (cfg.nof_segments - nshort);
    const size_t   nbytes = (G + 7) / 8;
    if (!encoded) {
      if (error.empty() && nbytes > MAX_CW_BYTES) {
        error = "codeword beyond get_max_supported_buff_size()";
      }
      srsgpu_pdsch_encoder_plan* plan = nullptr;
      if (error.empty()) {
        srsgpu_pdsch_tb_config c = {};
        c.base_graph       = (cfg.base_graph_index == ldpc_base_graph_type::BG1) ? 1 : 2;
        c.rv               = static_cast<uint8_t>(cfg.rv);
        c.modulation_order = static_cast<uint8_t>(qm);
        c.nof_layers       = static_cast<uint8_t>(
            cfg.cw_length_b > cfg.cw_length_a && qm != 0 ? (cfg.cw_length_b - cfg.cw_length_a) / qm : 1);
        c.tbs_bytes      = tb_bytes;
        c.nof_ch_symbols = qm != 0 ? G / qm : 0;
        c.Nref           = cfg.Nref;
        c.tb_offset      = 0;
        c.cw_offset      = 0;
        plan             = plan_for(c);
      }
      if (plan == nullptr) {
        report();
        std::memset(h_cw, 0, std::min<size_t>(nbytes, MAX_CW_BYTES));
      } else {
        hip_check(hipMemcpyAsync(d_tb, h_tb, tb_bytes, hipMemcpyHostToDevice, stream), "TB upload");
        if (srsgpu_pdsch_encoder_plan_execute(plan, d_tb, d_cw, stream) != SRSGPU_OK) {
          throw std::runtime_error(std::string(WHO) + ": " + srsgpu_last_error());
        }
        hip_check(hipMemcpyAsync(h_cw, d_cw, nbytes, hipMemcpyDeviceToHost, stream), "codeword download");
        hip_check(hipStreamSynchronize(stream), "synchronise");
      }
      encoded = true;
    }
    const size_t avail = std::min<size_t>(nbytes, MAX_CW_BYTES);
    if (!aux_data.empty()) {
      std::memcpy(aux_data.data(), h_cw, std::min(aux_data.size(), avail));
    }
    if (cfg.do_unpack) {
      const size_t n = std::min<size_t>(data.size(), 8 * avail);
      for (size_t i = 0; i != n; ++i) {
        data[i] = (h_cw[i >> 3] >> (7 - (i & 7))) & 1U;
      }
    } else {
      std::memcpy(data.data(), h_cw, std::min(data.size(), avail));
    }
    return true;
  }

private:
  struct cached_plan {
    srsgpu_pdsch_tb_config     key;
    srsgpu_pdsch_encoder_plan* plan;
  };

  srsgpu_pdsch_encoder_plan* plan_for(const srsgpu_pdsch_tb_config& key)
  {
    for (auto it = cache.begin(); it != cache.end(); ++it) {
      if (std::memcmp(&it->key, &key, sizeof(key)) == 0) {
        cache.splice(cache.begin(), cache, it);
        return cache.front().plan;
      }
    }
    srsgpu_pdsch_encoder_plan* plan = nullptr;
    if (srsgpu_pdsch_encoder_plan_create(ctx, &key, 1, &plan) != SRSGPU_OK) {
      error = srsgpu_last_error();
      return nullptr;
    }
    cache.push_front({key, plan});
    if (cache.size() > PLAN_CACHE_SIZE) {
      srsgpu_pdsch_encoder_plan_destroy(cache.back().plan);
      cache.pop_back();
    }
    return plan;
  }

  std::shared_ptr<srsgpu_context> owner;
  srsgpu_context*                ctx;
  hipStream_t                    stream = nullptr;
  uint8_t*                       d_tb   = nullptr;
  uint8_t*                       d_cw   = nullptr;
  uint8_t*                       h_tb   = nullptr;
  uint8_t*                       h_cw   = nullptr;
  unsigned                       tb_bytes = 0;
  bool                           encoded  = false;
  hw_pdsch_encoder_configuration cfg      = {};
  std::list<cached_plan>         cache;
  std::string                    error;  ///< Configuration error of the current TB (its codeword is zero).
  bool                           reported = false;

  void report()
  {
    if (!reported) {
      std::fprintf(stderr, "%s: %s (codeword zeroed; further errors not logged)\n", WHO, error.c_str());
      reported = true;
    }
  }
};

class hw_accelerator_pdsch_enc_factory_gpu : public hw_accelerator_pdsch_enc_factory
{
public:
  explicit hw_accelerator_pdsch_enc_factory_gpu(int device) : ctx(gpu::shared_context(device)) {}

  std::unique_ptr<hw_accelerator_pdsch_enc> create() override
  {
    return std::make_unique<hw_accelerator_pdsch_enc_gpu>(ctx);
  }

private:
  std::shared_ptr<srsgpu_context> ctx;
};

std::shared_ptr<hw_accelerator_pdsch_enc_factory> create_hw_accelerator_pdsch_enc_factory_gpu(int device)
{
  return std::make_shared<hw_accelerator_pdsch_enc_factory_gpu>(device);
}

} // namespace hal
} // namespace srsran
