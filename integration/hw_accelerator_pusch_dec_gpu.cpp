// Reference-side binding (the file a srsRAN maintainer adds next to the HAL, e.g. lib/hal/phy/upper/channel_processors/
// pusch/hw_accelerator_pusch_dec_gpu.cpp): srsran::hal::hw_accelerator_pusch_dec
// (include/srsran/hal/phy/upper/channel_processors/pusch/hw_accelerator_pusch_dec.h:83-115) over the srsgpu C ABI, so
// that the reference's own pusch_decoder_hw_impl (lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.cpp:94-
// 149, created by create_pusch_decoder_factory_hw) decodes on an MI355X unchanged.
//
// Batching: pusch_decoder_hw_impl configures and enqueues every codeblock of a transport block before the first
// dequeue (is_harq_external() is true, :226-:245), so the first dequeue launches the whole TB as one
// srsgpu_pusch_cb_plan (rate dematching into the HBM-resident HARQ soft buffers + LDPC decoding + CB CRC): one H2D copy
// of the staged LLRs from pinned memory, one execute, one D2H copy of messages / flags / iterations, one stream
// synchronisation per TB. Plans are cached per codeblock-configuration list (a cell's grants repeat), so steady state
// allocates nothing.
//
// HARQ: one HBM arena per factory, one 66 x 384-LLR slot per absolute codeblock identifier, shared by every
// accelerator the factory creates. The reference makes one accelerator per decoder thread and hands them out through a
// concurrent_thread_local_object_pool (factories.cpp:132-139, pusch_decoder_hw_impl.h:57, .cpp:151), so the first
// transmission and a retransmission of a codeblock can run on different accelerators: both address the same slot.
// The rx buffer pool keeps one codeblock on one thread at a time (unique_rx_buffer lock) and run() synchronises its
// stream before the results are read, so consecutive transmissions of a slot are ordered. free_harq_context_entry()
// (called once the TB CRC passes, :411/:423) releases the slot: a later retransmission into a released slot combines
// with zeros, the state of a new soft buffer, as the reference's ext_harq_buffer_context_repository::get() resets a
// freed entry (ext_harq_buffer_context_repository.h:70-96; its debug mode, which keeps freed entries for HARQ unit
// tests, is the factory's debug_mode). The arena and the srsgpu context live as long as any accelerator.
#include "gpu_context.h"
#include "hw_accelerator_pusch_dec_gpu.h"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <list>
#include <map>
#include <stdexcept>
#include <vector>

namespace srsran {
namespace hal {

namespace {

constexpr unsigned MAX_CB_LLRS     = 66 * 384;  // N of BG1 at Z = 384: one HARQ slot
constexpr unsigned MAX_E           = 66 * 384 * 8;
constexpr unsigned PLAN_CACHE_SIZE = 64;

constexpr const char* WHO = "hw_accelerator_pusch_dec_gpu";

void hip_check(hipError_t e, const char* what)
{
  gpu::hip_check(e, WHO, what);
}

uint8_t crc_poly_of(hw_dec_cb_crc_type t)
{
  switch (t) {
    case hw_dec_cb_crc_type::CRC16:
      return SRSGPU_CRC16;
    case hw_dec_cb_crc_type::CRC24A:
      return SRSGPU_CRC24A;
    default:
      return SRSGPU_CRC24B;
  }
}

/// Bits per symbol of a modulation scheme (modulation_scheme values are the bits per symbol).
uint8_t qm_of(modulation_scheme m)
{
  return static_cast<uint8_t>(m);
}

/// The HBM HARQ arena of a factory: one slot per absolute codeblock identifier, shared by its accelerators.
struct harq_arena {
  harq_arena(std::shared_ptr<srsgpu_context> ctx_, unsigned max_cb_ids_, bool debug_mode_) :
    ctx(std::move(ctx_)), max_cb_ids(max_cb_ids_), debug_mode(debug_mode_), in_use(max_cb_ids_, 0)
  {
    if (max_cb_ids == 0) {
      throw std::invalid_argument(std::string(WHO) + ": max_cb_ids must be positive");
    }
    hip_check(hipSetDevice(srsgpu_context_device(ctx.get())), "device");
    hip_check(hipMalloc(&d_soft, static_cast<size_t>(max_cb_ids) * MAX_CB_LLRS), "HARQ arena");
    hip_check(hipMemset(d_soft, 0, static_cast<size_t>(max_cb_ids) * MAX_CB_LLRS), "HARQ arena");
  }
  ~harq_arena() { (void)hipFree(d_soft); }

  /// Marks the slots of a launch as holding soft bits; returns the released slots a retransmission reads (to be
  /// cleared first).
  std::vector<unsigned> acquire(const std::vector<std::pair<unsigned, bool>>& ids_new_data)
  {
    std::lock_guard<std::mutex> lock(mtx);
    std::vector<unsigned>       clear;
    for (const auto& e : ids_new_data) {
      if (!e.second && in_use[e.first] == 0) {
        clear.push_back(e.first);
      }
      in_use[e.first] = 1;
    }
    return clear;
  }

  void release(unsigned id)
  {
    std::lock_guard<std::mutex> lock(mtx);
    if (id < max_cb_ids && !debug_mode) {
      in_use[id] = 0;
    }
  }

  std::shared_ptr<srsgpu_context> ctx;
  unsigned                        max_cb_ids;
  bool                            debug_mode;
  int8_t*                         d_soft = nullptr;
  std::mutex                      mtx;
  std::vector<uint8_t>            in_use;  ///< 1: the slot holds soft bits of a live HARQ process.
};

} // namespace

class hw_accelerator_pusch_dec_gpu : public hw_accelerator_pusch_dec
{
public:
  explicit hw_accelerator_pusch_dec_gpu(std::shared_ptr<harq_arena> arena_) :
    arena(std::move(arena_)), ctx(arena->ctx.get()), max_cb_ids(arena->max_cb_ids), d_harq(arena->d_soft)
  {
    hip_check(hipSetDevice(srsgpu_context_device(ctx)), "device");
    hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream");
    grow(MAX_E, 8);
  }

  ~hw_accelerator_pusch_dec_gpu() override
  {
    for (auto& e : cache) {
      srsgpu_pusch_cb_plan_destroy(e.plan);
    }
    (void)hipFree(d_llrs);
    (void)hipFree(d_msgs);
    (void)hipFree(d_iters);
    (void)hipFree(d_flags);
    (void)hipHostFree(h_llrs);
    (void)hipHostFree(h_msgs);
    (void)hipHostFree(h_iters);
    (void)hipHostFree(h_flags);
    (void)hipStreamDestroy(stream);
  }

  void reserve_queue() override
  {
    ops.clear();
    staged  = 0;
    decoded = false;
  }

  void free_queue() override { ops.clear(); }

  void configure_operation(const hw_pusch_decoder_configuration& config, unsigned cb_index) override
  {
    if (cb_index >= cfgs.size()) {
      cfgs.resize(cb_index + 1);
    }
    cfgs[cb_index] = config;
  }

  bool enqueue_operation(span<const int8_t> data, span<const int8_t> /*aux_data*/, unsigned cb_index) override
  {
    gpu::device_scope dev(ctx, WHO);
    // Configuration errors are not back-pressure: pusch_decoder_hw_impl retries a false enqueue forever
    // (pusch_decoder_hw_impl.cpp:204-354), and an exception would unwind through a thread-pool task that is not
    // exception-safe (std::terminate). The codeblock is accepted and reported as failed instead (CRC fail, all
    // iterations, zero message), and the error is logged once per accelerator.
    std::string error;
    if (cb_index >= cfgs.size()) {
      error = "codeblock " + std::to_string(cb_index) + " enqueued unconfigured";
    } else if (cfgs[cb_index].absolute_cb_id >= max_cb_ids) {
      error = "absolute codeblock id " + std::to_string(cfgs[cb_index].absolute_cb_id) +
              " beyond the HARQ arena (max_cb_ids " + std::to_string(max_cb_ids) +
              ": size it for the rx buffer pool's codeblocks)";
    } else if (data.size() > MAX_E) {
      error = "rate-matched length " + std::to_string(data.size()) + " beyond the accelerator's limit";
    }
    if (!error.empty()) {
      report(error);
      grow(staged, static_cast<unsigned>(ops.size()) + 1);
      ops.push_back({cb_index, static_cast<uint32_t>(staged), 0, true});
      decoded = false;
      return true;
    }
    grow(staged + data.size(), static_cast<unsigned>(ops.size()) + 1);
    std::memcpy(h_llrs + staged, data.data(), data.size());
    ops.push_back({cb_index, static_cast<uint32_t>(staged), static_cast<uint32_t>(data.size()), false});
    staged += data.size();
    decoded = false;
    return true;
  }

  bool dequeue_operation(span<uint8_t> data, span<int8_t> /*aux_data*/, unsigned cb_index) override
  {
    gpu::device_scope dev(ctx, WHO);
    if (!decoded) {
      run();
    }
    const int i = op_of(cb_index);
    if (i < 0) {
      return false;
    }
    std::memcpy(data.data(), h_msgs + static_cast<size_t>(i) * SRSGPU_CB_MSG_STRIDE,
                std::min<size_t>(data.size(), SRSGPU_CB_MSG_STRIDE));
    return true;
  }

  void read_operation_outputs(hw_pusch_decoder_outputs& out, unsigned cb_index, unsigned /*absolute_cb_id*/) override
  {
    const int i             = op_of(cb_index);
    const bool ok           = (i >= 0) && !ops[i].failed;
    const int  it           = ok ? h_iters[i] : -1;
    out.CRC_pass            = ok && h_flags[i] != 0;
    out.nof_ldpc_iterations = (it > 0) ? static_cast<unsigned>(it)
                                       : (cb_index < cfgs.size() ? cfgs[cb_index].max_nof_ldpc_iterations : 0U);
  }

  void free_harq_context_entry(unsigned absolute_cb_id) override { arena->release(absolute_cb_id); }

  bool is_harq_external() const override { return true; }

private:
  struct op {
    unsigned cb_index;
    uint32_t llr_offset;
    uint32_t length;
    bool     failed;  ///< Rejected at enqueue or by the plan: reported as a CRC failure.
  };

  /// Logs a configuration error (once per accelerator: a misconfigured cell would repeat it every slot).
  void report(const std::string& error)
  {
    if (!reported) {
      std::fprintf(stderr, "%s: %s (codeblock reported as failed; further errors not logged)\n", WHO, error.c_str());
      reported = true;
    }
  }
  struct cached_plan {
    std::vector<srsgpu_pusch_cb_config> key;
    srsgpu_pusch_cb_plan*               plan;
  };

  int op_of(unsigned cb_index) const
  {
    for (size_t i = 0; i != ops.size(); ++i) {
      if (ops[i].cb_index == cb_index) {
        return static_cast<int>(i);
      }
    }
    return -1;
  }

  /// Pinned staging and device buffers for `llrs` LLRs and `cbs` codeblocks (grown, never shrunk).
  void grow(size_t llrs, unsigned cbs)
  {
    if (llrs > cap_llrs) {
      const size_t n = std::max(llrs, 2 * cap_llrs);
      int8_t*      h = nullptr;
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&h), n), "pinned LLR staging");
      if (h_llrs != nullptr) {
        std::memcpy(h, h_llrs, staged);
        (void)hipHostFree(h_llrs);
        (void)hipFree(d_llrs);
      }
      h_llrs = h;
      hip_check(hipMalloc(&d_llrs, n), "LLR buffer");
      cap_llrs = n;
    }
    if (cbs > cap_cbs) {
      const unsigned n = std::max(cbs, 2 * cap_cbs);
      (void)hipHostFree(h_msgs);
      (void)hipHostFree(h_iters);
      (void)hipHostFree(h_flags);
      (void)hipFree(d_msgs);
      (void)hipFree(d_iters);
      (void)hipFree(d_flags);
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&h_msgs), static_cast<size_t>(n) * SRSGPU_CB_MSG_STRIDE),
                "pinned messages");
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&h_iters), n * sizeof(int32_t)), "pinned iterations");
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&h_flags), n), "pinned flags");
      hip_check(hipMalloc(&d_msgs, static_cast<size_t>(n) * SRSGPU_CB_MSG_STRIDE), "messages");
      hip_check(hipMalloc(&d_iters, n * sizeof(int32_t)), "iterations");
      hip_check(hipMalloc(&d_flags, n), "flags");
      cap_cbs = n;
    }
  }

  /// The plan of the staged codeblocks, from the cache (most recently used first) or created.
  srsgpu_pusch_cb_plan* plan_for(const std::vector<srsgpu_pusch_cb_config>& key)
  {
    for (auto it = cache.begin(); it != cache.end(); ++it) {
      if (it->key.size() == key.size() &&
          std::memcmp(it->key.data(), key.data(), key.size() * sizeof(srsgpu_pusch_cb_config)) == 0) {
        cache.splice(cache.begin(), cache, it);
        return cache.front().plan;
      }
    }
    srsgpu_pusch_cb_plan* plan = nullptr;
    if (srsgpu_pusch_cb_plan_create(ctx, SRSGPU_LDPC_IMPL_SIMD, key.data(), static_cast<uint32_t>(key.size()), &plan) !=
        SRSGPU_OK) {
      report(srsgpu_last_error());
      return nullptr;
    }
    cache.push_front({key, plan});
    if (cache.size() > PLAN_CACHE_SIZE) {
      srsgpu_pusch_cb_plan_destroy(cache.back().plan);
      cache.pop_back();
    }
    return plan;
  }

  /// Decodes every enqueued codeblock of the TB on the device (the failed ones are skipped; their message is zero).
  void run()
  {
    const size_t n = ops.size();
    std::memset(h_msgs, 0, n * SRSGPU_CB_MSG_STRIDE);
    std::memset(h_flags, 0, n);
    std::vector<srsgpu_pusch_cb_config>    key;
    std::vector<std::pair<unsigned, bool>> ids;
    std::vector<size_t>                    key_op;  // the op of each plan position (rejected ops are not planned)
    for (size_t i = 0; i != n; ++i) {
      h_iters[i] = -1;
      if (ops[i].failed) {
        continue;
      }
      key_op.push_back(i);
      const hw_pusch_decoder_configuration& c = cfgs[ops[i].cb_index];
      srsgpu_pusch_cb_config                k;
      std::memset(&k, 0, sizeof(k));
      k.base_graph       = (c.base_graph_index == ldpc_base_graph_type::BG1) ? 1 : 2;
      k.rv               = static_cast<uint8_t>(c.rv);
      k.modulation_order = qm_of(c.modulation);
      k.crc_poly         = crc_poly_of(c.cb_crc_type);
      k.lifting_size     = static_cast<uint16_t>(c.lifting_size);
      k.nof_filler_bits  = static_cast<uint16_t>(c.nof_filler_bits);
      k.nof_crc_bits     = static_cast<uint8_t>(c.cb_crc_len);
      k.max_iterations   = static_cast<uint8_t>(c.max_nof_ldpc_iterations);
      k.new_data         = c.new_data ? 1 : 0;
      k.use_early_stop   = c.use_early_stop ? 1 : 0;
      k.scaling_factor   = 0.8F;  // ldpc_decoder::configuration::algorithm_details default (ldpc_decoder.h:50)
      k.Nref             = c.Nref;
      k.rm_length        = ops[i].length;
      k.llr_offset       = ops[i].llr_offset;
      k.harq_offset      = c.absolute_cb_id * MAX_CB_LLRS;
      k.out_offset       = static_cast<uint32_t>(i * SRSGPU_CB_MSG_STRIDE);
      key.push_back(k);
      ids.emplace_back(c.absolute_cb_id, c.new_data);
    }
    decoded = true;
    if (key.empty()) {
      return;
    }
    srsgpu_pusch_cb_plan* plan = plan_for(key);
    if (plan == nullptr) {  // rejected by the plan's validation (reported): every codeblock of the TB fails
      for (op& o : ops) {
        o.failed = true;
      }
      return;
    }
    // A retransmission into a released slot combines with zeros (a new soft buffer).
    for (unsigned id : arena->acquire(ids)) {
      hip_check(hipMemsetAsync(d_harq + static_cast<size_t>(id) * MAX_CB_LLRS, 0, MAX_CB_LLRS, stream), "HARQ reset");
    }
    hip_check(hipMemcpyAsync(d_llrs, h_llrs, staged, hipMemcpyHostToDevice, stream), "LLR upload");
    hip_check(hipMemsetAsync(d_flags, 0, n, stream), "flags");
    hip_check(hipMemsetAsync(d_msgs, 0, n * SRSGPU_CB_MSG_STRIDE, stream), "messages");
    if (srsgpu_pusch_cb_plan_execute(plan, d_llrs, d_harq, d_msgs, d_iters, d_flags, stream) != SRSGPU_OK) {
      throw std::runtime_error(std::string(WHO) + ": " + srsgpu_last_error());
    }
    hip_check(hipMemcpyAsync(h_msgs, d_msgs, n * SRSGPU_CB_MSG_STRIDE, hipMemcpyDeviceToHost, stream), "messages");
    hip_check(hipMemcpyAsync(h_iters, d_iters, n * sizeof(int32_t), hipMemcpyDeviceToHost, stream), "iterations");
    hip_check(hipMemcpyAsync(h_flags, d_flags, n, hipMemcpyDeviceToHost, stream), "flags");
    hip_check(hipStreamSynchronize(stream), "synchronise");
    // The plan reports the CRC flag and iterations of its k-th codeblock at position k (srsgpu_pusch_cb_plan_create
    // numbers the codeblocks by their position in the configuration array); read_operation_outputs reads them by op.
    // With ops rejected at enqueue the two differ: scatter the results back to their ops (messages already land at
    // out_offset = op * stride).
    if (key_op.size() != n) {
      const std::vector<uint8_t> flags(h_flags, h_flags + key_op.size());
      const std::vector<int32_t> iters(h_iters, h_iters + key_op.size());
      for (size_t i = 0; i != n; ++i) {
        h_flags[i] = 0;
        h_iters[i] = -1;
      }
      for (size_t k = 0; k != key_op.size(); ++k) {
        h_flags[key_op[k]] = flags[k];
        h_iters[key_op[k]] = iters[k];
      }
    }
  }

  std::shared_ptr<harq_arena>                 arena;
  srsgpu_context*                             ctx;
  unsigned                                    max_cb_ids;
  int8_t*                                     d_harq;
  hipStream_t                                 stream  = nullptr;
  int8_t*                                     d_llrs  = nullptr;
  uint8_t*                                    d_msgs  = nullptr;
  int32_t*                                    d_iters = nullptr;
  uint8_t*                                    d_flags = nullptr;
  int8_t*                                     h_llrs  = nullptr;
  uint8_t*                                    h_msgs  = nullptr;
  int32_t*                                    h_iters = nullptr;
  uint8_t*                                    h_flags = nullptr;
  size_t                                      cap_llrs = 0;
  unsigned                                    cap_cbs  = 0;
  size_t                                      staged   = 0;
  bool                                        decoded  = false;
  bool                                        reported = false;
  std::vector<hw_pusch_decoder_configuration> cfgs;
  std::vector<op>                             ops;
  std::list<cached_plan>                      cache;
};

/// Factory (hw_accelerator_pusch_dec_factory.h): one accelerator per decoder-pool entry (one per worker thread), all
/// sharing the factory's HARQ arena and the device's srsgpu context (shared ownership: the accelerators outlive the
/// factory). The absolute codeblock identifiers of the rx buffer pool index the HARQ arena: max_cb_ids must cover the
/// pool's codeblocks (an identifier beyond it throws).
class hw_accelerator_pusch_dec_factory_gpu : public hw_accelerator_pusch_dec_factory
{
public:
  hw_accelerator_pusch_dec_factory_gpu(int device, unsigned max_cb_ids, bool debug_mode) :
    arena(std::make_shared<harq_arena>(gpu::shared_context(device), max_cb_ids, debug_mode))
  {
  }

  std::unique_ptr<hw_accelerator_pusch_dec> create() override
  {
    return std::make_unique<hw_accelerator_pusch_dec_gpu>(arena);
  }

private:
  std::shared_ptr<harq_arena> arena;
};

std::shared_ptr<hw_accelerator_pusch_dec_factory>
create_hw_accelerator_pusch_dec_factory_gpu(int device, unsigned max_cb_ids, bool debug_mode)
{
  return std::make_shared<hw_accelerator_pusch_dec_factory_gpu>(device, max_cb_ids, debug_mode);
}

} // namespace hal
} // namespace srsran
