// TEST INFRASTRUCTURE ONLY: C entry points that run the reference's own transport-block processors with the GPU
// bindings of integration/ plugged in through the reference's interfaces, and the reference's CPU implementations
// beside them, on the same inputs (built by oracle/build_hal.sh into oracle/_ref/libsrshal.so; tests/test_hal_gpu.py):
//
//   PUSCH decoder, mode 0: pusch_decoder_impl (pusch_decoder_impl.cpp) with the reference's pusch_codeblock_decoder
//                          (AVX2 rate dematcher + AVX-512 / AVX2 LDPC decoder) - the CPU path;
//                  mode 1: the same pusch_decoder_impl, its ldpc_decoder replaced by integration/ldpc_decoder_gpu.cpp;
//                  mode 2: pusch_decoder_hw_impl (pusch_decoder_hw_impl.cpp) over the GPU hal::hw_accelerator_pusch_dec
//                          of integration/hw_accelerator_pusch_dec_gpu.cpp (HARQ soft buffers in HBM);
//   PDSCH encoder, mode 0: pdsch_encoder_impl (AVX2 LDPC encoder); mode 1: pdsch_encoder_hw_impl over the GPU
//                          hal::hw_accelerator_pdsch_enc (integration/hw_accelerator_pdsch_enc_gpu.cpp).
//
// The rx buffers are a minimal unique_rx_buffer::callback (soft bits, data bits, CRC flags per codeblock, absolute
// codeblock identifiers harq_id * 160 + cb), one per (mode, HARQ process), so retransmissions combine like the pool's.
//
// Pool harness (hal_pool_*): the reference's own wiring of the HW decoder (pusch_decoder_factory_hw, factories.cpp:
// 122-140): a temporary accelerator factory creates one accelerator per decoder thread and is dropped before anything
// is decoded; the accelerators form a pusch_decoder_hw_impl::hw_decoder_pool (concurrent_thread_local_object_pool:
// each thread gets its own accelerator); persistent worker threads each own a pusch_decoder_hw_impl over that pool, so
// a transmission and its retransmission can be decoded by different threads, i.e. different accelerators.
#include "hw_accelerator_pusch_dec_gpu.h"

#include "srsran/phy/upper/channel_coding/channel_coding_factories.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_notifier.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_result.h"
#include "srsran/phy/upper/unique_rx_buffer.h"

#include "lib/phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_decoder_avx2.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_decoder_avx512.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_encoder_avx2.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_avx2_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_rx_impl.h"
#include "lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_encoder_hw_impl.h"
#include "lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_codeblock_decoder.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.h"
#include "lib/phy/upper/channel_processors/pusch/pusch_decoder_impl.h"

#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace srsran {
std::shared_ptr<ldpc_decoder_factory> create_ldpc_decoder_factory_gpu(int device);
}

using namespace srsran;

namespace {

constexpr unsigned CB_IDS_PER_HARQ = 160;  // >= MAX_NOF_SEGMENTS

class test_rx_buffer : public unique_rx_buffer::callback
{
public:
  test_rx_buffer(unsigned nof_cbs, unsigned first_abs_id) :
    crcs(nof_cbs, false), soft(nof_cbs, std::vector<log_likelihood_ratio>(66 * 384)),
    data(nof_cbs, std::vector<uint8_t>(22 * 384 / 8)), abs0(first_abs_id)
  {
  }
  unsigned   get_nof_codeblocks() const override { return static_cast<unsigned>(crcs.size()); }
  void       reset_codeblocks_crc() override { std::fill(crcs.begin(), crcs.end(), false); }
  span<bool> get_codeblocks_crc() override { return span<bool>(reinterpret_cast<bool*>(crcs.data()), crcs.size()); }
  unsigned   get_absolute_codeblock_id(unsigned cb) const override { return abs0 + cb; }
  span<log_likelihood_ratio> get_codeblock_soft_bits(unsigned cb, unsigned size) override
  {
    return span<log_likelihood_ratio>(soft[cb]).first(size);
  }
  bit_buffer get_codeblock_data_bits(unsigned cb, unsigned size) override
  {
    return bit_buffer::from_bytes(data[cb]).first(size);
  }
  bool       try_lock() override { return true; }
  void       unlock() override {}
  void       release() override { reset_codeblocks_crc(); }

private:
  std::vector<char>                              crcs;  // storage for span<bool>
  std::vector<std::vector<log_likelihood_ratio>> soft;
  std::vector<std::vector<uint8_t>>              data;
  unsigned                                       abs0;
};

class result_capture : public pusch_decoder_notifier
{
public:
  void on_sch_data(const pusch_decoder_result& r) override
  {
    result = r;
    done   = true;
  }
  pusch_decoder_result result;
  bool                 done = false;
};

template <typename S>
S make_sch_crc()
{
  S s;
  s.crc16  = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC16);
  s.crc24A = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24A);
  s.crc24B = std::make_unique<crc_calculator_generic_impl>(crc_generator_poly::CRC24B);
  return s;
}

std::unique_ptr<ldpc_decoder> cpu_decoder()
{
  if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) {
    return std::make_unique<ldpc_decoder_avx512>();
  }
  return std::make_unique<ldpc_decoder_avx2>();
}

struct hal_harness {
  std::shared_ptr<ldpc_decoder_factory>                   gpu_ldpc;
  std::shared_ptr<hal::hw_accelerator_pusch_dec_factory>  gpu_dec;
  std::shared_ptr<hal::hw_accelerator_pdsch_enc_factory>  gpu_enc;
  std::unique_ptr<pusch_decoder>                          dec[3];
  std::unique_ptr<pdsch_encoder>                          enc[2];
  std::map<std::pair<int, unsigned>, std::unique_ptr<test_rx_buffer>> rx;
};

std::unique_ptr<pusch_decoder> make_sw_decoder(std::unique_ptr<ldpc_decoder> ldpc)
{
  auto cb_crc = make_sch_crc<pusch_codeblock_decoder::sch_crc>();
  std::vector<std::unique_ptr<pusch_codeblock_decoder>> cbs;
  cbs.push_back(std::make_unique<pusch_codeblock_decoder>(std::make_unique<ldpc_rate_dematcher_avx2_impl>(),
                                                          std::move(ldpc), cb_crc));
  auto pool = std::make_shared<pusch_decoder_impl::codeblock_decoder_pool>(std::move(cbs));
  return std::make_unique<pusch_decoder_impl>(std::make_unique<ldpc_segmenter_rx_impl>(), pool,
                                              make_sch_crc<pusch_decoder_impl::sch_crc>(), nullptr, 275, 4);
}

/// A persistent thread running posted jobs one at a time (run() blocks until the job is done).
class worker_thread
{
public:
  worker_thread() : th([this] { loop(); }) {}
  ~worker_thread()
  {
    {
      std::lock_guard<std::mutex> lock(mtx);
      quit = true;
    }
    cv.notify_all();
    th.join();
  }
  void run(std::function<void()> f)
  {
    std::unique_lock<std::mutex> lock(mtx);
    job  = std::move(f);
    done = false;
    cv.notify_all();
    cv.wait(lock, [this] { return done; });
  }

private:
  void loop()
  {
    std::unique_lock<std::mutex> lock(mtx);
    for (;;) {
      cv.wait(lock, [this] { return quit || job; });
      if (quit) {
        return;
      }
      std::function<void()> f = std::move(job);
      job                      = nullptr;
      lock.unlock();
      f();
      lock.lock();
      done = true;
      cv.notify_all();
    }
  }
  std::mutex              mtx;
  std::condition_variable cv;
  std::function<void()>   job;
  bool                    done = true;
  bool                    quit = false;
  std::thread             th;
};

struct pool_harness {
  std::unique_ptr<pusch_decoder>                                       cpu;
  std::vector<std::unique_ptr<pusch_decoder>>                          decs;  // one per worker
  std::vector<std::unique_ptr<worker_thread>>                          workers;
  std::map<std::pair<int, unsigned>, std::unique_ptr<test_rx_buffer>> rx;    // (cpu 0 / gpu 1, HARQ process)
};

/// new_data + on_new_softbits + on_end_softbits of one TB on `dec`; stats as hal_pusch_decode.
int run_decode(pusch_decoder&        dec,
               test_rx_buffer&       rxb,
               const pusch_decoder::configuration& cfg,
               const int8_t*         llrs,
               unsigned              nof_llrs,
               uint8_t*              tb,
               unsigned              tb_bytes,
               double*               stats)
{
  result_capture        notifier;
  pusch_decoder_buffer& buf = dec.new_data(span<uint8_t>(tb, tb_bytes), unique_rx_buffer(rxb), notifier, cfg);
  buf.on_new_softbits(span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs), nof_llrs));
  buf.on_end_softbits();
  if (!notifier.done) {
    return -1;
  }
  const auto& r = notifier.result;
  stats[0]      = r.tb_crc_ok ? 1 : 0;
  stats[1]      = r.nof_codeblocks_total;
  stats[2]      = r.ldpc_decoder_stats.get_nof_observations();
  stats[3]      = r.ldpc_decoder_stats.get_nof_observations() ? r.ldpc_decoder_stats.get_min() : -1;
  stats[4]      = r.ldpc_decoder_stats.get_nof_observations() ? r.ldpc_decoder_stats.get_max() : -1;
  stats[5]      = r.ldpc_decoder_stats.get_nof_observations() ? r.ldpc_decoder_stats.get_mean() : -1;
  return 0;
}

} // namespace

extern "C" {

/// Pool harness: nof_threads worker threads, each with its own pusch_decoder_hw_impl over one shared
/// hw_decoder_pool of nof_threads GPU accelerators (made by a factory that is destroyed before this returns), plus the
/// reference CPU decoder (pusch_decoder_impl, AVX-512 / AVX2 LDPC) on the calling thread.
void* hal_pool_create(int device, unsigned max_cb_ids, unsigned nof_threads)
{
  auto*                                                   h = new pool_harness();
  std::vector<std::unique_ptr<hal::hw_accelerator_pusch_dec>> accs;
  {
    std::shared_ptr<hal::hw_accelerator_pusch_dec_factory> factory =
        hal::create_hw_accelerator_pusch_dec_factory_gpu(device, max_cb_ids);
    for (unsigned i = 0; i != nof_threads; ++i) {
      accs.push_back(factory->create());
    }
  }  // the factory is gone: the accelerators keep the context and the HARQ arena alive
  auto pool = std::make_shared<pusch_decoder_hw_impl::hw_decoder_pool>(std::move(accs));
  for (unsigned i = 0; i != nof_threads; ++i) {
    auto crcs = make_sch_crc<pusch_decoder_hw_impl::sch_crc>();
    h->decs.push_back(
        std::make_unique<pusch_decoder_hw_impl>(std::make_unique<ldpc_segmenter_rx_impl>(), crcs, pool, nullptr));
    h->workers.push_back(std::make_unique<worker_thread>());
  }
  h->cpu = make_sw_decoder(cpu_decoder());
  return h;
}

void hal_pool_destroy(void* p)
{
  delete static_cast<pool_harness*>(p);
}

/// One TB decoded by worker thread `worker` (GPU, through the thread's pool accelerator) or, for worker < 0, by the
/// reference CPU decoder. Arguments and stats as hal_pusch_decode.
int hal_pool_decode(void*         p,
                    int           worker,
                    unsigned      harq_id,
                    unsigned      nof_cbs,
                    int           bg,
                    int           rv,
                    int           qm,
                    int           nof_layers,
                    unsigned      Nref,
                    int           max_iter,
                    int           early_stop,
                    int           new_data,
                    const int8_t* llrs,
                    unsigned      nof_llrs,
                    uint8_t*      tb,
                    unsigned      tb_bytes,
                    double*       stats)
{
  auto*    h   = static_cast<pool_harness*>(p);
  auto     key = std::make_pair(worker < 0 ? 0 : 1, harq_id);
  auto     it  = h->rx.find(key);
  if (it == h->rx.end() || it->second->get_nof_codeblocks() != nof_cbs) {
    h->rx[key] = std::make_unique<test_rx_buffer>(nof_cbs, harq_id * CB_IDS_PER_HARQ);
  }
  pusch_decoder::configuration cfg;
  cfg.base_graph          = bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  cfg.rv                  = rv;
  cfg.mod                 = static_cast<modulation_scheme>(qm);
  cfg.Nref                = Nref;
  cfg.nof_layers          = nof_layers;
  cfg.nof_ldpc_iterations = max_iter;
  cfg.use_early_stop      = early_stop != 0;
  cfg.new_data            = new_data != 0;
  test_rx_buffer& rxb     = *h->rx[key];
  if (worker < 0) {
    return run_decode(*h->cpu, rxb, cfg, llrs, nof_llrs, tb, tb_bytes, stats);
  }
  if (static_cast<size_t>(worker) >= h->workers.size()) {
    return -2;
  }
  int r = -1;
  h->workers[worker]->run([&] { r = run_decode(*h->decs[worker], rxb, cfg, llrs, nof_llrs, tb, tb_bytes, stats); });
  return r;
}

void* hal_create(int device, unsigned max_cb_ids)
{
  auto* h     = new hal_harness();
  h->gpu_ldpc = create_ldpc_decoder_factory_gpu(device);
  // Debug mode (entries kept after a passing TB CRC): the tests retransmit after success and compare with the CPU
  // decoder, whose test rx buffer keeps its soft bits.
  h->gpu_dec  = hal::create_hw_accelerator_pusch_dec_factory_gpu(device, max_cb_ids, true);
  h->gpu_enc  = hal::create_hw_accelerator_pdsch_enc_factory_gpu(device);
  h->dec[0]   = make_sw_decoder(cpu_decoder());
  h->dec[1]   = make_sw_decoder(h->gpu_ldpc->create());
  {
    std::vector<std::unique_ptr<hal::hw_accelerator_pusch_dec>> accs;
    accs.push_back(h->gpu_dec->create());
    auto pool  = std::make_shared<pusch_decoder_hw_impl::hw_decoder_pool>(std::move(accs));
    auto crcs  = make_sch_crc<pusch_decoder_hw_impl::sch_crc>();
    h->dec[2]  = std::make_unique<pusch_decoder_hw_impl>(std::make_unique<ldpc_segmenter_rx_impl>(), crcs, pool, nullptr);
  }
  {
    auto seg_crc = make_sch_crc<ldpc_segmenter_tx_impl::sch_crc>();
    h->enc[0]    = std::make_unique<pdsch_encoder_impl>(std::make_unique<ldpc_segmenter_tx_impl>(seg_crc),
                                                     std::make_unique<ldpc_encoder_avx2>(),
                                                     std::make_unique<ldpc_rate_matcher_impl>());
    auto seg_crc2 = make_sch_crc<ldpc_segmenter_tx_impl::sch_crc>();
    auto crcs     = make_sch_crc<pdsch_encoder_hw_impl::sch_crc>();
    h->enc[1]     = std::make_unique<pdsch_encoder_hw_impl>(crcs, std::make_unique<ldpc_segmenter_tx_impl>(seg_crc2),
                                                        h->gpu_enc->create());
  }
  return h;
}

void hal_destroy(void* p)
{
  delete static_cast<hal_harness*>(p);
}

/// pusch_decoder::new_data + on_new_softbits + on_end_softbits of one transport block (synchronous: no executor).
/// stats[] = {tb_crc_ok, nof_codeblocks_total, ldpc observations, min, max, mean iterations}. Returns 0, or -1 when
/// the decoder did not notify.
int hal_pusch_decode(void*          p,
                     int            mode,
                     unsigned       harq_id,
                     unsigned       nof_cbs,
                     int            bg,
                     int            rv,
                     int            qm,
                     int            nof_layers,
                     unsigned       Nref,
                     int            max_iter,
                     int            early_stop,
                     int            new_data,
                     const int8_t*  llrs,
                     unsigned       nof_llrs,
                     uint8_t*       tb,
                     unsigned       tb_bytes,
                     double*        stats)
{
  auto* h   = static_cast<hal_harness*>(p);
  auto  key = std::make_pair(mode, harq_id);
  auto  it  = h->rx.find(key);
  if (it == h->rx.end() || it->second->get_nof_codeblocks() != nof_cbs) {
    h->rx[key] = std::make_unique<test_rx_buffer>(nof_cbs, harq_id * CB_IDS_PER_HARQ);
  }
  pusch_decoder::configuration cfg;
  cfg.base_graph          = bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  cfg.rv                  = rv;
  cfg.mod                 = static_cast<modulation_scheme>(qm);
  cfg.Nref                = Nref;
  cfg.nof_layers          = nof_layers;
  cfg.nof_ldpc_iterations = max_iter;
  cfg.use_early_stop      = early_stop != 0;
  cfg.new_data            = new_data != 0;
  result_capture        notifier;
  pusch_decoder_buffer& buf = h->dec[mode]->new_data(span<uint8_t>(tb, tb_bytes), unique_rx_buffer(*h->rx[key]),
                                                     notifier, cfg);
  buf.on_new_softbits(span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs), nof_llrs));
  buf.on_end_softbits();
  if (!notifier.done) {
    return -1;
  }
  const auto& r = notifier.result;
  stats[0]      = r.tb_crc_ok ? 1 : 0;
  stats[1]      = r.nof_codeblocks_total;
  stats[2]      = r.ldpc_decoder_stats.get_nof_observations();
  stats[3]      = r.ldpc_decoder_stats.get_nof_observations() ? r.ldpc_decoder_stats.get_min() : -1;
  stats[4]      = r.ldpc_decoder_stats.get_nof_observations() ? r.ldpc_decoder_stats.get_max() : -1;
  stats[5]      = r.ldpc_decoder_stats.get_nof_observations() ? r.ldpc_decoder_stats.get_mean() : -1;
  return 0;
}

/// pdsch_encoder::encode of one transport block into cw (G = nof_ch_symbols x Qm bits, one per byte).
int hal_pdsch_encode(void*          p,
                     int            mode,
                     int            bg,
                     int            rv,
                     int            qm,
                     int            nof_layers,
                     unsigned       nof_ch_symbols,
                     unsigned       Nref,
                     const uint8_t* tb,
                     unsigned       tb_bytes,
                     uint8_t*       cw)
{
  auto*                        h = static_cast<hal_harness*>(p);
  pdsch_encoder::configuration cfg;
  cfg.base_graph     = bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  cfg.rv             = rv;
  cfg.mod            = static_cast<modulation_scheme>(qm);
  cfg.Nref           = Nref;
  cfg.nof_layers     = nof_layers;
  cfg.nof_ch_symbols = nof_ch_symbols;
  h->enc[mode]->encode(span<uint8_t>(cw, nof_ch_symbols * qm), span<const uint8_t>(tb, tb_bytes), cfg);
  return 0;
}

/// One TB's codeblocks through one GPU accelerator directly (hw_accelerator_pusch_dec: configure, enqueue, dequeue,
/// read_operation_outputs), BG1 / CRC24B / rv 0 / new data: codeblock c has E = rm_lengths[c] LLRs at llrs + offsets;
/// codeblocks with reject[c] != 0 are enqueued with an oversized span, which the accelerator rejects (reports as a
/// failed codeblock). Outputs per codeblock: crc_pass[c], iters[c], msg bytes at msgs + c * msg_stride.
int hal_accel_decode_ops(int            device,
                         unsigned       nof_cbs,
                         unsigned       lifting_size,
                         unsigned       nof_filler_bits,
                         unsigned       qm,
                         const unsigned* rm_lengths,
                         const int8_t*  llrs,
                         const uint8_t* reject,
                         int*           crc_pass,
                         int*           iters,
                         uint8_t*       msgs,
                         unsigned       msg_stride)
{
  try {
    auto factory = hal::create_hw_accelerator_pusch_dec_factory_gpu(device, 64);
    auto acc     = factory->create();
    std::vector<int8_t> oversized(66 * 384 * 8 + 1, 0);
    size_t              off = 0;
    acc->reserve_queue();
    for (unsigned c = 0; c != nof_cbs; ++c) {
      hal::hw_pusch_decoder_configuration cfg = {};
      cfg.base_graph_index        = ldpc_base_graph_type::BG1;
      cfg.modulation              = qm == 2 ? modulation_scheme::QPSK
                                    : qm == 4 ? modulation_scheme::QAM16
                                    : qm == 6 ? modulation_scheme::QAM64
                                              : modulation_scheme::QAM256;
      cfg.nof_segments            = nof_cbs;
      cfg.rv                      = 0;
      cfg.cw_length               = rm_lengths[c];
      cfg.lifting_size            = lifting_size;
      cfg.Ncb                     = 66 * lifting_size;
      cfg.Nref                    = 0;
      cfg.nof_segment_bits        = 22 * lifting_size;
      cfg.nof_filler_bits         = nof_filler_bits;
      cfg.max_nof_ldpc_iterations = 6;
      cfg.use_early_stop          = true;
      cfg.new_data                = true;
      cfg.cb_crc_len              = 24;
      cfg.cb_crc_type             = hal::hw_dec_cb_crc_type::CRC24B;
      cfg.absolute_cb_id          = c;
      acc->configure_operation(cfg, c);
      span<const int8_t> data = reject[c] != 0 ? span<const int8_t>(oversized) : span<const int8_t>(llrs + off, rm_lengths[c]);
      if (!acc->enqueue_operation(data, {}, c)) {
        return -2;
      }
      off += rm_lengths[c];
    }
    for (unsigned c = 0; c != nof_cbs; ++c) {
      if (!acc->dequeue_operation(span<uint8_t>(msgs + c * msg_stride, msg_stride), {}, c)) {
        return -3;
      }
      hal::hw_pusch_decoder_outputs out = {};
      acc->read_operation_outputs(out, c, c);
      crc_pass[c] = out.CRC_pass ? 1 : 0;
      iters[c]    = static_cast<int>(out.nof_ldpc_iterations);
    }
    acc->free_queue();
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "hal_accel_decode_ops: %s\n", e.what());
    return -1;
  }
}

} // extern "C"
