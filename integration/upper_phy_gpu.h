// Slot-batched GPU processing behind the reference's upper-PHY slot processors (the declarations a srsRAN maintainer
// adds next to lib/phy/upper/upper_phy_factories.cpp).
//
// The reference's processors hand their channel processors one PDU at a time: uplink_processor_impl::process_pusch
// (uplink_processor_impl.cpp:191-247) runs pusch_processor::process per PDU on the PUSCH executor, and
// downlink_processor_single_executor_impl::process_pdsch (downlink_processor_single_executor_impl.cpp:96-135) runs
// pdsch_processor::process per PDU on its executor; the slot boundary is visible only to the processor
// (handle_rx_symbol after the last symbol of a PDU, finish_processing_pdus). On a GPU one PDU is far too small a
// launch and each would pay its own PCIe round trip, so the reference's processors stay in charge of their state
// machines, PDU repositories and notifications, and only the PUSCH / PDSCH work is gathered into one launch sequence
// per slot:
//
//  * UL: the reference's uplink_processor_impl is built with a pusch_processor that registers each PDU in a slot batch
//    (create_pusch_processor_batch_gpu) and an executor that runs the PUSCH task on the caller (pusch_inline_executor),
//    and is wrapped by create_uplink_processor_batch_gpu, whose handle_rx_symbol runs the reference's and then hands the
//    PDUs it registered to the PUSCH executor as one job: one upload of the grid, channel estimation, demodulation and
//    decoding of every PDU (HARQ soft bits kept in HBM across slots, one arena slot per absolute codeblock identifier of
//    the reference's rx buffer pool), one download. The results then go through the reference's own
//    pusch_processor_impl per PDU, fed the GPU results (channel-estimate metrics, LLRs + scrambling sequence +
//    post-equalisation statistics, decoded TB), so the CSI report, the UCI demultiplexing / decoding, the notifier
//    order and the rx buffer bookkeeping are the reference's. PDUs the batch does not cover (CSI Part 2, non-identity
//    rx port lists, more than four layers) go to a caller-supplied pusch_processor.
//
//  * DL: the reference's downlink_processor_single_executor_impl is built with a pdsch_processor that runs the
//    reference's pdsch_processor_impl over recording encoder / modulator / DM-RS stages (create_pdsch_processor_batch_gpu)
//    and with pdsch_batch_executor, which runs the PDSCH task on the caller while create_downlink_processor_batch_gpu's
//    process_pdsch is inside it; at finish_processing_pdus the wrapper runs the slot's PDSCHs as one launch sequence
//    (TB CRC + LDPC encoding + rate matching, DM-RS, scrambling + modulation + layer mapping + precoding into one grid)
//    on the real executor, writes exactly the REs they map into the slot's grid and reports each PDSCH finished, after
//    which the reference's state machine sends the grid.
#pragma once

#include "signal_chain_gpu.h"
#include "srsran/phy/upper/channel_processors/pdsch/pdsch_processor.h"
#include "srsran/phy/upper/channel_processors/pusch/factories.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor.h"
#include "srsran/phy/upper/channel_processors/uci/factories.h"
#include "srsran/phy/upper/channel_state_information.h"
#include "srsran/phy/upper/downlink_processor.h"
#include "srsran/phy/upper/signal_processors/ptrs/ptrs_pdsch_generator.h"
#include "srsran/phy/upper/uplink_processor.h"
#include "srsran/support/executors/task_executor.h"

#include <memory>

namespace srsran {
namespace gpu {

/// PUSCH slot batching parameters (the reference's pusch_processor_impl::configuration and the rx buffer pool size).
struct pusch_batch_configuration {
  int                                  device = 0;
  pusch_estimator_options              estimator;
  pusch_demodulator_options            demodulator;
  unsigned                             max_cb_ids          = 4096;  ///< rx buffer pool codeblocks (HARQ arena slots).
  unsigned                             nof_ldpc_iterations = 6;
  bool                                 ldpc_early_stop     = true;
  channel_state_information::sinr_type csi_sinr_calc_method = channel_state_information::sinr_type::post_equalization;
};

/// The HBM HARQ arena shared by every PUSCH batch of a sector (the rx buffer pool is shared too).
class pusch_harq_arena;
std::shared_ptr<pusch_harq_arena> create_pusch_harq_arena(int device, unsigned max_cb_ids);

/// A slot batch of PUSCH transmissions (one per uplink processor).
class pusch_slot_batch;

/// demux / uci: factories of the reference's UL-SCH demultiplexer and UCI decoder (host-side parts of the result
/// assembly, one per thread that runs batches); fallback: the processor for PDUs the batch does not cover.
std::shared_ptr<pusch_slot_batch> create_pusch_slot_batch(const pusch_batch_configuration&           config,
                                                          std::shared_ptr<pusch_harq_arena>          arena,
                                                          std::shared_ptr<ulsch_demultiplex_factory> demux,
                                                          std::shared_ptr<uci_decoder_factory>       uci,
                                                          std::unique_ptr<pusch_processor>           fallback);

/// The pusch_processor given to the reference's uplink_processor_impl: process() registers the PDU in the batch.
std::unique_ptr<pusch_processor> create_pusch_processor_batch_gpu(std::shared_ptr<pusch_slot_batch> batch);

/// The PUSCH executor given to the reference's uplink_processor_impl: runs each task on the calling thread.
task_executor& pusch_inline_executor();

/// Wraps the reference's uplink_processor_impl (built with the two objects above): after each handle_rx_symbol the PDUs
/// it registered run as one GPU job on `executor`.
std::unique_ptr<uplink_processor> create_uplink_processor_batch_gpu(std::unique_ptr<uplink_processor>  inner,
                                                                    std::shared_ptr<pusch_slot_batch> batch,
                                                                    task_executor&                    executor);

/// A slot batch of PDSCH transmissions (one per downlink processor). ptrs: the reference's PT-RS generator (host);
/// fallback: the processor for PDUs the batch does not cover (two codewords).
class pdsch_slot_batch;
std::shared_ptr<pdsch_slot_batch> create_pdsch_slot_batch(int                                   device,
                                                          std::unique_ptr<ptrs_pdsch_generator> ptrs,
                                                          std::unique_ptr<pdsch_processor>      fallback);

/// The pdsch_processor given to the reference's downlink processor: records each PDSCH into the batch.
std::unique_ptr<pdsch_processor> create_pdsch_processor_batch_gpu(std::shared_ptr<pdsch_slot_batch> batch);

/// The executor given to the reference's downlink processor: runs a task on the caller while the batching wrapper's
/// process_pdsch is in progress on this thread, forwards every other task to `real`.
class pdsch_batch_executor : public task_executor
{
public:
  explicit pdsch_batch_executor(task_executor& real_) : real(real_) {}
  [[nodiscard]] bool execute(unique_task task) override;
  [[nodiscard]] bool defer(unique_task task) override;

private:
  task_executor& real;
};

/// Wraps the reference's downlink_processor_single_executor_impl (built with the two objects above).
std::unique_ptr<downlink_processor_base> create_downlink_processor_batch_gpu(std::unique_ptr<downlink_processor_base> inner,
                                                                             std::shared_ptr<pdsch_slot_batch> batch,
                                                                             task_executor&                    executor);

} // namespace gpu
} // namespace srsran
