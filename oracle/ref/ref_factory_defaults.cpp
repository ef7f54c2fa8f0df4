// TEST INFRASTRUCTURE ONLY. The reference's channel-processor factory interfaces declare one non-pure virtual each, the
// logging create() overload, defined next to the reference's software factories (their key functions, so the classes'
// type information lives there too):
//   channel_processor_factories.cpp:206 prach_detector_factory::create(logger, log_all_opportunities)
//   pucch/factories.cpp:268            pucch_processor_factory::create(logger)
//   pusch/factories.cpp:390            pusch_processor_factory::create(logger)
//   pdsch/factories.cpp:555            pdsch_processor_factory::create(logger, enable_logging_broadcast)
//   pdcch/factories.cpp:202            pdcch_processor_factory::create(logger, enable_logging_broadcast)
//   ssb/factories.cpp:209              ssb_processor_factory::create(logger)
//   signal_processor_factories.cpp:439 nzp_csi_rs_generator_factory::create(logger)
//   prs/factories.cpp:64               prs_generator_factory::create(logger)
//   srs/srs_estimator_factory.cpp:119  srs_estimator_factory::create(logger)
// Those files build every software factory of the PHY and so need the whole channel-processor library, which
// oracle/build_chain.sh does not compile. The factories of integration/upper_phy_factories_gpu.cpp (row b8) derive from
// these interfaces, and the tests give them small factories of their own, so the harness needs the classes' key
// functions: here they return the plain processor (the reference wraps it in a logging decorator; the tests never log,
// and the logging overloads are not called by them). A maintainer's build links the reference's own definitions.
#include "srsran/phy/upper/channel_processors/channel_processor_factories.h"
#include "srsran/phy/upper/channel_processors/pdcch/factories.h"
#include "srsran/phy/upper/channel_processors/pdsch/factories.h"
#include "srsran/phy/upper/channel_processors/pucch/factories.h"
#include "srsran/phy/upper/channel_processors/pusch/factories.h"
#include "srsran/phy/upper/channel_processors/ssb/factories.h"
#include "srsran/phy/upper/signal_processors/prs/factories.h"
#include "srsran/phy/upper/signal_processors/signal_processor_factories.h"
#include "srsran/phy/upper/signal_processors/srs/srs_estimator_factory.h"

using namespace srsran;

std::unique_ptr<prach_detector> prach_detector_factory::create(srslog::basic_logger& /*logger*/, bool /*log_all*/)
{
  return create();
}

std::unique_ptr<pucch_processor> pucch_processor_factory::create(srslog::basic_logger& /*logger*/)
{
  return create();
}

std::unique_ptr<pusch_processor> pusch_processor_factory::create(srslog::basic_logger& /*logger*/)
{
  return create();
}

std::unique_ptr<pdsch_processor> pdsch_processor_factory::create(srslog::basic_logger& /*logger*/, bool /*broadcast*/)
{
  return create();
}

std::unique_ptr<pdcch_processor> pdcch_processor_factory::create(srslog::basic_logger& /*logger*/, bool /*broadcast*/)
{
  return create();
}

std::unique_ptr<ssb_processor> ssb_processor_factory::create(srslog::basic_logger& /*logger*/)
{
  return create();
}

std::unique_ptr<nzp_csi_rs_generator> nzp_csi_rs_generator_factory::create(srslog::basic_logger& /*logger*/)
{
  return create();
}

std::unique_ptr<prs_generator> prs_generator_factory::create(srslog::basic_logger& /*logger*/)
{
  return create();
}

std::unique_ptr<srs_estimator> srs_estimator_factory::create(srslog::basic_logger& /*logger*/)
{
  return create();
}
