#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.
# Builds oracle/_ref/libsrsref.so from the srsRAN reference sources where they lie under /root/reference (nothing is
# copied into this repository) plus oracle/ref/ref_shim.cpp. Output goes only to oracle/_ref/ (git-ignored, shipped to
# the GPU box with the snapshot). Skips quietly when the reference tree is absent (GPU box).
# SRSREF_MARCH=<level> builds a second copy, libsrsref_<level>.so, with every file at -march=<level> (the reference's
# own CMake builds at -march=native): the reference's floating-point results depend on the ISA it is built for
# (SIMD widths of its srsvec reductions, FMA contraction), and tests/test_reference_isa_variance.py measures by how much.
set -euo pipefail
REF=${SRSRAN_REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -d "$REF/lib/phy/upper/channel_coding/ldpc" ]; then
  echo "build_ref: reference tree not present; keeping existing $OUT" >&2
  exit 0
fi
MARCH=${SRSREF_MARCH:-}
LIBNAME=libsrsref.so
OBJDIR="$OUT/obj"
if [ -n "$MARCH" ]; then
  LIBNAME=libsrsref_$MARCH.so
  OBJDIR="$OUT/obj_$MARCH"
fi
mkdir -p "$OBJDIR"
CXX=${CXX:-g++}
FLAGS="-std=c++17 -O3 -fPIC -DNDEBUG -DFMT_HEADER_ONLY -DASSERTS_ENABLED=0 -I$REF/include -I$REF/external/fmt/include -I$REF/external -I$REF/lib/phy/upper/channel_coding"
LDPC=$REF/lib/phy/upper/channel_coding/ldpc
PDSCH=$REF/lib/phy/upper/channel_processors/pdsch
SRCS=(
  "$LDPC/ldpc_graph_impl.cpp:"
  "$LDPC/ldpc_luts_impl.cpp:"
  "$LDPC/ldpc_encoder_impl.cpp:"
  "$LDPC/ldpc_encoder_generic.cpp:"
  "$LDPC/ldpc_encoder_avx2.cpp:-mavx2"
  "$LDPC/ldpc_decoder_impl.cpp:"
  "$LDPC/ldpc_decoder_generic.cpp:"
  "$LDPC/ldpc_decoder_avx2.cpp:-mavx2"
  "$LDPC/ldpc_decoder_avx512.cpp:-mavx512f -mavx512bw"
  "$LDPC/ldpc_rate_matcher_impl.cpp:"
  "$LDPC/ldpc_rate_dematcher_impl.cpp:"
  "$LDPC/ldpc_rate_dematcher_avx2_impl.cpp:-mavx2"
  "$LDPC/ldpc_rate_dematcher_avx512_impl.cpp:-mavx512f -mavx512bw -mavx512vbmi"
  "$LDPC/ldpc_segmenter_tx_impl.cpp:"
  "$REF/lib/phy/upper/channel_coding/crc_calculator_generic_impl.cpp:"
  "$REF/lib/phy/upper/log_likelihood_ratio.cpp:-mavx2"
  "$REF/lib/srsvec/bit.cpp:-mavx2"
  "$REF/lib/srsvec/compare.cpp:-mavx2"
  "$REF/lib/srsvec/dot_prod.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/sc_prod.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/conversion.cpp:-mavx2 -mfma"
  "$HERE/ref/ref_shim.cpp:-mavx2"
  "$PDSCH/pdsch_modulator_impl.cpp:-mavx2 -I$PDSCH"
  "$REF/lib/phy/upper/channel_modulation/modulation_mapper_lut_impl.cpp:-mavx2"
  "$REF/lib/phy/upper/sequence_generators/pseudo_random_generator_impl.cpp:-mavx2"
  "$REF/lib/phy/support/resource_grid_mapper_impl.cpp:-mavx2"
  "$REF/lib/phy/support/resource_grid_impl.cpp:-mavx2"
  "$REF/lib/phy/support/resource_grid_writer_impl.cpp:-mavx2"
  "$REF/lib/phy/support/resource_grid_reader_impl.cpp:-mavx2"
  "$REF/lib/phy/support/re_pattern.cpp:-mavx2"
  "$REF/lib/phy/generic_functions/precoding/channel_precoder_generic.cpp:-mavx2"
  "$REF/lib/phy/generic_functions/precoding/channel_precoder_impl.cpp:-mavx2"
  "$REF/lib/phy/upper/rb_allocation.cpp:-mavx2"
  "$REF/lib/ran/resource_allocation/vrb_to_prb.cpp:-mavx2"
  "$HERE/ref/ref_pdsch_mod.cpp:-mavx2 -I$REF"
  "$REF/lib/phy/lower/modulation/ofdm_modulator_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/lower/modulation/ofdm_demodulator_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/generic_functions/dft_processor_generic_impl.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/prod.cpp:-mavx2 -mfma"
  "$HERE/ref/ref_ofdm.cpp:-mavx2 -mfma -I$REF"
  "$REF/lib/phy/upper/channel_processors/pusch/pusch_demodulator_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/equalization/channel_equalizer_generic_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/channel_modulation/demodulation_mapper_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/channel_modulation/demodulation_mapper_qpsk.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/channel_modulation/demodulation_mapper_qam16.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/channel_modulation/demodulation_mapper_qam64.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/channel_modulation/demodulation_mapper_qam256.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/channel_modulation/evm_calculator_generic_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/generic_functions/transform_precoding/transform_precoder_dft_impl.cpp:-mavx2 -mfma"
  "$HERE/ref/ref_pusch_demod.cpp:-mavx2 -mfma -I$REF"
  "$REF/lib/phy/upper/channel_processors/pusch/ulsch_demultiplex_impl.cpp:-mavx2 -mfma"
  "$HERE/ref/ref_ulsch_demux.cpp:-mavx2 -mfma -I$REF"
  "$REF/lib/phy/upper/signal_processors/dmrs_pusch_estimator_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/signal_processors/dmrs_helper.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/signal_processors/port_channel_estimator_average_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/signal_processors/port_channel_estimator_helpers.cpp:-mavx2 -mfma"
  "$REF/lib/phy/support/interpolator/interpolator_linear_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/support/time_alignment_estimator/time_alignment_estimator_dft_impl.cpp:-mavx2 -mfma"
  "$REF/lib/phy/upper/sequence_generators/low_papr_sequence_generator_impl.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/convolution.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/unwrap.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/add.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/subtract.cpp:-mavx2 -mfma"
  "$REF/lib/srsvec/modulus_square.cpp:-mavx2 -mfma"
  "$REF/lib/support/math_utils.cpp:-mavx2 -mfma"
  "$HERE/ref/ref_pusch_chest.cpp:-mavx2 -mfma -I$REF"
  "$REF/lib/phy/upper/signal_processors/dmrs_pdsch_processor_impl.cpp:-mavx2"
  "$HERE/ref/ref_dmrs_pdsch.cpp:-mavx2 -I$REF"
  "$HERE/ref/ref_slot_timed.cpp:-mavx2 -mfma -I$REF"
)
OBJS=()
pids=()
for entry in "${SRCS[@]}"; do
  src=${entry%%:*}; extra=${entry#*:}
  obj="$OBJDIR/$(basename "${src%.cpp}").o"
  [ -n "$MARCH" ] && extra="$extra -march=$MARCH"
  OBJS+=("$obj")
  if [ ! -f "$obj" ] || [ "$src" -nt "$obj" ] || [ "$0" -nt "$obj" ]; then
    $CXX $FLAGS $extra -c "$src" -o "$obj" &
    pids+=($!)
  fi
done
rc=0
for p in "${pids[@]:-}"; do [ -n "$p" ] && { wait "$p" || rc=1; }; done
[ $rc -eq 0 ] || { echo "build_ref: compilation failed" >&2; exit 1; }
$CXX -shared -o "$OUT/$LIBNAME" "${OBJS[@]}"
echo "build_ref: $OUT/$LIBNAME"
