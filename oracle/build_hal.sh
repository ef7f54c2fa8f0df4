#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.
# Builds oracle/_ref/libsrshal.so: the reference's own transport-block processors (pusch_decoder_impl,
# pusch_codeblock_decoder, pusch_decoder_hw_impl, pdsch_encoder_impl, pdsch_encoder_hw_impl, the rx segmenter) compiled
# from their sources where they lie under /root/reference, the GPU bindings a maintainer adds (integration/*.cpp) and
# the C harness oracle/ref/ref_hal.cpp, linked against oracle/_ref/libsrsref.so (the rest of the reference build) and
# srsran-5g_amd/lib/libsrsgpu_phy.so. Output only into oracle/_ref/ (git-ignored, shipped to the GPU box with the
# snapshot). Skips quietly when the reference tree is absent (GPU box).
set -euo pipefail
REF=${SRSRAN_REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/.." && pwd)
OUT="$HERE/_ref"
if [ ! -d "$REF/lib/phy/upper/channel_processors/pusch" ]; then
  echo "build_hal: reference tree not present; keeping existing $OUT" >&2
  exit 0
fi
mkdir -p "$OUT/obj_hal"
CXX=${CXX:-g++}
FLAGS="-std=c++17 -O2 -fPIC -DNDEBUG -DFMT_HEADER_ONLY -DASSERTS_ENABLED=0 -mavx2 -mfma -I$REF/include
       -I$REF/external/fmt/include -I$REF/external -I$REF -I$REF/lib/phy/upper/channel_coding -I$ROOT/include
       -I$ROOT/integration -I/opt/rocm/include -D__HIP_PLATFORM_AMD__"
SRCS=(
  "$REF/lib/phy/upper/channel_processors/pusch/pusch_decoder_impl.cpp"
  "$REF/lib/phy/upper/channel_processors/pusch/pusch_codeblock_decoder.cpp"
  "$REF/lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.cpp"
  "$REF/lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp"
  "$REF/lib/phy/upper/channel_processors/pdsch/pdsch_encoder_hw_impl.cpp"
  "$REF/lib/phy/upper/channel_coding/ldpc/ldpc_segmenter_rx_impl.cpp"
  "$ROOT/integration/ldpc_decoder_gpu.cpp"
  "$ROOT/integration/hw_accelerator_pusch_dec_gpu.cpp"
  "$ROOT/integration/hw_accelerator_pdsch_enc_gpu.cpp"
  "$HERE/ref/ref_hal.cpp"
)
OBJS=()
pids=()
for src in "${SRCS[@]}"; do
  obj="$OUT/obj_hal/$(basename "${src%.cpp}").o"
  OBJS+=("$obj")
  if [ ! -f "$obj" ] || [ "$src" -nt "$obj" ] || [ "$0" -nt "$obj" ] || [ "$ROOT/integration/hw_accelerator_pusch_dec_gpu.h" -nt "$obj" ] || [ "$ROOT/integration/gpu_context.h" -nt "$obj" ] || [ "$ROOT/include/srsgpu_phy.h" -nt "$obj" ]; then
    $CXX $FLAGS -c "$src" -o "$obj" &
    pids+=($!)
  fi
done
rc=0
for p in "${pids[@]:-}"; do [ -n "$p" ] && { wait "$p" || rc=1; }; done
[ $rc -eq 0 ] || { echo "build_hal: compilation failed" >&2; exit 1; }
$CXX -shared -o "$OUT/libsrshal.so" "${OBJS[@]}" -L"$OUT" -lsrsref -L"$ROOT/srsran-5g_amd/lib" -lsrsgpu_phy \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN' -Wl,-rpath,'$ORIGIN/../../srsran-5g_amd/lib' -Wl,-rpath,/opt/rocm/lib \
  -Wl,--no-undefined
echo "build_hal: $OUT/libsrshal.so"
