#!/usr/bin/env bash
# Builds libsrsgpu_phy.so (HIP kernels for gfx950 + the C-ABI host code) in-tree: srsran-5g_amd/lib/.
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/.." && pwd)
OUT="${SRSGPU_OUT_DIR:-$HERE/lib}"
mkdir -p "$OUT/obj"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$HERE/csrc ${SRSGPU_EXTRA_FLAGS:-}"
SRCS=("$HERE"/csrc/*.hip "$HERE"/csrc/*.cpp)
OBJS=()
pids=()
for src in "${SRCS[@]}"; do
  obj="$OUT/obj/$(basename "$src").o"
  OBJS+=("$obj")
  newest_hdr=$(ls -t "$HERE"/csrc/*.h "$ROOT"/include/*.h | head -1)
  if [ ! -f "$obj" ] || [ "$src" -nt "$obj" ] || [ "$newest_hdr" -nt "$obj" ] || [ "$0" -nt "$obj" ]; then
    # The demodulator's complex arithmetic is scalar f32: SLP packing into v_pk_* costs moves and ~40 VGPRs there.
    extra=""
    # The OFDM kernels likewise: the two-wave 4096-point transform spills under SLP at its 128-VGPR bound, and the
    # one-wave-per-16-points kernels take fewer VGPRs without it (74 vs 92 at 2048 points).
    [[ "$(basename "$src")" == pusch_demodulator.hip || "$(basename "$src")" == ofdm.hip ]] && extra="-fno-slp-vectorize"
    if [[ "$src" == *.hip ]]; then
      $HIPCC $FLAGS $extra -x hip -c "$src" -o "$obj" &
    else
      $HIPCC $FLAGS -c "$src" -o "$obj" &
    fi
    pids+=($!)
  fi
done
rc=0
for p in "${pids[@]:-}"; do [ -n "$p" ] && { wait "$p" || rc=1; }; done
[ $rc -eq 0 ] || { echo "build failed" >&2; exit 1; }
$HIPCC -shared -fPIC --offload-arch=gfx950 -o "$OUT/libsrsgpu_phy.so" "${OBJS[@]}"
echo "built $OUT/libsrsgpu_phy.so"
