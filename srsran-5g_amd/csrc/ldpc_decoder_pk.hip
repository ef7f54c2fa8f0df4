// Batched LDPC decoder for 5G NR, two lifted check rows per lane in packed 16-bit arithmetic, for gfx950.
//
// Same drop-in semantics and the same bit-exact results as ldpc_decoder.hip (reference
// lib/phy/upper/channel_coding/ldpc/ldpc_decoder_impl.cpp:60, check-node arithmetic of ldpc_decoder_avx2.cpp or
// ldpc_decoder_generic.cpp), for even lifting sizes. The check-node update is VALU-bound, so every instruction works
// on two rows at once: lane z (0 <= z < H = Z/2) owns rows z and z + H of every layer, and the v_pk_* 16-bit
// instructions (add/sub/min/max/shift/mad on both halves of a VGPR) carry the two rows' messages side by side. All
// intermediate values fit 16 bits: soft bits in [-121, 121], v2c in [-632, 632], search keys < 20243.
//
// LDS layout: column c of the lifted graph at c * 384, position p of the column at byte 2 * (p mod H) + (p >= H),
// so that the positions (z + s) mod Z and (z + H + s) mod Z that a lane reads for an edge of shift s are the two
// bytes of one pair: address a = min(2z + A_s, 2z + B_s) for a row-z value, a ^ 1 for the row-(z + H) value, with
// A_s = 2 (s mod H) + [s >= H] and B_s = A_s - 2H + 1 - 2 [s >= H] precomputed per (Z, edge) on the host.
//
// Compressed check-to-variable state per layer and lane (both rows, one per 16-bit half):
//   mag word:  min1 (7 b) | min2 (7 b) << 7            (scaled magnitudes)
//   sign word: sign bits of edges 0..10 | argmin << 11
//   hi word:   sign bits of edges 11..18 (the four 19-edge core rows of BG1 only)
#include "common.h"
#include "ldpc_base_graphs.h"
#include "ldpc_decoder_common.h"
#include "srsgpu_internal.h"

namespace srsgpu {
namespace {
using namespace ldpc_dec;

#ifdef LDPC_DEC_PROFILE
__device__ uint64_t g_dec_prof_pk[LDPC_DEC_PROF_CBS * LDPC_DEC_PROF_SLOTS];
#define DEC_PROF(slot, value)                                                                                          \
  do {                                                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < LDPC_DEC_PROF_CBS) {                                                          \
      g_dec_prof_pk[blockIdx.x * LDPC_DEC_PROF_SLOTS + (slot)] = (value);                                              \
    }                                                                                                                  \
  } while (0)
#else
#define DEC_PROF(slot, value)                                                                                          \
  do {                                                                                                                 \
  } while (0)
#endif
#define DEC_STAMP(slot) DEC_PROF(slot, __builtin_amdgcn_s_memtime())

typedef short          s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t bits(s16x2 v)
{
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ uint32_t bits(u16x2 v)
{
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ s16x2 as_s16(uint32_t v)
{
  return __builtin_bit_cast(s16x2, v);
}
__device__ __forceinline__ u16x2 as_u16(uint32_t v)
{
  return __builtin_bit_cast(u16x2, v);
}
__device__ __forceinline__ s16x2 ss(int x)
{
  return s16x2{static_cast<short>(x), static_cast<short>(x)};
}
__device__ __forceinline__ u16x2 uu(int x)
{
  return u16x2{static_cast<unsigned short>(x), static_cast<unsigned short>(x)};
}
/// Packed 16-bit VALU instructions issue at about two thirds of the rate of 32-bit ones on gfx950
/// (profiles/r3_valu_rate_probe_*.log): where an operation is bitwise the 32-bit form serves both halves.
/// 1 where IDX != e, 0 where IDX == e (both halves): IDX ^ e (one 32-bit v_xor on both 5-bit halves), then one
/// v_pk_min_u16 against an opaque 0x00010001 (a visible constant 1 gets the min rewritten into per-half compares and
/// cndmasks).
__device__ __forceinline__ u16x2 not_argmin(u16x2 idx, int e, u16x2 one)
{
  return __builtin_elementwise_min(as_u16(bits(idx) ^ (0x00010001u * static_cast<uint32_t>(e))), one);
}

/// Opaque packed multipliers 32 and 512: with a visible power of two the compiler splits a multiply-add into a
/// shift and an add / or (two VALU instead of one v_pk_mad).
struct pk_consts {
  u16x2    k32;
  uint32_t k271, kn271, kn21;  ///< 271, -271, -21 in both halves (SGPRs)
};
__device__ __forceinline__ pk_consts make_pk_consts()
{
  uint32_t a = 0x00200020u;
  asm("" : "+v"(a));
  uint32_t c = 0x010f010fu, d = 0xfef1fef1u, f = 0xffebffebu;
  asm("" : "+s"(c), "+s"(d), "+s"(f));
  return {as_u16(a), c, d, f};
}

/// v2c of an edge from its soft bit sb and t = sb - c2v: clamp(t, +/-LLR_MAX), plus +/-512 for an infinite soft bit
/// (|v2c| >= 392 stays infinite).
__device__ __forceinline__ s16x2 v2c_from_t(s16x2 t, s16x2 sb, const pk_consts& kc)
{
  const s16x2 ct  = __builtin_elementwise_min(__builtin_elementwise_max(t, ss(-LLR_MAX)), ss(LLR_MAX));
  // Infinity marker without clamping sb: g = sat16(271 sb) - 271 sb is 0 for |sb| <= 120 (271 x 120 = 32520) and
  // -24 / +23 for sb = +121 / -121 (the saturating v_pk_mad_i16 clamps 32791 to 32767); v = clamp(t) - 21 g puts an
  // infinite soft bit's v2c at +505..624 / -603..-484 (|v2c| >= 392 stays infinite; keys < 2^16).
  uint32_t sat;
  asm("v_pk_mad_i16 %0, %1, %2, 0 clamp" : "=v"(sat) : "v"(bits(sb)), "s"(kc.k271));
  const s16x2 g = sb * as_s16(kc.kn271) + as_s16(sat);
  return g * as_s16(kc.kn21) + ct;
}

/// v2c from the previous c2v magnitude om with sign mask n (0 / -1): sb - c2v is one multiply-add on
/// -(n | 1) = ~n | 1.
__device__ __forceinline__ s16x2 v2c_pk(s16x2 sb, u16x2 om, s16x2 n, const pk_consts& kc)
{
  const s16x2 nn = as_s16(~bits(n) | 0x00010001u);
  return v2c_from_t(as_s16(bits(om)) * nn + sb, sb, kc);
}

/// Check-to-variable messages kept whole (C2V layers): the signed c2v of both rows of edge e as int8, two edges per
/// word [c_z(e + 1), c_z(e), c_zH(e + 1), c_zH(e)] for even e, so that the even edge sits on the odd bytes, whose sign
/// bits v_perm replicates (selectors 8 / 9): one v_perm gives its two sign-extended 16-bit halves; the odd edge takes a
/// v_perm into the high bytes and an arithmetic shift. Against the compressed state (sign bits, argmin, min1 / min2)
/// this replaces the sign expansion, the argmin test and the magnitude select of pass 1 (6 VALU) by 1-2.
template <int e>
__device__ __forceinline__ s16x2 c2v_get(const uint32_t* cw)
{
  const uint32_t w = cw[e / 2];
  if constexpr (e % 2 == 0) {
    return as_s16(__builtin_amdgcn_perm(w, w, 0x09030801u));
  } else {
    return as_s16(__builtin_amdgcn_perm(w, w, 0x020c000cu)) >> ss(8);
  }
}
/// Words of c2v storage of a row of DEG edges.
constexpr int c2v_words(int deg)
{
  return (deg + 1) / 2;
}
/// Most words of c2v storage over the first L rows of a base graph.
template <typename G>
constexpr int c2v_words_max(int L)
{
  int w = 0;
  for (int m = 0; m < L; ++m) {
    w = c2v_words(G::rs(m + 1) - G::rs(m)) > w ? c2v_words(G::rs(m + 1) - G::rs(m)) : w;
  }
  return w;
}

/// Search key |v| * 32 + e of the two-minimum scan (one v_pk_mad).
__device__ __forceinline__ u16x2 key_pk(s16x2 v, int e, const pk_consts& kc)
{
  return __builtin_bit_cast(u16x2, __builtin_elementwise_max(v, -v)) * kc.k32 + uu(e);
}

__device__ __forceinline__ s16x2 clamp2(s16x2 v, int lo, int hi)
{
  return __builtin_elementwise_min(__builtin_elementwise_max(v, ss(lo)), ss(hi));
}

/// Byte address of the row-z soft bit of an edge: min(2z + A, 2z + B) in 16-bit halves (B < 0 wraps above every
/// valid address): one v_pk_add_u16 and a 16-bit min across the halves.
__device__ __forceinline__ uint32_t pair_address(uint32_t z2x2, uint32_t ab)
{
  const u16x2 t = as_u16(z2x2) + as_u16(ab);
  return t.x < t.y ? t.x : t.y;
}

/// Fixed-point normalisation parameters: MODE 1 scales m by (m * sf16) >> 16, evaluated in 16-bit halves as
/// ((m * hi) + ((m * lo) >> 8)) >> 8 with sf16 = hi * 256 + lo (exact: every product stays below 2^16).
struct scale_t {
  u16x2 hi;
  u16x2 lo;
  float sf;
};

template <int MODE>
__device__ __forceinline__ u16x2 scale_pk(u16x2 m, const scale_t& sc)
{
  if constexpr (MODE == 1) {
    const u16x2 l = (m * sc.lo) >> uu(8);
    return (m * sc.hi + l) >> uu(8);
  } else {
    // ldpc_decoder_generic.cpp:70 scale_llr: round half away from zero of m * sf (m >= 0).
    const unsigned short a = static_cast<unsigned short>(roundf(static_cast<float>(m.x) * sc.sf));
    const unsigned short b = static_cast<unsigned short>(roundf(static_cast<float>(m.y) * sc.sf));
    return u16x2{a, b};
  }
}

/// Bound on the CRC table loads in flight (each holds a result register): a scheduling barrier every CRC_CHUNK
/// systematic columns.
constexpr int CRC_CHUNK = 8;

/// Occupancy of the 8-layer class: at least 5 workgroups per CU (96 VGPRs, 5 waves per SIMD); 8 with the pass-1
/// addresses recomputed measured slower (r2: 117.8k vs 112.6k slots/s).
constexpr int PK_MIN_BLOCKS_8 = 5;
/// The one-codeblock 8-layer kernel keeps the core layers' c2v whole (C2V_CORE, 40 VGPRs instead of 12): up to 128
/// VGPRs, 4 waves per SIMD, which still holds the bench's whole launch (2 048 two-wave codeblocks on 1 024 SIMDs).
constexpr int PK_MIN_WAVES_C2V = 4;
/// Layers whose c2v messages the 8-layer kernel keeps whole: the four core rows (19 edges each in BG1).
constexpr int C2V_LAYERS = 4;
/// Layer bound up to which a row's pass-1 pair addresses stay in VGPRs for pass 2 (above it they are recomputed).
constexpr int PK_KEEP_ADDR_MAXL = 16;

/// Sign bits of edge e: bit e (e < 11) of the sign word or bit e - 11 of the hi word, in both halves.
constexpr int SIGNS_W0 = 11;

/// Two lifted check rows (z, z + H) of layer m: v2c messages, min-sum analysis, c2v messages, soft-bit update
/// (ldpc_decoder_impl.cpp:195, :255, :240; arithmetic of ldpc_decoder_avx2.cpp:69/:111/:165/:205).
template <int BG, int MODE, int m, bool KEEP_ADDR, int CS = SOFT_COL_STRIDE, bool C2V = false>
__device__ __forceinline__ void row_update_pk(int8_t* __restrict__ soft,
                                              const_u32_ptr  ab,  // A | B << 16 address constants of this Z
                                              uint32_t       z2x2,  // 2z in both halves
                                              const scale_t& sc,
                                              uint32_t&      magw,
                                              uint32_t&      sgw,
                                              uint32_t&      hiw,
                                              uint32_t*      cw = nullptr)  // C2V: the row's c2v words
{
  using G           = bg_t<BG>;
  constexpr int e0  = G::rs(m);
  constexpr int deg = G::rs(m + 1) - e0;
  static_assert(deg <= SIGNS_W0 + 8, "at most 19 edges per row");
  const u16x2 S1  = as_u16(magw & 0x007f007fu);
  const u16x2 S2  = as_u16((magw >> 7) & 0x007f007fu);
  const u16x2 D   = S1 - S2;
  const u16x2 IDX = as_u16(sgw) >> uu(11);
  s16x2       v2c[deg];
  u16x2       k1 = uu(KEY_INIT), k2 = uu(KEY_INIT);
  uint32_t    sx = 0;
  uint32_t    one_bits = 0x00010001u;
  asm("" : "+v"(one_bits));
  const u16x2     one = as_u16(one_bits);
  const pk_consts kc  = make_pk_consts();

  uint32_t addr[KEEP_ADDR ? deg : 1];
  static_for<deg>([&](auto E) {
    constexpr int  e   = decltype(E)::value;
    constexpr int  col = G::col(e0 + e);
    const uint32_t a   = pair_address(z2x2, ab[e0 + e]);
    if constexpr (KEEP_ADDR) {
      addr[e] = a;
    }
    // Two byte loads merged by one v_perm (d16 loads do not preserve the other half with SRAM ECC on gfx950).
    const s16x2 sb{static_cast<short>(soft[col * CS + a]), static_cast<short>(soft[col * CS + (a ^ 1u)])};
    // v2c = soft - c2v saturated to +/-LLR_MAX; infinite soft bits give |v2c| >= 392 (stay infinite).
    s16x2 v;
    if constexpr (C2V) {
      v = v2c_from_t(sb - c2v_get<e>(cw), sb, kc);
    } else {
      // Previous c2v of this edge: magnitude min2 at the argmin, min1 elsewhere; sign from the sign bits.
      constexpr int  pos = (e < SIGNS_W0) ? e : e - SIGNS_W0;
      const uint32_t sw  = (e < SIGNS_W0) ? sgw : hiw;
      const s16x2    n   = (as_s16(sw) << ss(15 - pos)) >> ss(15);
      const u16x2    ne  = not_argmin(IDX, e, one);
      const u16x2    om  = ne * D + S2;
      v                  = v2c_pk(sb, om, n, kc);
    }
    v2c[e]          = v;
    const u16x2 key = key_pk(v, e, kc);
    k2              = __builtin_elementwise_min(__builtin_elementwise_max(key, k1), k2);
    k1              = __builtin_elementwise_min(key, k1);
    sx ^= bits(v);
  });

  const u16x2 IDXN = k1 & uu(31);
  const u16x2 S1N  = scale_pk<MODE>(k1 >> uu(5), sc);
  const u16x2 S2N  = scale_pk<MODE>(k2 >> uu(5), sc);
  const u16x2 DN   = S1N - S2N;
  uint32_t    nsg  = bits(IDXN << uu(11));
  uint32_t    nhi  = 0;

  // With many layers of state the addresses are recomputed (2 VALU per edge) rather than kept: 19 fewer live VGPRs
  // for the core rows. The opaque copy stops the compiler from reusing pass-1 results.
  uint32_t z2x2_b = z2x2;
  if constexpr (!KEEP_ADDR) {
    asm volatile("" : "+v"(z2x2_b));
  }
  s16x2 c_even = ss(0);  // C2V: the c2v of the row's last even edge, packed with the next one
  // C2V: min1 / min2 signed once per layer by the sign of the product of all edges, so that an edge's c2v is its
  // magnitude times its own v2c sign (the product of the others' signs): no per-edge parity term.
  s16x2 M2s = ss(0), DMs = ss(0);
  if constexpr (C2V) {
    const s16x2 sall = as_s16(bits(as_s16(sx) >> ss(15)) | 0x00010001u);
    M2s              = as_s16(bits(S2N)) * sall;
    DMs              = as_s16(bits(S1N)) * sall - M2s;
  }
  static_for<deg>([&](auto E) {
    constexpr int e   = decltype(E)::value;
    constexpr int col = G::col(e0 + e);
    const s16x2   v   = v2c[e];
    // c2v sign = product of the other edges' signs; magnitude min2 at the argmin, min1 elsewhere.
    const s16x2 n   = C2V ? (v >> ss(15)) : (as_s16(sx ^ bits(v)) >> ss(15));
    const u16x2 ne  = not_argmin(IDXN, e, one);
    const u16x2 mag = C2V ? as_u16(bits(as_s16(bits(ne)) * DMs + M2s)) : ne * DN + S2N;
    // c2v + v2c as one multiply-add on the sign +/-1 (n | 1).
    const s16x2 sgn = as_s16(bits(n) | 0x00010001u);
    // Promotion sum (log_likelihood_ratio.cpp:75): |sum| > LLR_MAX becomes +/-infinity (SOFT_INF).
    s16x2 sb;
    if constexpr (C2V) {
      const s16x2 c = as_s16(bits(mag)) * sgn;
      sb            = clamp2(c + v, -SOFT_INF, SOFT_INF);
      if constexpr (e % 2 == 0) {
        c_even = c;
        if constexpr (e == deg - 1) {
          cw[e / 2] = __builtin_amdgcn_perm(bits(c), bits(c), 0x060c040cu);
        }
      } else {
        cw[e / 2] = __builtin_amdgcn_perm(bits(c_even), bits(c), 0x06020400u);
      }
    } else {
      sb = clamp2(as_s16(bits(mag)) * sgn + v, -SOFT_INF, SOFT_INF);
    }
    uint32_t       a;
    if constexpr (KEEP_ADDR) {
      a = addr[e];
    } else {
      a = pair_address(z2x2_b, ab[e0 + e]);
    }
    soft[col * CS + a]        = static_cast<int8_t>(sb.x);
    soft[col * CS + (a ^ 1u)] = static_cast<int8_t>(sb.y);
    constexpr int      pos  = (e < SIGNS_W0) ? e : e - SIGNS_W0;
    constexpr uint32_t mask = (1u << pos) | (1u << (16 + pos));
    if constexpr (C2V) {
    } else if constexpr (e < SIGNS_W0) {
      nsg |= bits(n) & mask;
    } else {
      nhi |= bits(n) & mask;
    }
  });
  if constexpr (!C2V) {
    magw = bits(S1N | (S2N << uu(7)));
    sgw  = nsg;
    if constexpr (deg > SIGNS_W0) {
      hiw = nhi;
    }
  }
}

/// Edge-split layer update (SPLIT = 2 kernels): the workgroup's two halves own the same rows; the lanes of half 0
/// process edges [0, ceil(deg / 2)) of their two rows, the lanes of half 1 the remaining edges, so each lane issues
/// about half the VALU instructions of a layer (a lone wave issues one VALU per ~6.5 cycles: with few codeblocks per
/// launch the per-codeblock latency, i.e. the instructions per wave, sets the kernel time). The two-minimum searches
/// are merged through LDS between the two passes; keys carry the global edge index, so the merge is exactly the
/// sequential scan. Each half keeps the sign bits of its own edges (at most 10: no hi word).
constexpr int HALF_MAX = 10;

struct half_state {
  s16x2    v2c[HALF_MAX];
  uint32_t addr[HALF_MAX];
  u16x2    k1, k2;
  uint32_t sx;
};

template <int BG, int MODE, int m, int EB, int EE>
__device__ __forceinline__ void pass1_half(const int8_t* __restrict__ soft,
                                           const_u32_ptr ab,
                                           uint32_t      z2x2,
                                           uint32_t      magw,
                                           uint32_t      sgw,
                                           half_state&   st)
{
  using G          = bg_t<BG>;
  constexpr int e0 = G::rs(m);
  static_assert(EE - EB <= HALF_MAX, "at most 10 edges per half row");
  const u16x2 S1  = as_u16(magw & 0x007f007fu);
  const u16x2 S2  = as_u16((magw >> 7) & 0x007f007fu);
  const u16x2 D   = S1 - S2;
  const u16x2 IDX = as_u16(sgw) >> uu(11);
  uint32_t    one_bits = 0x00010001u;
  asm("" : "+v"(one_bits));
  const u16x2     one = as_u16(one_bits);
  const pk_consts kc  = make_pk_consts();
  st.k1               = uu(KEY_INIT);
  st.k2           = uu(KEY_INIT);
  st.sx           = 0;
  static_for<EE - EB>([&](auto E) {
    constexpr int  j   = decltype(E)::value;
    constexpr int  e   = EB + j;
    constexpr int  col = G::col(e0 + e);
    const uint32_t a   = pair_address(z2x2, ab[e0 + e]);
    st.addr[j]         = a;
    const s16x2 sb{static_cast<short>(soft[col * SOFT_COL_STRIDE + a]),
                   static_cast<short>(soft[col * SOFT_COL_STRIDE + (a ^ 1u)])};
    const s16x2 n   = (as_s16(sgw) << ss(15 - j)) >> ss(15);
    const u16x2 ne  = not_argmin(IDX, e, one);
    const u16x2 om  = ne * D + S2;
    const s16x2 v   = v2c_pk(sb, om, n, kc);
    st.v2c[j]       = v;
    const u16x2 key = key_pk(v, e, kc);
    st.k2           = __builtin_elementwise_min(__builtin_elementwise_max(key, st.k1), st.k2);
    st.k1           = __builtin_elementwise_min(key, st.k1);
    st.sx ^= bits(v);
  });
}

template <int BG, int MODE, int m, int EB, int EE>
__device__ __forceinline__ void pass2_half(int8_t* __restrict__ soft,
                                           const scale_t&    sc,
                                           u16x2             k1,
                                           u16x2             k2,
                                           uint32_t          sx,
                                           const half_state& st,
                                           uint32_t&         magw,
                                           uint32_t&         sgw)
{
  using G          = bg_t<BG>;
  constexpr int e0 = G::rs(m);
  uint32_t      one_bits = 0x00010001u;
  asm("" : "+v"(one_bits));
  const u16x2 one  = as_u16(one_bits);
  const u16x2 IDXN = k1 & uu(31);
  const u16x2 S1N  = scale_pk<MODE>(k1 >> uu(5), sc);
  const u16x2 S2N  = scale_pk<MODE>(k2 >> uu(5), sc);
  const u16x2 DN   = S1N - S2N;
  uint32_t    nsg  = bits(IDXN << uu(11));
  static_for<EE - EB>([&](auto E) {
    constexpr int j   = decltype(E)::value;
    constexpr int e   = EB + j;
    constexpr int col = G::col(e0 + e);
    const s16x2   v   = st.v2c[j];
    const s16x2   n   = as_s16(sx ^ bits(v)) >> ss(15);
    const u16x2   ne  = not_argmin(IDXN, e, one);
    const u16x2   mag = ne * DN + S2N;
    const s16x2   sgn = as_s16(bits(n) | 0x00010001u);
    const s16x2   sb  = clamp2(as_s16(bits(mag)) * sgn + v, -SOFT_INF, SOFT_INF);
    const uint32_t a  = st.addr[j];
    soft[col * SOFT_COL_STRIDE + a]        = static_cast<int8_t>(sb.x);
    soft[col * SOFT_COL_STRIDE + (a ^ 1u)] = static_cast<int8_t>(sb.y);
    constexpr uint32_t mask = (1u << j) | (1u << (16 + j));
    nsg |= bits(n) & mask;
  });
  magw = bits(S1N | (S2N << uu(7)));
  sgw  = nsg;
}

/// LDS byte offset of position l (0 <= l < Z) inside a column.
__device__ __forceinline__ uint32_t pair_pos(uint32_t l, uint32_t H)
{
  return (l < H) ? 2u * l : 2u * (l - H) + 1u;
}

/// Hard decisions of the K*Z systematic bits, packed MSB first (log_likelihood_ratio.cpp:350 hard_decision).
__device__ __forceinline__ void write_hard_bits_pk(const int8_t* __restrict__ soft,
                                                   uint8_t* __restrict__ out,
                                                   int      nbits,
                                                   int      Z,
                                                   uint32_t magic)
{
  const uint32_t H      = static_cast<uint32_t>(Z) / 2u;
  const int      nbytes = (nbits + 7) / 8;
  for (int b = threadIdx.x; b < nbytes; b += blockDim.x) {
    uint32_t byte = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = 8 * b + k;
      if (i < nbits) {
        const uint32_t col = __umulhi(static_cast<uint32_t>(i), magic);
        const uint32_t l   = static_cast<uint32_t>(i) - col * static_cast<uint32_t>(Z);
        byte |= static_cast<uint32_t>(soft[col * SOFT_COL_STRIDE + pair_pos(l, H)] <= 0) << (7 - k);
      }
    }
    out[b] = static_cast<uint8_t>(byte);
  }
}

/// MAXL: compile-time bound on the number of layers (host-proven from the input length, dec_desc::nof_llr), so that
/// only MAXL layers of check-to-variable state occupy VGPRs: the 4-layer high-rate codeblocks of a loaded cell run at
/// twice the occupancy of the 46-layer worst case.
/// FUSE: the codeblock is a first transmission whose rate dematching is a plain copy (rv 0, no limited buffer,
/// ninfo <= E <= V: every systematic position is reached and nothing repeats): the kernel dematches the codeword LLRs
/// itself (dms[blockIdx.x]) into the LDS image and writes the HARQ soft buffer the separate rate_dematch_kernel would
/// have written (rate_dematcher.hip dematch_new_data: copies symbol-major, fillers +127, the unreached tail zeroed).
template <int BG, int MODE, int MAXL, int SPLIT, bool FUSE>
__global__ __launch_bounds__(192 * SPLIT, (SPLIT == 2 ? 2 : (MAXL > 16 ? 3 : (MAXL > 8 ? 4 : PK_MIN_WAVES_C2V)))) void ldpc_decode_pk_kernel(const dec_desc* __restrict__ descs,
                                                             const int8_t* __restrict__ llrs,
                                                             uint8_t* __restrict__ out,
                                                             int32_t* __restrict__ results,
                                                             const uint32_t* __restrict__ ab_table,
                                                             const uint32_t* __restrict__ crc_tables,
                                                             uint8_t* __restrict__ cb_crc_ok,
                                                             const dm_desc* __restrict__ dms,
                                                             int8_t* __restrict__ harq,
                                                             int8_t* const* __restrict__ harq_cbs)
{
  using G = bg_t<BG>;
  // Only the first K + MAXL columns can be touched by MAXL layers: the soft-bit image shrinks with the layer bound
  // (11.8 KB for 8 layers of BG1 instead of 26 KB), so more codeblocks share a CU.
  constexpr int NCOL = G::K + MAXL;
  // SPLIT = 2: the halves exchange (k1, k2, sign parity) per row through MERGE_BYTES of LDS every layer.
  constexpr int MERGE_BYTES = (SPLIT == 2) ? 2 * 192 * 16 : 0;
  __shared__ __attribute__((aligned(16))) int8_t smem[NCOL * SOFT_COL_STRIDE + SCRATCH_BYTES + MERGE_BYTES];
  int8_t* soft    = smem;
  int*    scratch = reinterpret_cast<int*>(smem + NCOL * SOFT_COL_STRIDE);
  uint4*  merge   = reinterpret_cast<uint4*>(smem + NCOL * SOFT_COL_STRIDE + SCRATCH_BYTES);

  DEC_STAMP(0);
  DEC_PROF(29, __builtin_amdgcn_s_memrealtime());
  const dec_desc d = descs[blockIdx.x];
  if constexpr (FUSE) {
    // New data invalidates the codeblock CRC flag of the HARQ context (pusch_decoder_impl.cpp:132).
    if (cb_crc_ok != nullptr && threadIdx.x == 0) {
      cb_crc_ok[d.cb_index] = 0;
    }
  } else if (cb_crc_ok != nullptr && cb_crc_ok[d.cb_index] != 0) {
    // HARQ context (pusch_decoder_impl.cpp:300): a codeblock whose CRC already passed is not decoded again.
    if (threadIdx.x == 0) {
      results[d.cb_index] = 0;
    }
    return;
  }
  const int      Z  = d.Z;
  const uint32_t H  = static_cast<uint32_t>(Z) / 2u;
  const auto     ab = (const_u32_ptr)(uintptr_t)(ab_table + static_cast<uint32_t>(d.zpos) * G::NE);
  asm volatile("" ::"s"(llrs), "s"(out), "s"(results), "s"(crc_tables), "s"(cb_crc_ok), "s"(blockDim.x));
  // Scalar-cache warm-up of this Z's address constants while the LLRs load (see ldpc_decoder.hip).
  constexpr int AB_BYTES = G::NE * 4;
  constexpr int AB_LINES = (AB_BYTES - 4) / 64 + 2;
  uint32_t      pf[AB_LINES];
  static_for<AB_LINES>([&](auto L) {
    constexpr int l = decltype(L)::value;
    scalar_touch<(l * 64 < AB_BYTES - 4) ? l * 64 : AB_BYTES - 4>(pf[l], ab);
  });
  // SPLIT = 2: threads [0, hb) and [hb, 2 hb) are the two edge halves of the same rows.
  const int  hb     = (SPLIT == 2) ? static_cast<int>(blockDim.x) / 2 : static_cast<int>(blockDim.x);
  const int  half   = (SPLIT == 2 && static_cast<int>(threadIdx.x) >= hb) ? 1 : 0;
  const int  z      = static_cast<int>(threadIdx.x) - half * hb;
  const bool active = static_cast<uint32_t>(z) < H;
  const int  wave   = threadIdx.x / WAVE;
  const int  nwaves = blockDim.x / WAVE;
  const int  lane   = threadIdx.x % WAVE;

  // ---- LLRs -> soft-bit image (ldpc_decoder_impl.cpp:152), last non-zero LLR (:94); as ldpc_decoder.hip but with
  // the pair layout: a 16-byte vector inside one half of one column is a stride-2 run of bytes. ----
  // The codeblock's HARQ soft buffer (the input of an unfused codeblock, the output of a fused one): at its offset in
  // the batch buffer, or wherever harq_cbs[cb] points (a persistent rx-buffer arena slot).
  const int8_t*  llr   = (!FUSE && harq_cbs != nullptr) ? harq_cbs[d.cb_index] : llrs + d.llr_offset;
  const int      n_llr = static_cast<int>(d.nof_llr);
  const uint32_t ncols = __umulhi(static_cast<uint32_t>(n_llr), d.div_magic);
  const uint32_t full  = ncols * static_cast<uint32_t>(Z);
  int            last  = -1;
  if constexpr (FUSE) {
    const dm_desc  dm    = dms[blockIdx.x];
    const int      E     = static_cast<int>(dm.E), Qm = dm.Qm, R = E / Qm;
    const int      Fl    = dm.nof_filler;
    const int      ninfo = static_cast<int>(dm.nsys) - Fl;
    const int      Nh    = static_cast<int>(dm.N);
    const int8_t*  in    = llrs + dm.llr_offset;
    int8_t*        hb    = (harq_cbs != nullptr) ? harq_cbs[d.cb_index] : harq + dm.harq_offset;
    // The whole image starts at zero (punctured columns, positions beyond the input and the unreached tail).
    {
      uint4* s16 = reinterpret_cast<uint4*>(soft);
      for (int q = threadIdx.x; q < NCOL * SOFT_COL_STRIDE / 16; q += blockDim.x) {
        s16[q] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    __syncthreads();
    // Decoder input clamp (ldpc_decoder_impl.cpp:152): +/-64 in the whole lifted columns of the input, the
    // reference's LLR range (+/-infinity kept) in a trailing partial column; trailing-zero trim over [0, n_llr).
    auto soft_put = [&](int k, int v) {
      if (static_cast<uint32_t>(k) < static_cast<uint32_t>(n_llr)) {
        last              = (v != 0 && k > last) ? k : last;
        const uint32_t cq = __umulhi(static_cast<uint32_t>(k), d.div_magic);
        const int      cv = (static_cast<uint32_t>(k) < full) ? clamp_i(v, -64, 64) : clamp_i(v, -SOFT_INF, SOFT_INF);
        soft[(cq + 2) * SOFT_COL_STRIDE + pair_pos(static_cast<uint32_t>(k) - cq * static_cast<uint32_t>(Z), H)] =
            static_cast<int8_t>(cv);
      }
    };
    auto put = [&](int k, int v) {
      hb[k] = static_cast<int8_t>(v);
      soft_put(k, v);
    };
    // Copies, symbol-major: lane r reads the Qm LLRs of symbol r and stores bit j at visit n = j R + r (position k =
    // n, past the fillers once n >= ninfo); for a fixed j the lanes' HARQ stores are consecutive bytes. 256QAM with
    // 4-aligned R, ninfo, fillers and HARQ buffer (every bench codeblock): a lane takes four consecutive symbols and
    // writes each bit row's four HARQ bytes as one dword (8 dword stores per 4 symbols instead of 32 byte stores).
    const bool q8 = Qm == 8 && ((dm.llr_offset & 7u) == 0u);
    const bool q8x4 = q8 &&
                      ((R | ninfo | Fl | static_cast<int>(reinterpret_cast<uintptr_t>(hb))) & 3) == 0;
    if (q8x4) {
      for (int r0 = 4 * static_cast<int>(threadIdx.x); r0 < R; r0 += 4 * static_cast<int>(blockDim.x)) {
        uint2 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = *reinterpret_cast<const uint2*>(in + 8 * (r0 + q));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          uint32_t w = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t byte = (((j < 4) ? v[q].x : v[q].y) >> (8 * (j & 3))) & 0xffu;
            w |= byte << (8 * q);
          }
          const int n = j * R + r0;  // n .. n + 3 on one side of ninfo (both multiples of 4)
          const int k = n < ninfo ? n : n + Fl;
          *reinterpret_cast<uint32_t*>(hb + k) = w;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            soft_put(k + q, static_cast<int8_t>(w >> (8 * q)));
          }
        }
      }
    } else {
      for (int r = threadIdx.x; r < R; r += blockDim.x) {
        int8_t sym[8];
        if (q8) {
          const uint2 v = *reinterpret_cast<const uint2*>(in + 8 * r);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            sym[j] = static_cast<int8_t>(((j < 4) ? v.x : v.y) >> (8 * (j & 3)));
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            sym[j] = (j < Qm) ? in[r * Qm + j] : 0;
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (j < Qm) {
            const int n = j * R + r;
            put(n < ninfo ? n : n + Fl, sym[j]);
          }
        }
      }
    }
    // Fillers: +infinity (ldpc_rate_dematcher_impl.cpp:172); then the unreached tail [E + F, N) zeroed (16-byte
    // stores between the unaligned head and tail bytes).
    for (int k = ninfo + static_cast<int>(threadIdx.x); k < ninfo + Fl; k += blockDim.x) {
      put(k, 127);
    }
    {
      const int t0 = E + Fl;
      const int a0 = min(Nh, t0 + static_cast<int>((16u - (reinterpret_cast<uintptr_t>(hb + t0) & 15u)) & 15u));
      const int nv = (Nh - a0) / 16;
      const int a1 = a0 + 16 * nv;
      if (static_cast<int>(threadIdx.x) < a0 - t0) {
        hb[t0 + static_cast<int>(threadIdx.x)] = 0;
      }
      uint4* z16 = reinterpret_cast<uint4*>(hb + a0);
      for (int q = threadIdx.x; q < nv; q += blockDim.x) {
        z16[q] = make_uint4(0u, 0u, 0u, 0u);
      }
      if (static_cast<int>(threadIdx.x) < Nh - a1) {
        hb[a1 + static_cast<int>(threadIdx.x)] = 0;
      }
    }
  } else {
    {
      const uint32_t head   = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(llr)) & 15u;
      const uint4*   vecs   = reinterpret_cast<const uint4*>(llr - head);
      const int      nvec   = static_cast<int>((head + static_cast<uint32_t>(n_llr) + 15u) >> 4);
      // 16-B vectors per lane in flight: the whole input span of the layer bound at Z = 384 with 192 lanes.
      constexpr int  BATCH  = ((NCOL - 2) * 384 / 16 + 191) / 192;
      int            last_w = -1;
      uint4          last_v = make_uint4(0u, 0u, 0u, 0u);
      for (int w0 = threadIdx.x; w0 < nvec; w0 += BATCH * blockDim.x) {
        uint4 val[BATCH];
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
          const int w = w0 + j * blockDim.x;
          val[j]      = (w < nvec) ? vecs[w] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
          const int w = w0 + j * blockDim.x;
          if (w >= nvec) {
            continue;
          }
          const uint32_t i0 = static_cast<uint32_t>(16 * w) - head;
          const uint32_t c0 = __umulhi(i0, d.div_magic);
          const uint32_t l0 = i0 - c0 * static_cast<uint32_t>(Z);
          // Short path: the 16 LLRs lie in one column (every vector but the unaligned head and the input's tail). A
          // vector may straddle the column's half boundary H: byte k >= H - l0 goes to 2 (l - H) + 1 instead of 2 l,
          // i.e. its address moves by 1 - 2H (one bit-extract and one 24-bit multiply-add per byte, no branch), so a
          // wave's straddling lane does not drag the whole wave through the per-byte general path.
          const bool short_path = (16u * static_cast<uint32_t>(w) >= head) && (i0 + 16u <= full) &&
                                  (l0 + 16u <= static_cast<uint32_t>(Z));
          if (short_path) {
            int8_t*        dst   = soft + (c0 + 2) * SOFT_COL_STRIDE + pair_pos(l0, H);
            const uint32_t cross = (l0 < H && l0 + 16u > H) ? (0xffffu << (H - l0)) : 0u;  // bit k: byte k moves
            const int      adj   = 1 - 2 * static_cast<int>(H);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const uint32_t word = (q == 0) ? val[j].x : (q == 1) ? val[j].y : (q == 2) ? val[j].z : val[j].w;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const int kk  = 4 * q + k;
                const int mv  = static_cast<int>((cross >> kk) & 1u) * adj;
                dst[2 * kk + mv] = static_cast<int8_t>(clamp_i(static_cast<int8_t>(word >> (8 * k)), -64, 64));
              }
            }
            if ((val[j].x | val[j].y | val[j].z | val[j].w) != 0u) {
              last_w = w;
              last_v = val[j];
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const uint32_t word = (q == 0) ? val[j].x : (q == 1) ? val[j].y : (q == 2) ? val[j].z : val[j].w;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const uint32_t i = i0 + static_cast<uint32_t>(4 * q + k);
                if (i < static_cast<uint32_t>(n_llr)) {
                  int v = static_cast<int8_t>(word >> (8 * k));
                  last  = (v != 0) ? static_cast<int>(i) : last;
                  v     = (i < full) ? clamp_i(v, -64, 64) : clamp_i(v, -SOFT_INF, SOFT_INF);
                  const uint32_t cq = __umulhi(i, d.div_magic);
                  soft[(cq + 2) * SOFT_COL_STRIDE + pair_pos(i - cq * static_cast<uint32_t>(Z), H)] =
                      static_cast<int8_t>(v);
                }
              }
            }
          }
        }
      }
      if (last_w >= 0) {
        const uint32_t words[4] = {last_v.x, last_v.y, last_v.z, last_v.w};
        int            hb       = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          hb = (words[q] != 0u) ? 4 * q + (31 - __clz(static_cast<int>(words[q]))) / 8 : hb;
        }
        const int i = 16 * last_w - static_cast<int>(head) + hb;
        last        = i > last ? i : last;
      }
    }
    // Zero the punctured columns 0, 1 and every position beyond the input.
    if (active && half == 0) {
      auto* soft16 = reinterpret_cast<uint16_t*>(soft);
      soft16[(0 * SOFT_COL_STRIDE) / 2 + z] = 0;
      soft16[(1 * SOFT_COL_STRIDE) / 2 + z] = 0;
      int c = 2 + static_cast<int>(ncols);
      if (static_cast<uint32_t>(n_llr) > full) {
        const uint32_t rem = static_cast<uint32_t>(n_llr) - full;
        if (static_cast<uint32_t>(z) >= rem) {
          soft[c * SOFT_COL_STRIDE + 2 * z] = 0;
        }
        if (static_cast<uint32_t>(z) + H >= rem) {
          soft[c * SOFT_COL_STRIDE + 2 * z + 1] = 0;
        }
        ++c;
      }
      for (; c < NCOL; ++c) {
        soft16[(c * SOFT_COL_STRIDE) / 2 + z] = 0;
      }
    }
  }
  last = wave_max(last);
  if (lane == 0) {
    scratch[wave] = last;
  }
  __syncthreads();
  // Consume the scalar-cache warm-up loads (they landed long ago; the compiler places the wait).
  static_for<AB_LINES>([&](auto L) { keep_sgpr(pf[decltype(L)::value]); });
  int input_size = scratch[0];
  for (int w = 1; w < nwaves; ++w) {
    input_size = scratch[w] > input_size ? scratch[w] : input_size;
  }
  input_size += 1;

  const int  msg_len = G::K * Z;
  uint8_t*   cb_out  = out + d.out_offset;
  const bool use_crc = d.crc_table != NO_CRC_TABLE;
  if (input_size < msg_len) {
    // Not enough LLRs: no decoding; when the CRC is not the decoder's (no CRC, or checked by the caller after the
    // last iteration: no early stop, pusch_codeblock_decoder passes no calculator) the output is all ones
    // (ldpc_decoder_impl.cpp:95).
    if (!use_crc || (d.flags & DEC_FLAG_EARLY_STOP) == 0) {
      for (int b = threadIdx.x; b < (msg_len + 7) / 8; b += blockDim.x) {
        cb_out[b] = 0xff;
      }
    }
    if (threadIdx.x == 0) {
      results[d.cb_index] = -1;
    }
    return;
  }
  int cb_len = input_size + 2 * Z;
  cb_len     = cb_len > msg_len + 4 * Z ? cb_len : msg_len + 4 * Z;
  const int nof_layers =
      __builtin_amdgcn_readfirstlane(static_cast<int>(__umulhi(static_cast<uint32_t>(cb_len + Z - 1), d.div_magic)) -
                                     G::K);

  const uint32_t* crc_table = crc_tables + (use_crc ? d.crc_table : 0u);
  scale_t         sc;
  sc.hi = uu(static_cast<int>(d.sf16 >> 8));
  sc.lo = uu(static_cast<int>(d.sf16 & 255u));
  sc.sf = d.sf;

  static_assert(MAXL >= 4 && MAXL <= G::M, "layer bound");
  if (nof_layers > MAXL) {
    // The host bound is derived from the same input length: cannot happen; fail loudly rather than decode wrongly.
    if (threadIdx.x == 0) {
      results[d.cb_index] = -2;
    }
    return;
  }
  uint32_t magw[MAXL], sgw[MAXL];
  uint32_t hiw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int m = 0; m < MAXL; ++m) {
    magw[m] = 0;
    sgw[m]  = 0;
  }
  // The core layers' c2v kept whole (zero before the first iteration: v2c = soft, ldpc_decoder_impl.cpp:218).
  constexpr bool C2V_CORE = (SPLIT == 1 && MAXL == 8);
  constexpr int  C2V_W    = c2v_words_max<G>(C2V_LAYERS);
  uint32_t       c2vw[C2V_LAYERS][C2V_W];
#pragma unroll
  for (int m = 0; m < C2V_LAYERS; ++m) {
#pragma unroll
    for (int w = 0; w < C2V_W; ++w) {
      c2vw[m][w] = 0u;
    }
  }
  __syncthreads();

  const int max_iter = d.max_iter;
  DEC_STAMP(1);
  DEC_PROF(31, static_cast<uint64_t>(nof_layers));
  for (int it = 0; it < max_iter; ++it) {
    // Opaque per-iteration copies (see ldpc_decoder.hip).
    int           nl   = nof_layers;
    uint32_t      z2x2 = 0x00020002u * static_cast<uint32_t>(z);
    const_u32_ptr abi  = ab;
    asm volatile("" : "+s"(nl));
    asm volatile("" : "+v"(z2x2));
    asm volatile("" : "+s"(abi));
    static_for<MAXL>([&](auto Mi) {
      constexpr int m = decltype(Mi)::value;
      if (m < nl) {
        if constexpr (SPLIT == 1) {
          if (active) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (C2V_CORE && m < C2V_LAYERS) {
              row_update_pk<BG, MODE, m, true, SOFT_COL_STRIDE, true>(soft, abi, z2x2, sc, magw[m], sgw[m],
                                                                      hiw[m & 3], c2vw[m]);
            } else {
              row_update_pk<BG, MODE, m, (MAXL <= PK_KEEP_ADDR_MAXL)>(soft, abi, z2x2, sc, magw[m], sgw[m],
                                                                           hiw[m & 3]);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {
          constexpr int deg = G::rs(m + 1) - G::rs(m);
          constexpr int hm  = (deg + 1) / 2;
          half_state    st;
          if (active) {
            if (half == 0) {
              pass1_half<BG, MODE, m, 0, hm>(soft, abi, z2x2, magw[m], sgw[m], st);
            } else {
              pass1_half<BG, MODE, m, hm, deg>(soft, abi, z2x2, magw[m], sgw[m], st);
            }
            merge[half * hb + z] = make_uint4(bits(st.k1), bits(st.k2), st.sx, 0u);
          }
          __syncthreads();
          if (active) {
            const uint4 pr = merge[(1 - half) * hb + z];
            const u16x2 pk1 = as_u16(pr.x), pk2 = as_u16(pr.y);
            const u16x2 k1  = __builtin_elementwise_min(st.k1, pk1);
            const u16x2 k2  = __builtin_elementwise_min(__builtin_elementwise_max(st.k1, pk1),
                                                        __builtin_elementwise_min(st.k2, pk2));
            const uint32_t sx = st.sx ^ pr.z;
            if (half == 0) {
              pass2_half<BG, MODE, m, 0, hm>(soft, sc, k1, k2, sx, st, magw[m], sgw[m]);
            } else {
              pass2_half<BG, MODE, m, hm, deg>(soft, sc, k1, k2, sx, st, magw[m], sgw[m]);
            }
          }
        }
        __syncthreads();
      }
    });
    DEC_STAMP(2 + 2 * (it & 7));

    // CRC after every iteration with early stop (ldpc_decoder_impl.cpp:133), else after the last one.
    if (use_crc && ((d.flags & DEC_FLAG_EARLY_STOP) != 0 || it == max_iter - 1)) {
      uint32_t acc  = 0;
      uint32_t zero = 0;
      if (active) {
        // Opaque copies again: per-column table offsets would otherwise be hoisted out of the iteration loop. The
        // table loads are unconditional (index clamped, value masked): no divergent branches between them, all of
        // a chunk's loads in flight at once, saddr form (global base in SGPRs + 32-bit byte offset).
        uint32_t zz   = static_cast<uint32_t>(z);
        uint32_t ZZ   = static_cast<uint32_t>(Z);
        uint32_t HH   = H;
        asm volatile("" : "+v"(zz));
        asm volatile("" : "+s"(ZZ), "+s"(HH));
        // SPLIT = 2: half 0 sums the first K / 2 columns, half 1 the rest (hcol = half x K / 2).
        constexpr int KC   = (SPLIT == 2) ? G::K / 2 : G::K;
        const int     hcol = half * KC;
        uint32_t      ia   = zz + static_cast<uint32_t>(hcol) * ZZ;
        const int8_t* scol = soft + hcol * SOFT_COL_STRIDE;
        static_for<KC>([&](auto Ci) {
          constexpr int  c  = decltype(Ci)::value;
          const uint32_t ib = ia + HH;
          const int      sa = scol[c * SOFT_COL_STRIDE + 2 * zz];
          const int      sb = scol[c * SOFT_COL_STRIDE + 2 * zz + 1];
          zero |= static_cast<uint32_t>(sa == 0) | static_cast<uint32_t>(sb == 0);
          // ia, ib < K Z: positions past the message (fillers) read the table's zero tail (get_crc_table).
          const uint32_t ta = crc_table[ia];
          const uint32_t tb = crc_table[ib];
          acc ^= (sa <= 0) ? ta : 0u;
          acc ^= (sb <= 0) ? tb : 0u;
          ia += ZZ;
          // Bound the table loads in flight (each holds a result register).
          if constexpr (c % CRC_CHUNK == CRC_CHUNK - 1) {
            __builtin_amdgcn_sched_barrier(0);
          }
        });
      }
      acc      = wave_xor(acc);
      zero     = (__ballot(zero != 0) != 0) ? 1u : 0u;
      int* red = scratch + 8 + 16 * (it & 1);
      if (lane == 0) {
        red[2 * wave]     = static_cast<int>(acc);
        red[2 * wave + 1] = static_cast<int>(zero);
      }
      __syncthreads();
      uint32_t tacc = 0, tzero = 0;
      for (int w = 0; w < nwaves; ++w) {
        tacc ^= static_cast<uint32_t>(red[2 * w]);
        tzero |= static_cast<uint32_t>(red[2 * w + 1]);
      }
      const bool early = (d.flags & DEC_FLAG_EARLY_STOP) != 0;
      DEC_STAMP(3 + 2 * (it & 7));
      if ((tzero == 0 || !early) && tacc == 0) {
        write_hard_bits_pk(soft, cb_out, msg_len, Z, d.div_magic);
        DEC_STAMP(28);
        DEC_PROF(30, __builtin_amdgcn_s_memrealtime());
        if (threadIdx.x == 0) {
          results[d.cb_index] = it + 1;
          if (cb_crc_ok != nullptr) {
            cb_crc_ok[d.cb_index] = 1;
          }
        }
        return;
      }
    }
  }
  write_hard_bits_pk(soft, cb_out, msg_len, Z, d.div_magic);
  DEC_STAMP(28);
  DEC_PROF(30, __builtin_amdgcn_s_memrealtime());
  if (threadIdx.x == 0) {
    results[d.cb_index] = -1;
  }
}

// ---------------------------------------------------------------------------------------------------------------------
// Two-codeblock workgroups (SRSGPU_OPTION_DECODER_PAIRS). The plain kernel gives a codeblock 64 * ceil(Z / 128) lanes:
// a Z = 144..192 codeblock runs two waves of which the second is partly idle, and every wave issues the full instruction
// stream. Here two codeblocks of one lifting size share a workgroup: codeblock slot i owns lanes [i H, (i + 1) H), so
// two Z = 192 codeblocks fill three waves, and a wave whose codeblocks have both stopped skips the layer bodies.
//
// The soft-bit images of the slots are interleaved pair by pair: position p of column c of slot i is at byte
// c * CS + 2 * PKN * (p mod H) + 2 i + [p >= H]. With the lane constant u = 2 PKN z + 2 i and the per-(Z, edge)
// constants A = 2 PKN s' + hi, B = 2 PKN (s' - H) + 1 - hi (s' = shift mod H, hi = [shift >= H]; ctx d_pair_ab2) the
// packed kernel's address arithmetic (min(u + A, u + B) in 16-bit halves, partner byte a ^ 1) and its column
// immediates are unchanged: row_update_pk runs as is, with column stride CS.
//
// Per codeblock as in the plain kernel: HARQ skip, LLR load, layer count, CRC early stop, hard decisions and results.
// The slots of a workgroup share the iteration loop (a stopped codeblock's lanes idle through the layers and barriers
// until the other one stops). The host pairs codeblocks with the same Z, scaling, iteration limit and CRC mode
// (descs[2 w + i], an empty slot has nof_llr = 0). Measured (profiles/r5_decoder_pk2_scaling.txt): 2-7 % faster at six
// iterations, equal or slower under early stop - opt-in.
// ---------------------------------------------------------------------------------------------------------------------
/// Geometry of a PKN-codeblock workgroup (PKN = 2: two codeblocks of Z <= 192 fill three waves).
template <int PKN>
struct pk_geom {
  static constexpr int CS           = PKN * SOFT_COL_STRIDE;   ///< column stride of the interleaved image
  static constexpr int WAVES        = PKN * 192 / WAVE;        ///< most waves of a workgroup (Z = 384 slots)
  static constexpr int RED          = 2 * PKN * WAVES * 2;     ///< CRC reduction ints: [parity][slot][wave][acc, zero]
  static constexpr int SCRATCH_INTS = WAVES + RED + 2 * PKN;
};

/// Byte offset of position l (0 <= l < Z) of slot i within a column of the interleaved image.
template <int PKN>
__device__ __forceinline__ uint32_t pair_pos_pkn(uint32_t l, uint32_t H, uint32_t i)
{
  return ((l < H) ? 2u * PKN * l : 2u * PKN * (l - H) + 1u) + 2u * i;
}

/// LLRs of one codeblock -> its slot of the interleaved image (ldpc_decoder_impl.cpp:152; the plain kernel's load with
/// the slot's addresses), the punctured columns and every position beyond the input zeroed. Returns this thread's
/// index of the last non-zero LLR it saw (ldpc_decoder_impl.cpp:94), -1 if none.
template <int NCOL, int PKN>
__device__ __forceinline__ int load_llrs_pkn(int8_t* __restrict__ soft, const int8_t* __restrict__ llr,
                                             const dec_desc& d, uint32_t slot)
{
  const int      Z     = d.Z;
  const uint32_t H     = static_cast<uint32_t>(Z) / 2u;
  const int      n_llr = static_cast<int>(d.nof_llr);
  const uint32_t ncols = __umulhi(static_cast<uint32_t>(n_llr), d.div_magic);
  const uint32_t full  = ncols * static_cast<uint32_t>(Z);
  int            last  = -1;
  const uint32_t head  = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(llr)) & 15u;
  const uint4*   vecs  = reinterpret_cast<const uint4*>(llr - head);
  const int      nvec  = static_cast<int>((head + static_cast<uint32_t>(n_llr) + 15u) >> 4);
  constexpr int  BATCH = ((NCOL - 2) * 384 / 16 + 191) / 192;
  int            last_w = -1;
  uint4          last_v = make_uint4(0u, 0u, 0u, 0u);
  for (int w0 = threadIdx.x; w0 < nvec; w0 += BATCH * blockDim.x) {
    uint4 val[BATCH];
#pragma unroll
    for (int j = 0; j < BATCH; ++j) {
      const int w = w0 + j * blockDim.x;
      val[j]      = (w < nvec) ? vecs[w] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int j = 0; j < BATCH; ++j) {
      const int w = w0 + j * blockDim.x;
      if (w >= nvec) {
        continue;
      }
      const uint32_t i0 = static_cast<uint32_t>(16 * w) - head;
      const uint32_t c0 = __umulhi(i0, d.div_magic);
      const uint32_t l0 = i0 - c0 * static_cast<uint32_t>(Z);
      const bool short_path = (16u * static_cast<uint32_t>(w) >= head) && (i0 + 16u <= full) &&
                              (l0 + 16u <= static_cast<uint32_t>(Z));
      if (short_path) {
        // Consecutive positions are 2 PKN bytes apart; a byte past the half boundary moves by 1 - 2 PKN H.
        int8_t*        dst   = soft + (c0 + 2) * pk_geom<PKN>::CS + pair_pos_pkn<PKN>(l0, H, slot);
        const uint32_t cross = (l0 < H && l0 + 16u > H) ? (0xffffu << (H - l0)) : 0u;
        const int      adj   = 1 - 2 * PKN * static_cast<int>(H);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t word = (q == 0) ? val[j].x : (q == 1) ? val[j].y : (q == 2) ? val[j].z : val[j].w;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int kk = 4 * q + k;
            const int mv = static_cast<int>((cross >> kk) & 1u) * adj;
            dst[2 * PKN * kk + mv] = static_cast<int8_t>(clamp_i(static_cast<int8_t>(word >> (8 * k)), -64, 64));
          }
        }
        if ((val[j].x | val[j].y | val[j].z | val[j].w) != 0u) {
          last_w = w;
          last_v = val[j];
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t word = (q == 0) ? val[j].x : (q == 1) ? val[j].y : (q == 2) ? val[j].z : val[j].w;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t i = i0 + static_cast<uint32_t>(4 * q + k);
            if (i < static_cast<uint32_t>(n_llr)) {
              int v = static_cast<int8_t>(word >> (8 * k));
              last  = (v != 0) ? static_cast<int>(i) : last;
              v     = (i < full) ? clamp_i(v, -64, 64) : clamp_i(v, -SOFT_INF, SOFT_INF);
              const uint32_t cq = __umulhi(i, d.div_magic);
              soft[(cq + 2) * pk_geom<PKN>::CS + pair_pos_pkn<PKN>(i - cq * static_cast<uint32_t>(Z), H, slot)] = static_cast<int8_t>(v);
            }
          }
        }
      }
    }
  }
  if (last_w >= 0) {
    const uint32_t words[4] = {last_v.x, last_v.y, last_v.z, last_v.w};
    int            hb       = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      hb = (words[q] != 0u) ? 4 * q + (31 - __clz(static_cast<int>(words[q]))) / 8 : hb;
    }
    const int i = 16 * last_w - static_cast<int>(head) + hb;
    last        = i > last ? i : last;
  }
  // Punctured columns 0, 1 and every position beyond the input: threads [0, H) take position pair z.
  const uint32_t z = threadIdx.x;
  if (z < H) {
    auto* soft16 = reinterpret_cast<uint16_t*>(soft);
    const uint32_t pz = PKN * z + slot;  // 16-bit index of pair z within a column
    soft16[(0 * pk_geom<PKN>::CS) / 2 + pz] = 0;
    soft16[(1 * pk_geom<PKN>::CS) / 2 + pz] = 0;
    int c = 2 + static_cast<int>(ncols);
    if (static_cast<uint32_t>(n_llr) > full) {
      const uint32_t rem = static_cast<uint32_t>(n_llr) - full;
      if (z >= rem) {
        soft[c * pk_geom<PKN>::CS + 2 * pz] = 0;
      }
      if (z + H >= rem) {
        soft[c * pk_geom<PKN>::CS + 2 * pz + 1] = 0;
      }
      ++c;
    }
    for (; c < NCOL; ++c) {
      soft16[(c * pk_geom<PKN>::CS) / 2 + pz] = 0;
    }
  }
  return last;
}

/// Hard decisions of one slot's K*Z systematic bits, written by the slot's H lanes (lane z: bytes z, z + H, ...).
template <int PKN>
__device__ __forceinline__ void write_hard_bits_pkn(const int8_t* __restrict__ soft, uint8_t* __restrict__ out,
                                                    int nbits, int Z, uint32_t magic, uint32_t slot, uint32_t z)
{
  const uint32_t H      = static_cast<uint32_t>(Z) / 2u;
  const int      nbytes = (nbits + 7) / 8;
  for (int b = static_cast<int>(z); b < nbytes; b += static_cast<int>(H)) {
    uint32_t byte = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = 8 * b + k;
      if (i < nbits) {
        const uint32_t col = __umulhi(static_cast<uint32_t>(i), magic);
        const uint32_t l   = static_cast<uint32_t>(i) - col * static_cast<uint32_t>(Z);
        byte |= static_cast<uint32_t>(soft[col * pk_geom<PKN>::CS + pair_pos_pkn<PKN>(l, H, slot)] <= 0) << (7 - k);
      }
    }
    out[b] = static_cast<uint8_t>(byte);
  }
}

/// FUSE (as the one-codeblock kernel's): slot i's first transmission is dematched by the workgroup from the codeword
/// LLRs (llrs + dms[PKN w + i].llr_offset) into its slot of the image and into its HARQ soft buffer (harq +
/// harq_offset, or llr_cbs[cb]); the image is zeroed first. Returns this thread's last non-zero input position.
template <int NCOL, int PKN>
__device__ __forceinline__ int load_fused_pkn(int8_t* __restrict__ soft, const int8_t* __restrict__ llrs,
                                              const dec_desc& d, const dm_desc& dm, int8_t* __restrict__ hb,
                                              uint32_t slot)
{
  const int      Z     = d.Z;
  const uint32_t H     = static_cast<uint32_t>(Z) / 2u;
  const int      n_llr = static_cast<int>(d.nof_llr);
  const uint32_t full  = __umulhi(static_cast<uint32_t>(n_llr), d.div_magic) * static_cast<uint32_t>(Z);
  const int      E = static_cast<int>(dm.E), Qm = dm.Qm, R = E / Qm;
  const int      Fl = dm.nof_filler, ninfo = static_cast<int>(dm.nsys) - Fl, Nh = static_cast<int>(dm.N);
  const int8_t*  in   = llrs + dm.llr_offset;
  int            last = -1;
  // The one-codeblock kernel's soft_put / put (ldpc_decoder_impl.cpp:152 clamps, :94 trailing-zero trim) at the slot's
  // interleaved addresses.
  auto soft_put = [&](int k, int v) {
    if (static_cast<uint32_t>(k) < static_cast<uint32_t>(n_llr)) {
      last              = (v != 0 && k > last) ? k : last;
      const uint32_t cq = __umulhi(static_cast<uint32_t>(k), d.div_magic);
      const int      cv = (static_cast<uint32_t>(k) < full) ? clamp_i(v, -64, 64) : clamp_i(v, -SOFT_INF, SOFT_INF);
      soft[(cq + 2) * pk_geom<PKN>::CS + pair_pos_pkn<PKN>(static_cast<uint32_t>(k) - cq * static_cast<uint32_t>(Z), H,
                                                        slot)] = static_cast<int8_t>(cv);
    }
  };
  auto put = [&](int k, int v) {
    hb[k] = static_cast<int8_t>(v);
    soft_put(k, v);
  };
  const bool q8   = Qm == 8 && ((dm.llr_offset & 7u) == 0u);
  const bool q8x4 = q8 &&
                    ((R | ninfo | Fl | static_cast<int>(reinterpret_cast<uintptr_t>(hb))) & 3) == 0;
  if (q8x4) {
    for (int r0 = 4 * static_cast<int>(threadIdx.x); r0 < R; r0 += 4 * static_cast<int>(blockDim.x)) {
      uint2 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = *reinterpret_cast<const uint2*>(in + 8 * (r0 + q));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          w |= ((((j < 4) ? v[q].x : v[q].y) >> (8 * (j & 3))) & 0xffu) << (8 * q);
        }
        const int n = j * R + r0;
        const int k = n < ninfo ? n : n + Fl;
        *reinterpret_cast<uint32_t*>(hb + k) = w;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          soft_put(k + q, static_cast<int8_t>(w >> (8 * q)));
        }
      }
    }
  } else {
    for (int r = threadIdx.x; r < R; r += blockDim.x) {
      int8_t sym[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sym[j] = (j < Qm) ? in[r * Qm + j] : 0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < Qm) {
          const int n = j * R + r;
          put(n < ninfo ? n : n + Fl, sym[j]);
        }
      }
    }
  }
  // Fillers: +infinity (ldpc_rate_dematcher_impl.cpp:172); the unreached tail [E + F, N) of the HARQ buffer zeroed.
  for (int k = ninfo + static_cast<int>(threadIdx.x); k < ninfo + Fl; k += blockDim.x) {
    put(k, 127);
  }
  {
    const int t0 = E + Fl;  // 16-byte stores between the unaligned head and tail bytes
    const int a0 = min(Nh, t0 + static_cast<int>((16u - (reinterpret_cast<uintptr_t>(hb + t0) & 15u)) & 15u));
    const int nv = (Nh - a0) / 16;
    const int a1 = a0 + 16 * nv;
    if (static_cast<int>(threadIdx.x) < a0 - t0) {
      hb[t0 + static_cast<int>(threadIdx.x)] = 0;
    }
    uint4* z16 = reinterpret_cast<uint4*>(hb + a0);
    for (int q = threadIdx.x; q < nv; q += blockDim.x) {
      z16[q] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (static_cast<int>(threadIdx.x) < Nh - a1) {
      hb[a1 + static_cast<int>(threadIdx.x)] = 0;
    }
  }
  return last;
}

template <int BG, int MODE, int MAXL, int PKN, bool FUSE>
__global__ __launch_bounds__(64 * pk_geom<PKN>::WAVES, (MAXL > 8 ? 4 : PK_MIN_BLOCKS_8)) void ldpc_decode_pairs_kernel(
    const dec_desc* __restrict__ descs,
    const int8_t* __restrict__ llrs,
    uint8_t* __restrict__ out,
    int32_t* __restrict__ results,
    const uint32_t* __restrict__ ab_table,
    const uint32_t* __restrict__ crc_tables,
    uint8_t* __restrict__ cb_crc_ok,
    int8_t* const* __restrict__ llr_cbs,
    const dm_desc* __restrict__ dms,
    int8_t* __restrict__ harq)
{
  using G = bg_t<BG>;
  static_assert(MAXL >= 4 && MAXL <= 16, "PKN: 8- and 16-layer classes (the 16-bit pair addresses and the LDS image)");
  constexpr int NCOL = G::K + MAXL;
  __shared__ __attribute__((aligned(16))) int8_t smem[NCOL * pk_geom<PKN>::CS + pk_geom<PKN>::SCRATCH_INTS * sizeof(int)];
  int8_t* soft  = smem;
  int*    wlast = reinterpret_cast<int*>(smem + NCOL * pk_geom<PKN>::CS);  // [wave]: last non-zero LLR of the slot being loaded
  int*    red   = wlast + pk_geom<PKN>::WAVES;                              // [parity][slot][wave][acc, zero]
  int*    cbi   = red + pk_geom<PKN>::RED;                                  // [slot][layers, running]

  const dec_desc* wd = descs + static_cast<size_t>(blockIdx.x) * PKN;
  // Workgroup-uniform parameters from slot 0 (the host groups codeblocks that share them).
  const dec_desc d0 = wd[0];
  const int      Z  = d0.Z;
  const uint32_t H  = static_cast<uint32_t>(Z) / 2u;
  const auto     ab = (const_u32_ptr)(uintptr_t)(ab_table + static_cast<uint32_t>(d0.zpos) * G::NE);
  asm volatile("" ::"s"(llrs), "s"(out), "s"(results), "s"(crc_tables), "s"(cb_crc_ok), "s"(blockDim.x));
  constexpr int AB_BYTES = G::NE * 4;
  constexpr int AB_LINES = (AB_BYTES - 4) / 64 + 2;
  uint32_t      pf[AB_LINES];
  static_for<AB_LINES>([&](auto L) {
    constexpr int l = decltype(L)::value;
    scalar_touch<(l * 64 < AB_BYTES - 4) ? l * 64 : AB_BYTES - 4>(pf[l], ab);
  });
  int cnt = 1;
#pragma unroll
  for (int i = 1; i < PKN; ++i) {
    cnt += (wd[i].nof_llr != 0u) ? 1 : 0;
  }
  const int      wave   = threadIdx.x / WAVE;
  const int      nwaves = blockDim.x / WAVE;
  const int      lane   = threadIdx.x % WAVE;
  const uint32_t slot   = threadIdx.x / H;
  const uint32_t z      = threadIdx.x - slot * H;
  const bool     in_cb  = slot < static_cast<uint32_t>(cnt);
  const int      msg_len = G::K * Z;
  const bool     use_crc = d0.crc_table != NO_CRC_TABLE;
  const bool     early   = (d0.flags & DEC_FLAG_EARLY_STOP) != 0;

  if constexpr (FUSE) {
    // The fused slots write only their input positions: the whole image starts at zero.
    uint4* s16 = reinterpret_cast<uint4*>(soft);
    for (int q = threadIdx.x; q < NCOL * pk_geom<PKN>::CS / 16; q += blockDim.x) {
      s16[q] = make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
  }
  // ---- per slot: HARQ skip (pusch_decoder_impl.cpp:300), LLR load, input length, layer count ----
  for (int i = 0; i < cnt; ++i) {
    const dec_desc d       = wd[i];
    int            layers  = 0;
    int            running = 0;
    if (!FUSE && cb_crc_ok != nullptr && cb_crc_ok[d.cb_index] != 0) {
      if (threadIdx.x == 0) {
        results[d.cb_index] = 0;
      }
    } else {
      int last;
      if constexpr (FUSE) {
        // New data invalidates the codeblock CRC flag of the HARQ context (pusch_decoder_impl.cpp:132).
        if (cb_crc_ok != nullptr && threadIdx.x == 0) {
          cb_crc_ok[d.cb_index] = 0;
        }
        const dm_desc dm = dms[static_cast<size_t>(blockIdx.x) * PKN + i];
        int8_t*       hb = (llr_cbs != nullptr) ? llr_cbs[d.cb_index] : harq + dm.harq_offset;
        last = load_fused_pkn<NCOL, PKN>(soft, llrs, d, dm, hb, static_cast<uint32_t>(i));
      } else {
        last = load_llrs_pkn<NCOL, PKN>(soft, (llr_cbs != nullptr) ? llr_cbs[d.cb_index] : llrs + d.llr_offset, d,
                                        static_cast<uint32_t>(i));
      }
      last     = wave_max(last);
      if (lane == 0) {
        wlast[wave] = last;
      }
      __syncthreads();
      int input_size = wlast[0];
      for (int w = 1; w < nwaves; ++w) {
        input_size = wlast[w] > input_size ? wlast[w] : input_size;
      }
      input_size += 1;
      __syncthreads();  // wlast is reused by the next slot
      if (input_size < msg_len) {
        // Not enough LLRs: no decoding; when the CRC is not the decoder's (no CRC, or checked by the caller after the
        // last iteration: no early stop, pusch_codeblock_decoder passes no calculator) the output is all ones
        // (ldpc_decoder_impl.cpp:95).
        if (!use_crc || (d0.flags & DEC_FLAG_EARLY_STOP) == 0) {
          for (int b = threadIdx.x; b < (msg_len + 7) / 8; b += blockDim.x) {
            out[d.out_offset + b] = 0xff;
          }
        }
        if (threadIdx.x == 0) {
          results[d.cb_index] = -1;
        }
      } else {
        int cb_len = input_size + 2 * Z;
        cb_len     = cb_len > msg_len + 4 * Z ? cb_len : msg_len + 4 * Z;
        layers     = static_cast<int>(__umulhi(static_cast<uint32_t>(cb_len + Z - 1), d.div_magic)) - G::K;
        if (layers > MAXL) {
          // The host bound is derived from the same input length: cannot happen; fail loudly.
          if (threadIdx.x == 0) {
            results[d.cb_index] = -2;
          }
          layers = 0;
        } else {
          running = 1;
        }
      }
    }
    if (threadIdx.x == 0) {
      cbi[2 * i]     = layers;
      cbi[2 * i + 1] = running;
    }
  }
  __syncthreads();
  static_for<AB_LINES>([&](auto L) { keep_sgpr(pf[decltype(L)::value]); });
  int nl_max = 0;
  for (int i = 0; i < cnt; ++i) {
    nl_max = (cbi[2 * i + 1] != 0 && cbi[2 * i] > nl_max) ? cbi[2 * i] : nl_max;
  }
  nl_max            = __builtin_amdgcn_readfirstlane(nl_max);
  // Per-lane loop state in one VGPR: the lane constant u = 2 PKN z + 2 slot (bits 0-15; z and slot are recovered from
  // it) and the lane's layer count while its codeblock runs (bits 16+; 0 once it stopped, or for lanes without a
  // codeblock): "layer m runs" is one compare, lane >= (m + 1) << 16.
  uint32_t lane_st = (2u * PKN * z + 2u * slot) |
                     (static_cast<uint32_t>((in_cb && cbi[2 * slot + 1] != 0) ? cbi[2 * slot] : 0) << 16);
  int      running = __syncthreads_or(lane_st >= (1u << 16) ? 1 : 0);

  scale_t sc;
  sc.hi = uu(static_cast<int>(d0.sf16 >> 8));
  sc.lo = uu(static_cast<int>(d0.sf16 & 255u));
  sc.sf = d0.sf;
  uint32_t magw[MAXL], sgw[MAXL];
  uint32_t hiw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int m = 0; m < MAXL; ++m) {
    magw[m] = 0;
    sgw[m]  = 0;
  }
  const int max_iter = d0.max_iter;
  int       it       = 0;
  for (; it < max_iter && running != 0; ++it) {
    int           nl   = nl_max;
    uint32_t      z2x2 = 0x00010001u * (lane_st & 0xffffu);
    const_u32_ptr abi  = ab;
    asm volatile("" : "+s"(nl));
    asm volatile("" : "+v"(z2x2));
    asm volatile("" : "+s"(abi));
    static_for<MAXL>([&](auto Mi) {
      constexpr int m = decltype(Mi)::value;
      if (m < nl) {
        if (lane_st >= static_cast<uint32_t>(m + 1) << 16) {
          __builtin_amdgcn_sched_barrier(0);
          row_update_pk<BG, MODE, m, (MAXL <= PK_KEEP_ADDR_MAXL), pk_geom<PKN>::CS>(soft, abi, z2x2, sc, magw[m], sgw[m],
                                                                              hiw[m & 3]);
          __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
      }
    });

    // CRC after every iteration with early stop (ldpc_decoder_impl.cpp:133), else after the last one; per slot.
    if (use_crc && (early || it == max_iter - 1)) {
      uint32_t       acc = 0, zero = 0;
      const bool     run = lane_st >= (1u << 16);
      const uint32_t ub  = lane_st & 0xffffu;
      const uint32_t lz = ub / (2u * PKN), ls = (ub / 2u) % PKN;  // z, slot
      if (run) {
        const dec_desc* md       = wd + ls;
        const uint32_t* table    = crc_tables + md->crc_table;
        uint32_t        zz = lz, ZZ = static_cast<uint32_t>(Z), HH = H;
        asm volatile("" : "+v"(zz));
        asm volatile("" : "+s"(ZZ), "+s"(HH));
        uint32_t      ia   = zz;
        const int8_t* scol = soft + ub;
        static_for<G::K>([&](auto Ci) {
          constexpr int  c  = decltype(Ci)::value;
          const uint32_t ib = ia + HH;
          const int      sa = scol[c * pk_geom<PKN>::CS];
          const int      sb = scol[c * pk_geom<PKN>::CS + 1];
          zero |= static_cast<uint32_t>(sa == 0) | static_cast<uint32_t>(sb == 0);
          const uint32_t ta = table[ia];  // zero tail past the message, as above
          const uint32_t tb = table[ib];
          acc ^= (sa <= 0) ? ta : 0u;
          acc ^= (sb <= 0) ? tb : 0u;
          ia += ZZ;
          if constexpr (c % CRC_CHUNK == CRC_CHUNK - 1) {
            __builtin_amdgcn_sched_barrier(0);
          }
        });
      }
      int* r = red + (it & 1) * (PKN * pk_geom<PKN>::WAVES * 2);
      static_for<PKN>([&](auto J) {
        constexpr uint32_t j  = decltype(J)::value;
        const bool         mine = run && ls == j;
        const uint32_t     a    = wave_xor(mine ? acc : 0u);
        const uint32_t     zr   = (__ballot(mine && zero != 0) != 0) ? 1u : 0u;
        if (lane == 0) {
          r[(j * pk_geom<PKN>::WAVES + wave) * 2]     = static_cast<int>(a);
          r[(j * pk_geom<PKN>::WAVES + wave) * 2 + 1] = static_cast<int>(zr);
        }
      });
      __syncthreads();
      if (run) {
        uint32_t tacc = 0, tzero = 0;
        for (int w = 0; w < nwaves; ++w) {
          tacc ^= static_cast<uint32_t>(r[(ls * pk_geom<PKN>::WAVES + w) * 2]);
          tzero |= static_cast<uint32_t>(r[(ls * pk_geom<PKN>::WAVES + w) * 2 + 1]);
        }
        if ((tzero == 0 || !early) && tacc == 0) {
          const dec_desc* md = wd + ls;
          write_hard_bits_pkn<PKN>(soft, out + md->out_offset, msg_len, Z, d0.div_magic, ls, lz);
          if (lz == 0) {
            results[md->cb_index] = it + 1;
            if (cb_crc_ok != nullptr) {
              cb_crc_ok[md->cb_index] = 1;
            }
          }
          lane_st = ub;
        }
      }
    }
    running = __syncthreads_or(lane_st >= (1u << 16) ? 1 : 0);
  }
  if (lane_st >= (1u << 16)) {
    const uint32_t  ub = lane_st & 0xffffu;
    const uint32_t  lz = ub / (2u * PKN), ls = (ub / 2u) % PKN;
    const dec_desc* md = wd + ls;
    write_hard_bits_pkn<PKN>(soft, out + md->out_offset, msg_len, Z, d0.div_magic, ls, lz);
    if (lz == 0) {
      results[md->cb_index] = -1;
    }
  }
}

} // namespace

#ifdef LDPC_DEC_PROFILE
int debug_read_decoder_profile_pk(uint64_t* dst, size_t n)
{
  const size_t max = static_cast<size_t>(LDPC_DEC_PROF_CBS) * LDPC_DEC_PROF_SLOTS;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_dec_prof_pk), (n < max ? n : max) * sizeof(uint64_t)) == hipSuccess
             ? 0
             : -1;
}
#endif

void launch_ldpc_decode_pk(int             bg,
                           int             mode,
                           int             max_layers,
                           int             split,
                           const dec_desc* d_desc,
                           int             nof_cbs,
                           int             block_threads,
                           const int8_t*   d_llrs,
                           uint8_t*        d_out,
                           int32_t*        d_results,
                           const uint32_t* d_ab,
                           const uint32_t* d_crc_tables,
                           uint8_t*        d_cb_crc_ok,
                           const dm_desc*  d_dm,
                           int8_t*         d_harq,
                           hipStream_t     stream,
                           int8_t* const*  d_harq_cbs)
{
  if (nof_cbs <= 0) {
    return;
  }
  dim3 grid(nof_cbs), block(block_threads);
  const bool fuse = d_dm != nullptr;
#define SRSGPU_PK_LAUNCH1(BG_, MODE_, MAXL_, SPLIT_)                                                                   \
  (fuse ? ldpc_decode_pk_kernel<BG_, MODE_, MAXL_, SPLIT_, true><<<grid, block, 0, stream>>>(                          \
              d_desc, d_llrs, d_out, d_results, d_ab, d_crc_tables, d_cb_crc_ok, d_dm, d_harq, d_harq_cbs)            \
        : ldpc_decode_pk_kernel<BG_, MODE_, MAXL_, SPLIT_, false><<<grid, block, 0, stream>>>(                         \
              d_desc, d_llrs, d_out, d_results, d_ab, d_crc_tables, d_cb_crc_ok, nullptr, nullptr, d_harq_cbs))
#define SRSGPU_PK_LAUNCH(BG_, MODE_, MAXL_)                                                                            \
  (split == 2 ? SRSGPU_PK_LAUNCH1(BG_, MODE_, MAXL_, 2) : SRSGPU_PK_LAUNCH1(BG_, MODE_, MAXL_, 1))
  if (bg == 1) {
    if (max_layers <= 8) {
      mode == 1 ? SRSGPU_PK_LAUNCH(1, 1, 8) : SRSGPU_PK_LAUNCH(1, 0, 8);
    } else if (max_layers <= 16) {
      mode == 1 ? SRSGPU_PK_LAUNCH(1, 1, 16) : SRSGPU_PK_LAUNCH(1, 0, 16);
    } else {
      mode == 1 ? SRSGPU_PK_LAUNCH(1, 1, kBG1_M) : SRSGPU_PK_LAUNCH(1, 0, kBG1_M);
    }
  } else {
    if (max_layers <= 8) {
      mode == 1 ? SRSGPU_PK_LAUNCH(2, 1, 8) : SRSGPU_PK_LAUNCH(2, 0, 8);
    } else if (max_layers <= 16) {
      mode == 1 ? SRSGPU_PK_LAUNCH(2, 1, 16) : SRSGPU_PK_LAUNCH(2, 0, 16);
    } else {
      mode == 1 ? SRSGPU_PK_LAUNCH(2, 1, kBG2_M) : SRSGPU_PK_LAUNCH(2, 0, kBG2_M);
    }
  }
#undef SRSGPU_PK_LAUNCH
#undef SRSGPU_PK_LAUNCH1
}

void launch_ldpc_decode_pairs(int             bg,
                              int             mode,
                              int             max_layers,
                              const dec_desc* d_desc,
                              int             nof_groups,
                              int             block_threads,
                              const int8_t*   d_llrs,
                              uint8_t*        d_out,
                              int32_t*        d_results,
                              const uint32_t* d_ab2,
                              const uint32_t* d_crc_tables,
                              uint8_t*        d_cb_crc_ok,
                              hipStream_t     stream,
                              int8_t* const*  d_llr_cbs,
                              const dm_desc*  d_dm,
                              int8_t*         d_harq)
{
  if (nof_groups <= 0) {
    return;
  }
  dim3 grid(nof_groups), block(block_threads);
#define SRSGPU_PAIRS_LAUNCH1(BG_, MODE_, MAXL_, FUSE_)                                                                  \
  ldpc_decode_pairs_kernel<BG_, MODE_, MAXL_, 2, FUSE_><<<grid, block, 0, stream>>>(                                   \
      d_desc, d_llrs, d_out, d_results, d_ab2, d_crc_tables, d_cb_crc_ok, d_llr_cbs, d_dm, d_harq)
#define SRSGPU_PAIRS_LAUNCH(BG_, MODE_, MAXL_)                                                                         \
  (d_dm != nullptr ? SRSGPU_PAIRS_LAUNCH1(BG_, MODE_, MAXL_, true) : SRSGPU_PAIRS_LAUNCH1(BG_, MODE_, MAXL_, false))
  if (bg == 1) {
    if (max_layers <= 8) {
      mode == 1 ? SRSGPU_PAIRS_LAUNCH(1, 1, 8) : SRSGPU_PAIRS_LAUNCH(1, 0, 8);
    } else {
      mode == 1 ? SRSGPU_PAIRS_LAUNCH(1, 1, 16) : SRSGPU_PAIRS_LAUNCH(1, 0, 16);
    }
  } else {
    if (max_layers <= 8) {
      mode == 1 ? SRSGPU_PAIRS_LAUNCH(2, 1, 8) : SRSGPU_PAIRS_LAUNCH(2, 0, 8);
    } else {
      mode == 1 ? SRSGPU_PAIRS_LAUNCH(2, 1, 16) : SRSGPU_PAIRS_LAUNCH(2, 0, 16);
    }
  }
#undef SRSGPU_PAIRS_LAUNCH
#undef SRSGPU_PAIRS_LAUNCH1
}

} // namespace srsgpu
