// fi_softfp.h -- IEEE 754 binary16/32/64 arithmetic with the RISC-V
// conventions gem5 executes its F/D/Zfh instructions with (gem5 links
// SoftFloat 3 with the RISC-V specialization: ext/softfloat/specialize.h).
// Host and device code from one source: the engine's device interpreter uses
// it, and tests/test_softfp.py pins the host build of the same functions
// against the reference's own SoftFloat library (oracle/_ref) on random and
// edge operands in every rounding mode, flags included.
//
// Written from the IEEE 754-2008 rules plus the specialization's choices:
//   * every NaN result is the canonical NaN (defaultNaN*UI, specialize.h);
//     invalid is raised for signalling NaN operands and invalid operations
//   * tininess is detected after rounding (init_detectTininess), and the
//     underflow flag is raised only for tiny AND inexact results
//   * out-of-range float->int conversions return the saturated value, NaN
//     converting like +overflow (i32_fromNaN == i32_fromPosOverflow, ...)
//   * inf*0 + c raises invalid even when c is a quiet NaN (f*_mulAdd)
// Operands and results are raw bit patterns in the low bits of a uint64_t;
// flags accumulate into `fl` with the fflags bit order (NX UF OF DZ NV).
#pragma once
#ifndef FI_SF_HD
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define FI_SF_HD __host__ __device__ inline
#else
#define FI_SF_HD inline
#endif
#endif

namespace fi {
namespace sf {

typedef unsigned __int128 u128;

enum : uint32_t { FL_NX = 1, FL_UF = 2, FL_OF = 4, FL_DZ = 8, FL_NV = 16 };
enum : int { RNE = 0, RTZ = 1, RDN = 2, RUP = 3, RMM = 4 };

template <int EB, int MB> struct Fmt {
    static constexpr int eb = EB, mb = MB;
    static constexpr int emax_b = (1 << EB) - 1;                 // exponent field of inf / NaN
    static constexpr int bias = (1 << (EB - 1)) - 1;
    static constexpr uint64_t frac = (1ULL << MB) - 1;
    static constexpr uint64_t sign = 1ULL << (EB + MB);
    static constexpr uint64_t inf = (uint64_t)emax_b << MB;
    static constexpr uint64_t qnan = inf | (1ULL << (MB - 1));   // the canonical NaN
    static constexpr uint64_t maxf = inf - 1;                      // largest finite magnitude
};
typedef Fmt<5, 10> H;
typedef Fmt<8, 23> S;
typedef Fmt<11, 52> D;

FI_SF_HD int clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }

template <class F> FI_SF_HD bool is_nan(uint64_t a) { return (a & ~F::sign) > F::inf; }
template <class F> FI_SF_HD bool is_snan(uint64_t a) { return is_nan<F>(a) && !((a >> (F::mb - 1)) & 1); }
template <class F> FI_SF_HD bool is_inf(uint64_t a) { return (a & ~F::sign) == F::inf; }
template <class F> FI_SF_HD bool is_zero(uint64_t a) { return (a & ~F::sign) == 0; }

// right shift with the shifted-out bits ORed into bit 0 ("jamming")
FI_SF_HD uint64_t srj64(uint64_t x, int n) {
    if (n <= 0) return x;
    if (n >= 64) return x != 0;
    return (x >> n) | ((x << (64 - n)) != 0);
}
FI_SF_HD u128 srj128(u128 x, int n) {
    if (n <= 0) return x;
    if (n >= 128) return x != 0;
    return (x >> n) | (u128)((x << (128 - n)) != 0);
}

// A finite nonzero operand as sig * 2^(e - 62), sig normalised to [2^62, 2^63).
template <class F> FI_SF_HD void unpack(uint64_t a, int &e, uint64_t &sig) {
    const int ef = (int)((a >> F::mb) & F::emax_b);
    const uint64_t fr = a & F::frac;
    if (ef == 0) {   // subnormal
        const int t = 63 - clz64(fr);   // position of the leading one
        sig = fr << (62 - t);
        e = (1 - F::bias) - F::mb + t;
    } else {
        sig = (fr | (1ULL << F::mb)) << (62 - F::mb);
        e = ef - F::bias;
    }
}

// Should a magnitude whose dropped bits are rb (half = the weight of the
// first dropped bit) be rounded up?  m is the kept significand (its lsb
// breaks ties to even).
FI_SF_HD bool round_up(int rm, bool neg, uint64_t m, uint64_t rb, uint64_t half) {
    switch (rm) {
    case RNE: return rb > half || (rb == half && (m & 1));
    case RMM: return rb >= half;
    case RDN: return neg && rb != 0;
    case RUP: return !neg && rb != 0;
    default: return false;   // RTZ
    }
}

// Round sig * 2^(e - 62) (sig in [2^62, 2^63), sticky bits jammed into bit 0)
// to format F: overflow, tininess after rounding, subnormal results.
template <class F> FI_SF_HD uint64_t round_pack(bool neg, int e, uint64_t sig, int rm, uint32_t &fl) {
    constexpr int sh = 62 - F::mb;   // dropped bits below the p-bit significand
    constexpr uint64_t rmask = (1ULL << sh) - 1, half = 1ULL << (sh - 1);
    const uint64_t sgn = neg ? F::sign : 0;
    int eb = e + F::bias;   // biased exponent of the leading bit
    if (eb >= 1) {
        uint64_t m = sig >> sh;
        const uint64_t rb = sig & rmask;
        m += round_up(rm, neg, m, rb, half) ? 1 : 0;
        if (m >> (F::mb + 1)) { m >>= 1; eb++; }
        if (eb >= F::emax_b) {
            fl |= FL_OF | FL_NX;
            const bool to_inf = rm == RNE || rm == RMM || (rm == RDN && neg) || (rm == RUP && !neg);
            return sgn | (to_inf ? F::inf : F::maxf);
        }
        if (rb) fl |= FL_NX;
        return sgn | ((uint64_t)eb << F::mb) | (m & F::frac);
    }
    // below the normal range: tiny unless rounding at full precision carries
    // into the smallest normal exponent
    bool tiny = true;
    if (eb == 0) {
        const uint64_t m0 = sig >> sh;
        if ((m0 + (round_up(rm, neg, m0, sig & rmask, half) ? 1 : 0)) >> (F::mb + 1)) tiny = false;
    }
    const uint64_t s2 = srj64(sig, 1 - eb);
    uint64_t m = s2 >> sh;
    const uint64_t rb = s2 & rmask;
    m += round_up(rm, neg, m, rb, half) ? 1 : 0;   // may carry into the smallest normal (encodes itself)
    if (rb) fl |= tiny ? (FL_NX | FL_UF) : FL_NX;
    return sgn | m;
}

// NaN operands of an arithmetic operation: the canonical NaN, invalid if
// one of them signals (softfloat_propagateNaN*UI of the specialization)
template <class F> FI_SF_HD uint64_t nan2(uint64_t a, uint64_t b, uint32_t &fl) {
    if (is_snan<F>(a) || is_snan<F>(b)) fl |= FL_NV;
    return F::qnan;
}

template <class F> FI_SF_HD uint64_t add(uint64_t a, uint64_t b, int rm, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) return nan2<F>(a, b, fl);
    const bool sa = a & F::sign, sb = b & F::sign;
    if (is_inf<F>(a)) {
        if (is_inf<F>(b) && sa != sb) { fl |= FL_NV; return F::qnan; }
        return a;
    }
    if (is_inf<F>(b)) return b;
    const bool za = is_zero<F>(a), zb = is_zero<F>(b);
    if (za && zb) return sa == sb ? a : (rm == RDN ? F::sign : 0);
    if (za) return b;
    if (zb) return a;
    int ea, eb;
    uint64_t ma, mb;
    unpack<F>(a, ea, ma);
    unpack<F>(b, eb, mb);
    ma >>= 1; mb >>= 1;   // leading one at bit 61: room for the carry (low bits are zero)
    bool neg = sa;
    if (ea < eb || (ea == eb && ma < mb)) {
        const int te = ea; ea = eb; eb = te;
        const uint64_t tm = ma; ma = mb; mb = tm;
        neg = sb;
    }
    mb = srj64(mb, ea - eb);
    const uint64_t m = sa == sb ? ma + mb : ma - mb;
    if (m == 0) return rm == RDN ? F::sign : 0;   // exact cancellation
    const int lz = clz64(m);                      // >= 1
    return round_pack<F>(neg, ea + 1 - (lz - 1), m << (lz - 1), rm, fl);
}

template <class F> FI_SF_HD uint64_t sub(uint64_t a, uint64_t b, int rm, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) return nan2<F>(a, b, fl);
    return add<F>(a, b ^ F::sign, rm, fl);
}

// 128-bit product / sum -> 64-bit significand with the leading one at bit 62
// (sticky jammed); returns the shift applied (value = x * 2^k == m * 2^(k + shift - 62 + ...))
FI_SF_HD uint64_t norm128(u128 x, int &lead) {
    const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
    lead = hi ? 127 - clz64(hi) : 63 - clz64(lo);
    if (lead > 62) return (uint64_t)srj128(x, lead - 62);
    return (uint64_t)x << (62 - lead);
}

template <class F> FI_SF_HD uint64_t mul(uint64_t a, uint64_t b, int rm, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) return nan2<F>(a, b, fl);
    const bool neg = ((a ^ b) & F::sign) != 0;
    const uint64_t sgn = neg ? F::sign : 0;
    if (is_inf<F>(a) || is_inf<F>(b)) {
        if (is_zero<F>(a) || is_zero<F>(b)) { fl |= FL_NV; return F::qnan; }
        return sgn | F::inf;
    }
    if (is_zero<F>(a) || is_zero<F>(b)) return sgn;
    int ea, eb, lead;
    uint64_t ma, mb;
    unpack<F>(a, ea, ma);
    unpack<F>(b, eb, mb);
    const uint64_t m = norm128((u128)ma * mb, lead);   // product = x * 2^(ea + eb - 124)
    return round_pack<F>(neg, ea + eb + lead - 124, m, rm, fl);
}

template <class F> FI_SF_HD uint64_t div(uint64_t a, uint64_t b, int rm, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) return nan2<F>(a, b, fl);
    const bool neg = ((a ^ b) & F::sign) != 0;
    const uint64_t sgn = neg ? F::sign : 0;
    if (is_inf<F>(a)) {
        if (is_inf<F>(b)) { fl |= FL_NV; return F::qnan; }
        return sgn | F::inf;
    }
    if (is_inf<F>(b)) return sgn;
    if (is_zero<F>(b)) {
        if (is_zero<F>(a)) { fl |= FL_NV; return F::qnan; }
        fl |= FL_DZ;
        return sgn | F::inf;
    }
    if (is_zero<F>(a)) return sgn;
    int ea, eb;
    uint64_t ma, mb;
    unpack<F>(a, ea, ma);
    unpack<F>(b, eb, mb);
    int e = ea - eb;
    uint64_t r = ma;
    if (ma < mb) { r = ma << 1; e--; }   // quotient in [1, 2)
    uint64_t q = 0;
    for (int i = 0; i < 63; i++) {        // 63 quotient bits: the leading one lands on bit 62
        q <<= 1;
        if (r >= mb) { r -= mb; q |= 1; }
        r <<= 1;
    }
    return round_pack<F>(neg, e, q | (r != 0), rm, fl);
}

template <class F> FI_SF_HD uint64_t sqrt(uint64_t a, int rm, uint32_t &fl) {
    if (is_nan<F>(a)) return nan2<F>(a, a, fl);
    if (is_zero<F>(a)) return a;
    if (a & F::sign) { fl |= FL_NV; return F::qnan; }
    if (is_inf<F>(a)) return a;
    int e;
    uint64_t m;
    unpack<F>(a, e, m);
    // sqrt(m * 2^(e - 62)) = isqrt(m << (62 + odd)) * 2^((e - odd) / 2 - 62)
    const int odd = e & 1;
    u128 rad = (u128)m << (62 + odd);
    u128 res = 0, bit = (u128)1 << 126;
    while (bit > rad) bit >>= 2;
    while (bit) {
        if (rad >= res + bit) { rad -= res + bit; res = (res >> 1) + bit; }
        else res >>= 1;
        bit >>= 2;
    }
    return round_pack<F>(false, (e - odd) / 2, (uint64_t)res | (rad != 0), rm, fl);
}

// a * b + c, rounded once (f*_mulAdd); negations are applied by the caller
template <class F> FI_SF_HD uint64_t fma(uint64_t a, uint64_t b, uint64_t c, int rm, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) {
        if (is_snan<F>(a) || is_snan<F>(b) || is_snan<F>(c)) fl |= FL_NV;
        return F::qnan;
    }
    const bool sp = ((a ^ b) & F::sign) != 0, sc = (c & F::sign) != 0;
    const bool ia = is_inf<F>(a), ib = is_inf<F>(b), za = is_zero<F>(a), zb = is_zero<F>(b);
    if ((ia && zb) || (za && ib)) { fl |= FL_NV; return F::qnan; }
    if (is_nan<F>(c)) return nan2<F>(c, c, fl);
    if (ia || ib) {
        if (is_inf<F>(c) && sc != sp) { fl |= FL_NV; return F::qnan; }
        return (sp ? F::sign : 0) | F::inf;
    }
    if (is_inf<F>(c)) return c;
    if (za || zb) {
        if (is_zero<F>(c)) return sp == sc ? (sp ? F::sign : 0) : (rm == RDN ? F::sign : 0);
        return c;
    }
    int ea, eb, lead;
    uint64_t ma, mb;
    unpack<F>(a, ea, ma);
    unpack<F>(b, eb, mb);
    u128 P = (u128)ma * mb;   // P * 2^(ep - 124)
    int ep = ea + eb;
    if (is_zero<F>(c)) {
        const uint64_t m = norm128(P, lead);
        return round_pack<F>(sp, ep + lead - 124, m, rm, fl);
    }
    int ec;
    uint64_t mc;
    unpack<F>(c, ec, mc);
    u128 Cc = (u128)mc << 62;   // Cc * 2^(ec - 124)
    int e;
    if (ep >= ec) { Cc = srj128(Cc, ep - ec); e = ep; }
    else { P = srj128(P, ec - ep); e = ec; }
    u128 Sm;
    bool neg;
    if (sp == sc) { Sm = P + Cc; neg = sp; }
    else if (P >= Cc) { Sm = P - Cc; neg = sp; }
    else { Sm = Cc - P; neg = sc; }
    if (Sm == 0) return rm == RDN ? F::sign : 0;
    const uint64_t m = norm128(Sm, lead);
    return round_pack<F>(neg, e + lead - 124, m, rm, fl);
}

// comparisons: eq is quiet, lt/le signal on any NaN; *_quiet signal on sNaN only
template <class F> FI_SF_HD bool eq(uint64_t a, uint64_t b, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) {
        if (is_snan<F>(a) || is_snan<F>(b)) fl |= FL_NV;
        return false;
    }
    return a == b || ((a | b) & ~F::sign) == 0;
}
template <class F> FI_SF_HD bool lt(uint64_t a, uint64_t b, bool quiet, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) {
        if (!quiet || is_snan<F>(a) || is_snan<F>(b)) fl |= FL_NV;
        return false;
    }
    const bool sa = a & F::sign, sb = b & F::sign;
    if (sa != sb) return sa && ((a | b) & ~F::sign) != 0;
    return a != b && (sa ^ (a < b));
}
template <class F> FI_SF_HD bool le(uint64_t a, uint64_t b, bool quiet, uint32_t &fl) {
    if (is_nan<F>(a) || is_nan<F>(b)) {
        if (!quiet || is_snan<F>(a) || is_snan<F>(b)) fl |= FL_NV;
        return false;
    }
    const bool sa = a & F::sign, sb = b & F::sign;
    if (sa != sb) return sa || ((a | b) & ~F::sign) == 0;
    return a == b || (sa ^ (a < b));
}

// float -> integer (exact = true: inexact results raise NX).  kind: 0 i32,
// 1 u32, 2 i64, 3 u64; the result is the two's complement bit pattern.
template <class F> FI_SF_HD uint64_t to_int(uint64_t a, int kind, int rm, uint32_t &fl) {
    const uint64_t pos_ovf = kind == 0 ? 0x7FFFFFFFULL : kind == 1 ? 0xFFFFFFFFULL : kind == 2 ? 0x7FFFFFFFFFFFFFFFULL : ~0ULL;
    const uint64_t neg_ovf = kind == 0 ? 0xFFFFFFFF80000000ULL : kind == 2 ? 0x8000000000000000ULL : 0ULL;
    const bool neg = (a & F::sign) != 0;
    if (is_nan<F>(a)) { fl |= FL_NV; return pos_ovf; }
    if (is_inf<F>(a)) { fl |= FL_NV; return neg ? neg_ovf : pos_ovf; }
    if (is_zero<F>(a)) return 0;
    int e;
    uint64_t m;
    unpack<F>(a, e, m);
    if (e >= 64) { fl |= FL_NV; return neg ? neg_ovf : pos_ovf; }
    uint64_t ip, fr;
    if (e >= 62) { ip = m << (e - 62); fr = 0; }
    else {
        const int sh = 62 - e;   // >= 1
        if (sh >= 128) { ip = 0; fr = 1; }
        else {
            const u128 x = srj128((u128)m << 64, sh);
            ip = (uint64_t)(x >> 64);
            fr = (uint64_t)x;
        }
    }
    if (round_up(rm, neg, ip, fr, 1ULL << 63)) ip++;
    bool bad;
    switch (kind) {
    case 0: bad = neg ? ip > 0x80000000ULL : ip > 0x7FFFFFFFULL; break;
    case 1: bad = neg ? ip != 0 : ip > 0xFFFFFFFFULL; break;
    case 2: bad = neg ? ip > 0x8000000000000000ULL : ip > 0x7FFFFFFFFFFFFFFFULL; break;
    default: bad = neg && ip != 0; break;
    }
    if (bad) { fl |= FL_NV; return neg ? neg_ovf : pos_ovf; }
    if (fr) fl |= FL_NX;
    return neg ? (uint64_t)(0 - ip) : ip;
}

// integer -> float; kind as above (the operand is the register value)
template <class F> FI_SF_HD uint64_t from_int(uint64_t x, int kind, int rm, uint32_t &fl) {
    bool neg = false;
    uint64_t mag;
    switch (kind) {
    case 0: { const int64_t v = (int32_t)(uint32_t)x; neg = v < 0; mag = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v; break; }
    case 1: mag = (uint32_t)x; break;
    case 2: { const int64_t v = (int64_t)x; neg = v < 0; mag = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v; break; }
    default: mag = x; break;
    }
    if (!mag) return 0;
    const int t = 63 - clz64(mag);
    const uint64_t m = t > 62 ? srj64(mag, t - 62) : mag << (62 - t);
    return round_pack<F>(neg, t, m, rm, fl);
}

// format conversion (widening is exact; narrowing rounds)
template <class FS, class FD> FI_SF_HD uint64_t convert(uint64_t a, int rm, uint32_t &fl) {
    const bool neg = (a & FS::sign) != 0;
    if (is_nan<FS>(a)) { if (is_snan<FS>(a)) fl |= FL_NV; return FD::qnan; }
    if (is_inf<FS>(a)) return (neg ? FD::sign : 0) | FD::inf;
    if (is_zero<FS>(a)) return neg ? FD::sign : 0;
    int e;
    uint64_t m;
    unpack<FS>(a, e, m);
    return round_pack<FD>(neg, e, m, rm, fl);
}

// roundToInt (Zfa fround / froundnx): the integral value nearest to a in
// rounding mode rm, in a's format; exact = raise inexact when it differs.
// NaN -> canonical NaN (invalid if signalling); zeros, infinities and values
// of magnitude >= 2^mb are returned as they are; a zero result keeps a's sign.
template <class F> FI_SF_HD uint64_t rint(uint64_t a, int rm, bool exact, uint32_t &fl) {
    if (is_nan<F>(a)) { if (is_snan<F>(a)) fl |= FL_NV; return F::qnan; }
    if (is_inf<F>(a) || is_zero<F>(a)) return a;
    const bool neg = (a & F::sign) != 0;
    int e;
    uint64_t m;
    unpack<F>(a, e, m);
    if (e >= F::mb) return a;
    const int sh = 62 - e;   // > 62 - mb
    uint64_t ip, fr;
    if (sh >= 128) { ip = 0; fr = 1; }
    else {
        const u128 x = srj128((u128)m << 64, sh);
        ip = (uint64_t)(x >> 64);
        fr = (uint64_t)x;
    }
    if (round_up(rm, neg, ip, fr, 1ULL << 63)) ip++;
    if (fr && exact) fl |= FL_NX;
    const uint64_t sgn = neg ? F::sign : 0;
    if (!ip) return sgn;
    const int t = 63 - clz64(ip);   // <= mb: exactly representable
    return sgn | ((uint64_t)(t + F::bias) << F::mb) | ((ip << (F::mb - t)) & F::frac);
}

// fli (Zfa; decoder.isa:3550-3700): entry i of the Zfa constant list in
// format F: -1, the minimum positive normal, 2^-16, 2^-15, 2^-8, 2^-7, 2^-4,
// 2^-3, then n/16, n/8, n/4 (n = 4..7), 2, 2.5, 3, 4, 8, 16, 2^7, 2^8, 2^15,
// 2^16, +inf, NaN; out-of-range values are +inf, tiny ones subnormal.
template <class F> FI_SF_HD uint64_t fli(uint32_t i) {
    if (i == 30) return F::inf;
    if (i == 31) return F::qnan;
    if (i == 1) return 1ULL << F::mb;
    uint64_t num = 1;
    int e = 0;
    if (i >= 2 && i < 8) { const int t = (int)(i - 2); e = t < 2 ? -16 + t : t < 4 ? -8 + (t - 2) : -4 + (t - 4); }
    else if (i >= 8 && i < 22) { num = 4 + (i - 8) % 4; e = (int)((i - 8) / 4) - 4; }
    else if (i == 22) num = 3;
    else if (i > 22) { const int t = (int)(i - 23); e = t < 3 ? t + 2 : t < 5 ? t + 4 : t + 10; }
    const int t = num >= 4 ? 2 : num >= 2 ? 1 : 0;
    const int be = e + t + F::bias;
    uint64_t r;
    if (be >= F::emax_b) r = F::inf;
    else if (be <= 0) r = num << (e + F::bias - 1 + F::mb);
    else r = ((uint64_t)be << F::mb) | ((num << (F::mb - t)) & F::frac);
    return i == 0 ? r | F::sign : r;
}

// fcvtmod.w.d (Zfa; decoder.isa:3320-3384): the binary64 value truncated to an
// integer, taken modulo 2^32 and sign-extended from bit 31; inexact when bits
// are dropped, invalid (instead of inexact) for NaN, infinity or a magnitude
// outside the int32 range.
FI_SF_HD uint64_t fcvtmod_w_d(uint64_t a, uint32_t &fl) {
    const bool neg = (a >> 63) != 0;
    const int ex = (int)((a >> 52) & 0x7FF);
    uint64_t frac = a & D::frac;
    bool inexact = false, invalid = false;
    if (ex == 0) {
        inexact = frac != 0;
        frac = 0;
    } else if (ex == 0x7FF) {
        invalid = true;
        frac = 0;
    } else {
        const int true_exp = ex - 1023, shift = true_exp - 52;
        frac |= 1ULL << 52;
        if (shift >= 64) frac = 0;
        else if (shift >= 0) frac <<= shift;
        else if (shift > -64) { inexact = (frac << (64 + shift)) != 0; frac >>= -shift; }
        else { frac = 0; inexact = true; }
        if (true_exp > 31 || frac > (neg ? 0x80000000ULL : 0x7FFFFFFFULL)) { invalid = true; inexact = false; }
        if (neg) frac = 0 - frac;
    }
    fl |= (inexact ? FL_NX : 0) | (invalid ? FL_NV : 0);
    return (uint64_t)(int64_t)(int32_t)(uint32_t)frac;
}

}  // namespace sf
}  // namespace fi

namespace fi {
namespace sf {
// One operation by code (the device interpreter's FP instructions, the pinning
// tests): op 0 add, 1 sub, 2 mul, 3 div, 4 sqrt, 5 mulAdd (a * b + c), 6 eq,
// 7 lt, 8 le, 9 lt_quiet, 10 le_quiet, 11..14 to i32/u32/i64/u64 (result as
// the reference returns it: i32 sign-extended, u32 zero-extended), 15..18
// from i32/u32/i64/u64, 19..21 convert to binary16/32/64; fmt 0 binary16,
// 1 binary32, 2 binary64 (the source format of a conversion); 22, 23
// roundToInt without / with the inexact flag (Zfa fround / froundnx).
enum : int { OP_ADD = 0, OP_SUB, OP_MUL, OP_DIV, OP_SQRT, OP_FMA, OP_EQ, OP_LT, OP_LE, OP_LTQ, OP_LEQ,
             OP_TO_I32, OP_TO_U32, OP_TO_I64, OP_TO_U64, OP_FROM_I32, OP_FROM_U32, OP_FROM_I64, OP_FROM_U64,
             OP_TO_H, OP_TO_S, OP_TO_D, OP_RINT, OP_RINTX, OP_COUNT };

template <class F> FI_SF_HD uint64_t op_fmt(int op, int rm, uint64_t a, uint64_t b, uint64_t c, uint32_t &fl) {
    switch (op) {
    case OP_ADD: return add<F>(a, b, rm, fl);
    case OP_SUB: return sub<F>(a, b, rm, fl);
    case OP_MUL: return mul<F>(a, b, rm, fl);
    case OP_DIV: return div<F>(a, b, rm, fl);
    case OP_SQRT: return sqrt<F>(a, rm, fl);
    case OP_FMA: return fma<F>(a, b, c, rm, fl);
    case OP_EQ: return eq<F>(a, b, fl);
    case OP_LT: return lt<F>(a, b, false, fl);
    case OP_LE: return le<F>(a, b, false, fl);
    case OP_LTQ: return lt<F>(a, b, true, fl);
    case OP_LEQ: return le<F>(a, b, true, fl);
    case OP_TO_I32: case OP_TO_U32: case OP_TO_I64: case OP_TO_U64: return to_int<F>(a, op - OP_TO_I32, rm, fl);
    case OP_FROM_I32: case OP_FROM_U32: case OP_FROM_I64: case OP_FROM_U64:
        return from_int<F>(a, op - OP_FROM_I32, rm, fl);
    case OP_RINT: case OP_RINTX: return rint<F>(a, rm, op == OP_RINTX, fl);
    default: return 0;
    }
}
template <class F> FI_SF_HD uint64_t cvt_from(int op, int rm, uint64_t a, uint32_t &fl) {
    switch (op) {
    case OP_TO_H: return convert<F, H>(a, rm, fl);
    case OP_TO_S: return convert<F, S>(a, rm, fl);
    default: return convert<F, D>(a, rm, fl);
    }
}
FI_SF_HD uint64_t op(int op, int fmt, int rm, uint64_t a, uint64_t b, uint64_t c, uint32_t &fl) {
    if (op >= OP_TO_H && op <= OP_TO_D) return fmt == 0 ? cvt_from<H>(op, rm, a, fl) : fmt == 1 ? cvt_from<S>(op, rm, a, fl)
                                                                    : cvt_from<D>(op, rm, a, fl);
    return fmt == 0 ? op_fmt<H>(op, rm, a, b, c, fl) : fmt == 1 ? op_fmt<S>(op, rm, a, b, c, fl)
                                                     : op_fmt<D>(op, rm, a, b, c, fl);
}
}  // namespace sf
}  // namespace fi
