// vcfxg_num.h -- exact `strtod(field) OP threshold` on the device, without computing the
// double for decimal inputs.
//
// VCFX_record_filter compares strtod(text) (glibc, correctly rounded, must consume the
// whole field: parseDouble, VCFX_record_filter.cpp:273-299) against a threshold t that
// was itself produced by strtod on the host.  For decimal text the 3-way relation of
// x = strtod(text) to t is decided exactly from the text against the two rounding
// boundaries of t (lo = midpoint(pred t, t), hi = midpoint(t, succ t)), whose exact
// decimal expansions the host precomputes (vcfxg_decimal.cpp):
//     x < t  <=>  text < lo  or (text == lo and the tie at lo rounds away from t)
//     x > t  <=>  text > hi  or (text == hi and the tie at hi rounds away from t)
// Hex floats are converted exactly (round half to even); inf/nan are compared as values.
// The accepted grammar is strtod's: leading isspace, sign, inf/infinity/nan/nan(...)
// (case-insensitive), 0x hex with optional binary exponent, decimal with optional
// exponent; anything left unconsumed makes the parse fail (criterion false).
// Byte sources (B: the text, PB: the threshold digit pool) are anything indexable as
// src[i] -> byte: a global pointer, or a wave's register copy (vcfxg_fq_walk.hip).
#pragma once
#include <stdint.h>

namespace vcfxg {

enum { OPN_GT = 0, OPN_GE, OPN_LT, OPN_LE, OPN_EQ, OPN_NE };

// normalized decimal: value = sign * 0.d1 d2 ... dn * 10^exp (d1 != 0), or zero (n == 0)
struct DecRef {
    int sign;        // -1 / +1 (0 for zero)
    int exp;
    uint32_t off;    // digits in the pool, '0'..'9'
    uint32_t n;
    int inf;         // boundary at +/- infinity (never equalled)
};

struct NumThreshold {
    double t;
    int kind;        // 0 finite, 1 nan
    DecRef lo, hi;
    int lo_to_t;     // a value exactly at lo rounds to t
    int hi_to_t;
};

__device__ __forceinline__ bool is_space(uint32_t c) { return c == ' ' || (c >= 9 && c <= 13); }
__device__ __forceinline__ uint32_t lower(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
__device__ __forceinline__ int hexval(uint32_t c) {
    if (c >= '0' && c <= '9') return (int)(c - '0');
    c = lower(c);
    if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
    return -1;
}

// parsed text
struct NumText {
    int kind;        // 0 decimal, 1 value (hex/inf/nan in v), -1 fail
    double v;
    int sign;        // decimal: -1/+1
    int64_t s0;      // decimal: position of the first significant digit ('.' may follow)
    int64_t end;     // decimal: end of the mantissa digits
    int exp;         // decimal: value = sign * 0.<digits from s0> * 10^exp
    bool zero;
};

template <class B>
__device__ __forceinline__ bool ieq(const B &buf, int64_t p, int64_t e, const char *w) {
    int i = 0;
    for (; w[i]; i++)
        if (p + i >= e || lower((uint8_t)buf[p + i]) != (uint32_t)w[i]) return false;
    return true;
}

// exact hex-float value (round half to even), mantissa digits [p, e) after "0x"
template <class B>
__device__ inline double hex_value(const B &buf, int64_t p, int64_t me, int64_t bexp) {
    // accumulate up to 64 significant bits; later nonzero bits -> sticky
    uint64_t m = 0;
    int shift = 0;   // binary exponent adjustment
    bool sticky = false, seen_dot = false, started = false;
    for (int64_t q = p; q < me; q++) {
        uint32_t c = (uint8_t)buf[q];
        if (c == '.') {
            seen_dot = true;
            continue;
        }
        int h = hexval(c);
        if (!started && h == 0) {
            if (seen_dot) shift -= 4;
            continue;
        }
        started = true;
        if (m >> 60) {  // no room: this digit only affects stickiness / exponent
            if (h) sticky = true;
            if (!seen_dot) shift += 4;
        } else {
            m = (m << 4) | (uint64_t)h;
            if (seen_dot) shift -= 4;
        }
    }
    if (m == 0) return 0.0;
    int64_t e2 = bexp + shift;  // value = m * 2^e2 (+ sticky)
    // normalize m to 64 bits with msb at bit 63
    int lz = __builtin_clzll(m);
    m <<= lz;
    e2 -= lz;
    // value = 1.xxx * 2^(e2 + 63)
    int64_t E = e2 + 63;
    if (E > 1023) return __longlong_as_double(0x7FF0000000000000ll);
    int keep;  // mantissa bits kept (incl. implicit)
    if (E >= -1022) keep = 53;
    else {
        keep = 53 - (int)(-1022 - E);
        if (keep < 0) keep = 0;
    }
    // round m (64 bits) to `keep` bits
    uint64_t r;
    int drop = 64 - keep;
    if (keep == 0) {
        // below half of the smallest subnormal unless exactly half with nothing else
        bool above_half = (E == -1075) && ((m << 1) != 0 || sticky);
        return above_half ? 4.9406564584124654e-324 : 0.0;
    }
    r = m >> drop;
    uint64_t rem = drop >= 64 ? m : (m & ((1ull << drop) - 1));
    uint64_t half = 1ull << (drop - 1);
    if (rem > half || (rem == half && (sticky || (r & 1)))) r += 1;
    else if (rem == half && !sticky && !(r & 1)) {}
    // r has `keep` (or keep+1 after carry) bits
    if (E >= -1022) {
        if (r >> 53) {
            r >>= 1;
            E += 1;
            if (E > 1023) return __longlong_as_double(0x7FF0000000000000ll);
        }
        uint64_t bits = ((uint64_t)(E + 1023) << 52) | (r & ((1ull << 52) - 1));
        return __longlong_as_double((long long)bits);
    }
    // subnormal: value = r * 2^-1074
    return __longlong_as_double((long long)r);  // r <= 2^52 (a carry into 2^52 is the min normal)
}

// parse text [p, e) with strtod's grammar; success only if everything is consumed
template <class B>
__device__ inline NumText parse_number(const B &buf, int64_t p, int64_t e) {
    NumText r;
    r.kind = -1;
    r.v = 0;
    r.sign = 1;
    r.s0 = r.end = 0;
    r.exp = 0;
    r.zero = false;
    while (p < e && is_space((uint8_t)buf[p])) p++;
    int sign = 1;
    if (p < e && (buf[p] == '+' || buf[p] == '-')) {
        if (buf[p] == '-') sign = -1;
        p++;
    }
    if (p >= e) return r;
    uint32_t c0 = lower((uint8_t)buf[p]);
    if (c0 == 'i') {
        if (ieq(buf, p, e, "infinity") && p + 8 == e) {}
        else if (!(ieq(buf, p, e, "inf") && p + 3 == e)) return r;
        r.kind = 1;
        r.v = sign * __longlong_as_double(0x7FF0000000000000ll);
        return r;
    }
    if (c0 == 'n') {
        if (!ieq(buf, p, e, "nan")) return r;
        int64_t q = p + 3;
        if (q < e) {
            if (buf[q] != '(') return r;
            q++;
            while (q < e && buf[q] != ')') {
                uint32_t c = (uint8_t)buf[q];
                if (!((c >= '0' && c <= '9') || (lower(c) >= 'a' && lower(c) <= 'z') || c == '_')) return r;
                q++;
            }
            if (q >= e || q + 1 != e) return r;  // needs ")" as the last byte
        }
        r.kind = 1;
        r.v = __longlong_as_double(0x7FF8000000000000ll);
        return r;
    }
    if (c0 == '0' && p + 1 < e && lower((uint8_t)buf[p + 1]) == 'x') {
        int64_t q = p + 2, ms = q;
        int nd = 0;
        bool dot = false;
        while (q < e) {
            uint32_t c = (uint8_t)buf[q];
            if (c == '.' && !dot) dot = true;
            else if (hexval(c) >= 0) nd++;
            else break;
            q++;
        }
        if (nd == 0) return r;  // strtod would stop after "0": not fully consumed
        int64_t me = q, bexp = 0;
        if (q < e && lower((uint8_t)buf[q]) == 'p') {
            int64_t t = q + 1;
            int es = 1;
            if (t < e && (buf[t] == '+' || buf[t] == '-')) {
                if (buf[t] == '-') es = -1;
                t++;
            }
            int64_t ds = t;
            int64_t ev = 0;
            while (t < e && buf[t] >= '0' && buf[t] <= '9') {
                if (ev < (1ll << 40)) ev = ev * 10 + (buf[t] - '0');
                t++;
            }
            if (t > ds) {
                bexp = es * ev;
                q = t;
            }
        }
        if (q != e) return r;
        r.kind = 1;
        r.v = sign * hex_value(buf, ms, me, bexp);
        return r;
    }
    // decimal
    int64_t q = p;
    int nint = 0, nfrac = 0;
    while (q < e && buf[q] >= '0' && buf[q] <= '9') { q++; nint++; }
    int64_t dotpos = -1;
    if (q < e && buf[q] == '.') {
        dotpos = q;
        q++;
        while (q < e && buf[q] >= '0' && buf[q] <= '9') { q++; nfrac++; }
    }
    if (nint + nfrac == 0) return r;
    int64_t me = q;
    int64_t ex = 0;
    if (q < e && lower((uint8_t)buf[q]) == 'e') {
        int64_t t = q + 1;
        int es = 1;
        if (t < e && (buf[t] == '+' || buf[t] == '-')) {
            if (buf[t] == '-') es = -1;
            t++;
        }
        int64_t ds = t;
        int64_t ev = 0;
        while (t < e && buf[t] >= '0' && buf[t] <= '9') {
            if (ev < (1ll << 30)) ev = ev * 10 + (buf[t] - '0');
            t++;
        }
        if (t > ds) {
            ex = es * ev;
            q = t;
        }
    }
    if (q != e) return r;
    // first significant digit
    int64_t s0 = -1;
    int lead_int = 0;  // integer digits before s0 that are zero... compute exponent
    int64_t k = p;
    int int_seen = 0;
    for (; k < me; k++) {
        if (k == dotpos) continue;
        if (buf[k] != '0') { s0 = k; break; }
        if (dotpos < 0 || k < dotpos) int_seen++;
    }
    (void)lead_int;
    r.kind = 0;
    r.sign = sign;
    if (s0 < 0) {
        r.zero = true;
        return r;
    }
    // digits before the point from s0
    int64_t exp10;
    if (dotpos < 0 || s0 < dotpos) {
        int64_t endint = dotpos < 0 ? me : dotpos;
        exp10 = endint - s0;  // 0.d1... * 10^(#int digits from s0)
    } else {
        exp10 = -(s0 - dotpos - 1);
    }
    exp10 += ex;
    if (exp10 > (1 << 30)) exp10 = (1 << 30);
    if (exp10 < -(1 << 30)) exp10 = -(1 << 30);
    r.s0 = s0;
    r.end = me;
    r.exp = (int)exp10;
    (void)int_seen;
    return r;
}

// compare |text| digits (from s0, skipping '.') with a pool digit string; both with the
// same exponent.  -1 / 0 / +1
template <class B, class PB>
__device__ inline int cmp_digits(const B &buf, int64_t s0, int64_t me, const PB &pool, uint32_t off, uint32_t n) {
    int64_t k = s0;
    uint32_t j = 0;
    for (;;) {
        while (k < me && buf[k] == '.') k++;
        bool ha = k < me, hb = j < n;
        if (!ha && !hb) return 0;
        uint32_t a = ha ? (uint8_t)buf[k] : '0', b = hb ? (uint8_t)pool[off + j] : '0';
        if (!ha) {
            // remaining b digits: any nonzero -> b bigger
            for (; j < n; j++)
                if (pool[off + j] != '0') return -1;
            return 0;
        }
        if (!hb) {
            for (; k < me; k++)
                if (buf[k] != '.' && buf[k] != '0') return 1;
            return 0;
        }
        if (a != b) return a < b ? -1 : 1;
        k++;
        j++;
    }
}

// 3-way compare of the decimal text with a boundary
template <class B, class PB>
__device__ inline int cmp_dec(const B &buf, const NumText &x, const DecRef &b, const PB &pool) {
    if (b.inf) return b.sign > 0 ? -1 : 1;
    int sa = x.zero ? 0 : x.sign, sb = b.n == 0 ? 0 : b.sign;
    if (sa != sb) return sa < sb ? -1 : 1;
    if (sa == 0) return 0;
    int mag;
    if (x.exp != b.exp) mag = x.exp < b.exp ? -1 : 1;
    else mag = cmp_digits(buf, x.s0, x.end, pool, b.off, b.n);
    return sa > 0 ? mag : -mag;
}

__device__ __forceinline__ bool apply_op(int op, int rel) {
    switch (op) {
    case OPN_GT: return rel > 0;
    case OPN_GE: return rel >= 0;
    case OPN_LT: return rel < 0;
    case OPN_LE: return rel <= 0;
    case OPN_EQ: return rel == 0;
    default: return rel != 0;
    }
}
__device__ __forceinline__ bool cmp_double(double x, int op, double y) {
    switch (op) {
    case OPN_GT: return x > y;
    case OPN_GE: return x >= y;
    case OPN_LT: return x < y;
    case OPN_LE: return x <= y;
    case OPN_EQ: return x == y;
    default: return x != y;
    }
}

// parseDouble(text) && compareDouble(x, op, t); *parsed = parse success
template <class B, class PB>
__device__ inline bool num_compare(const B &buf, int64_t p, int64_t e, const NumThreshold &T, int op, const PB &pool,
                                   bool *parsed) {
    NumText x = parse_number(buf, p, e);
    *parsed = x.kind >= 0;
    if (x.kind < 0) return false;
    if (x.kind == 1) return cmp_double(x.v, op, T.t);
    if (T.kind == 1) return op == OPN_NE;  // t is NaN
    int rel;
    int clo = cmp_dec(buf, x, T.lo, pool);
    if (clo < 0 || (clo == 0 && !T.lo_to_t)) rel = -1;
    else {
        int chi = cmp_dec(buf, x, T.hi, pool);
        if (chi > 0 || (chi == 0 && !T.hi_to_t)) rel = 1;
        else rel = 0;
    }
    return apply_op(op, rel);
}

}  // namespace vcfxg
