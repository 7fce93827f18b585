// vcfxg_decimal.cpp -- host side of the exact numeric compare (vcfxg_num.h): the exact
// decimal expansions of a threshold's two rounding boundaries.
//
// For a finite double t = M * 2^e (M integer, 53-bit for normals), the reals that strtod
// rounds to t form the interval between lo = midpoint(pred t, t) and hi = midpoint(t,
// succ t); the endpoints are dyadic rationals (2M+-1) * 2^(e-1) (or (4M-1) * 2^(e-2) below
// a power of two), so their decimal expansions are finite.  A value exactly on an endpoint
// rounds to the neighbour with the even significand (glibc round-half-even).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "vcfxg_decimal.h"

namespace vcfxg {
namespace {

// little-endian base 1e9 bignum
struct Big {
    std::vector<uint32_t> w;
    explicit Big(uint64_t v) {
        while (v) {
            w.push_back((uint32_t)(v % 1000000000u));
            v /= 1000000000u;
        }
    }
    void mul(uint32_t k) {
        uint64_t carry = 0;
        for (auto &x : w) {
            uint64_t t = (uint64_t)x * k + carry;
            x = (uint32_t)(t % 1000000000u);
            carry = t / 1000000000u;
        }
        while (carry) {
            w.push_back((uint32_t)(carry % 1000000000u));
            carry /= 1000000000u;
        }
    }
    std::string str() const {
        if (w.empty()) return "0";
        std::string s = std::to_string(w.back());
        char b[16];
        for (size_t i = w.size() - 1; i-- > 0;) {
            snprintf(b, sizeof b, "%09u", w[i]);
            s += b;
        }
        return s;
    }
};

// N * 2^k as normalized decimal (sign applied by caller)
void dyadic(uint64_t N, int k, int sign, DecHost &d) {
    d.sign = sign;
    d.inf = 0;
    if (N == 0) {
        d.sign = 0;
        d.exp = 0;
        d.digits.clear();
        return;
    }
    Big b(N);
    int scale = 0;  // value = b * 10^-scale
    if (k >= 0)
        for (int i = 0; i < k; i++) b.mul(2);
    else {
        for (int i = 0; i < -k; i++) b.mul(5);
        scale = -k;
    }
    std::string s = b.str();
    d.exp = (int)s.size() - scale;
    size_t z = s.find_last_not_of('0');
    d.digits = s.substr(0, z + 1);
}

}  // namespace

void threshold_bounds(double t, ThresholdHost &out) {
    out.t = t;
    out.kind = 0;
    if (std::isnan(t)) {
        out.kind = 1;
        return;
    }
    const int sg = std::signbit(t) ? -1 : 1;
    const double a = std::fabs(t);
    DecHost near_, far_;  // boundary toward zero / away from zero
    int near_to_t, far_to_t;
    if (std::isinf(a)) {
        // +inf: every real >= DBL_MAX + ulp/2 rounds to inf (the tie goes to inf)
        dyadic((2ull * ((1ull << 53) - 1)) + 1, 970, 1, near_);
        near_to_t = 1;
        far_.inf = 1;
        far_.sign = 1;
        far_to_t = 0;
    } else if (a == 0.0) {
        dyadic(1, -1075, 1, far_);
        far_to_t = 1;  // half the smallest subnormal rounds to (even) zero
        near_ = far_;
        near_.sign = -1;
        near_to_t = 1;
        // for zero: "near" is the negative side, "far" the positive side (no sign flip)
        out.lo = near_;
        out.hi = far_;
        out.lo_to_t = near_to_t;
        out.hi_to_t = far_to_t;
        return;
    } else {
        int ex;
        double fr = std::frexp(a, &ex);  // a = fr * 2^ex, fr in [0.5, 1)
        uint64_t M;
        int e;
        if (ex - 53 >= -1074) {
            M = (uint64_t)std::ldexp(fr, 53);
            e = ex - 53;
        } else {  // subnormal
            M = (uint64_t)std::ldexp(a, 1074);
            e = -1074;
        }
        const bool even = (M & 1) == 0;
        dyadic(2 * M + 1, e - 1, 1, far_);
        far_to_t = even;
        if (M == (1ull << 52) && e > -1074) dyadic(4 * M - 1, e - 2, 1, near_);
        else dyadic(2 * M - 1, e - 1, 1, near_);
        near_to_t = even;
    }
    if (sg > 0) {
        out.lo = near_;
        out.hi = far_;
        out.lo_to_t = near_to_t;
        out.hi_to_t = far_to_t;
    } else {
        out.lo = far_;
        out.hi = near_;
        out.lo.sign = -out.lo.sign;
        out.hi.sign = -out.hi.sign;
        out.lo_to_t = far_to_t;
        out.hi_to_t = near_to_t;
    }
}

}  // namespace vcfxg
