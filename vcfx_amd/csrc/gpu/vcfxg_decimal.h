// vcfxg_decimal.h -- exact decimal rounding boundaries of a double threshold (host).
#pragma once
#include <string>

namespace vcfxg {

struct DecHost {
    int sign = 0;  // -1 / +1, 0 = zero
    int exp = 0;   // value = sign * 0.<digits> * 10^exp
    std::string digits;
    int inf = 0;   // +/- infinity (never equalled)
};

struct ThresholdHost {
    double t = 0;
    int kind = 0;  // 0 finite/inf, 1 nan
    DecHost lo, hi;
    int lo_to_t = 0, hi_to_t = 0;
};

void threshold_bounds(double t, ThresholdHost &out);

}  // namespace vcfxg
