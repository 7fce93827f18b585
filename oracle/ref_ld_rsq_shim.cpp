// ref_ld_rsq_shim.cpp -- TEST INFRASTRUCTURE ONLY (the checker; never linked by the product).
//
// Exposes the reference's own r^2 function, computeRsqFast (VCFX_ld_calculator.cpp:397-401 ->
// computeRsqSIMD :352-393, with LDVariantOpt::computeStats :243-258 for the own-variance gate),
// as a C symbol, so the device's fp64 r^2 values can be compared with the REFERENCE's doubles
// bit for bit, not only with the oracle's restatement of them.  The reference source is not
// copied: oracle/Makefile.ref compiles this file with -I on the reference's tool directory, so
// the #include below reads /root/reference at build time, with the tool's main() renamed.
// Output: oracle/_ref/libref_ld_rsq.so (git-ignored).
#define main vcfx_ld_calculator_ref_main
#include "VCFX_ld_calculator.cpp"
#undef main

extern "C" double ref_rsq_fast(const int8_t *g1, const int8_t *g2, size_t n) {
    LDVariantOpt a, b;
    a.genotype.assign(g1, g1 + n);
    b.genotype.assign(g2, g2 + n);
    a.computeStats();
    b.computeStats();
    return computeRsqFast(a, b);
}
