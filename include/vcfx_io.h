// vcfx_io.h -- field-splitting helpers of the VCFX core API, source-compatible with the
// reference's include/vcfx_io.h (init_io, split_tabs, split_tabs_view, split_char,
// split_string, count_fields, vcfx::VCF field indices).
//
// Semantics kept: every split yields (number of delimiters + 1) fields, so a trailing
// delimiter DOES give an empty last field (unlike vcfx::split); output vectors are cleared
// but keep their capacity.  Header-only, host-only.
#ifndef VCFX_IO_H
#define VCFX_IO_H

#include <cstring>
#include <iostream>
#include <string>
#include <string_view>
#include <vector>

namespace vcfx {

inline void init_io() {
    std::ios::sync_with_stdio(false);
    std::cin.tie(nullptr);
}

namespace detail {
// calls emit(begin, length) for each field of s split at d
template <class Emit>
inline size_t for_each_field(const char *s, size_t n, char d, Emit emit) {
    size_t fields = 0, b = 0;
    for (;;) {
        const void *hit = n > b ? std::memchr(s + b, d, n - b) : nullptr;
        const size_t e = hit ? (size_t)(static_cast<const char *>(hit) - s) : n;
        emit(b, e - b);
        ++fields;
        if (!hit) return fields;
        b = e + 1;
    }
}
template <class V>
inline void prepare(V &out, size_t expected) {
    out.clear();
    if (out.capacity() < expected) out.reserve(expected);
}
}  // namespace detail

inline size_t split_tabs(const std::string &line, std::vector<std::string> &out, size_t expected = 16) {
    detail::prepare(out, expected);
    return detail::for_each_field(line.data(), line.size(), '\t',
                                  [&](size_t b, size_t len) { out.emplace_back(line, b, len); });
}

inline std::vector<std::string> split_tabs(const std::string &line) {
    std::vector<std::string> v;
    split_tabs(line, v);
    return v;
}

inline size_t split_tabs_view(std::string_view line, std::vector<std::string_view> &out, size_t expected = 16) {
    detail::prepare(out, expected);
    return detail::for_each_field(line.data(), line.size(), '\t',
                                  [&](size_t b, size_t len) { out.emplace_back(line.substr(b, len)); });
}

inline size_t split_char(std::string_view str, char delim, std::vector<std::string_view> &out,
                         size_t expected = 8) {
    detail::prepare(out, expected);
    return detail::for_each_field(str.data(), str.size(), delim,
                                  [&](size_t b, size_t len) { out.emplace_back(str.substr(b, len)); });
}

inline size_t split_string(const std::string &str, char delim, std::vector<std::string> &out,
                           size_t expected = 8) {
    detail::prepare(out, expected);
    return detail::for_each_field(str.data(), str.size(), delim,
                                  [&](size_t b, size_t len) { out.emplace_back(str, b, len); });
}

// fields of a tab-separated line (tabs + 1)
inline size_t count_fields(std::string_view line) {
    size_t tabs = 0;
    for (char ch : line) tabs += ch == '\t';
    return tabs + 1;
}

// VCF column indices
namespace VCF {
constexpr int CHROM = 0;
constexpr int POS = 1;
constexpr int ID = 2;
constexpr int REF = 3;
constexpr int ALT = 4;
constexpr int QUAL = 5;
constexpr int FILTER = 6;
constexpr int INFO = 7;
constexpr int FORMAT = 8;
constexpr int FIRST_SAMPLE = 9;
constexpr int MIN_FIELDS = 8;
}  // namespace VCF

}  // namespace vcfx

#endif  // VCFX_IO_H
