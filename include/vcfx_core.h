// vcfx_core.h -- the VCFX core library API (libvcfx_core), source-compatible with the
// reference's include/vcfx_core.h so code written against `vcfx::` builds unchanged.
//
// Declarations follow the reference API (include/vcfx_core.h); the implementations in
// vcfx_amd/csrc/host/vcfx_core.cpp are written for this project and cite the reference
// behaviour they keep (src/vcfx_core.cpp).  Host-only: nothing here touches the GPU.
#ifndef VCFX_CORE_H
#define VCFX_CORE_H

#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

namespace vcfx {

// whitespace (" \t\n\r") removed from both ends
std::string trim(const std::string &str);

// istringstream/getline split: a trailing delimiter adds no empty last field, "" -> {}
std::vector<std::string> split(const std::string &str, char delimiter);

// "Error: <msg>\n"
void print_error(const std::string &msg, std::ostream &os = std::cerr);
// "<tool> version <version>\n"
void print_version(const std::string &tool, const std::string &version, std::ostream &os = std::cout);

inline std::string get_version() {
#ifdef VCFX_VERSION
    return VCFX_VERSION;
#else
    return "unknown";
#endif
}

// true if argv[1..] holds long_flag (or short_flag when given)
bool flag_present(int argc, char *argv[], const char *long_flag, const char *short_flag = nullptr);

inline bool handle_version_flag(int argc, char *argv[], const std::string &tool, std::ostream &os = std::cout) {
    if (!flag_present(argc, argv, "--version", "-v")) return false;
    print_version(tool, get_version(), os);
    return true;
}

inline bool handle_help_flag(int argc, char *argv[], void (*print_help)()) {
    if (!flag_present(argc, argv, "--help", "-h")) return false;
    if (print_help) print_help();
    return true;
}

// --help first, then --version; true when the caller should exit
inline bool handle_common_flags(int argc, char *argv[], const std::string &tool, void (*print_help)(),
                                std::ostream &os = std::cout) {
    return handle_help_flag(argc, argv, print_help) || handle_version_flag(argc, argv, tool, os);
}

// whole stream into `out`, inflating when it starts with the gzip magic (1f 8b)
bool read_maybe_compressed(std::istream &in, std::string &out);
// whole file into `out`; inflated when named *.gz / *.bgz / *.bgzf or gzip-magic
bool read_file_maybe_compressed(const std::string &path, std::string &out);

// Line reader over a plain or gzip/BGZF (multi-member) stream with bounded memory.
// getline() returns lines without '\n' (and without a '\r' right before it).
class StreamingGzipReader {
public:
    explicit StreamingGzipReader(std::istream &in);
    ~StreamingGzipReader();
    StreamingGzipReader(const StreamingGzipReader &) = delete;
    StreamingGzipReader &operator=(const StreamingGzipReader &) = delete;
    StreamingGzipReader(StreamingGzipReader &&other) noexcept;
    StreamingGzipReader &operator=(StreamingGzipReader &&other) noexcept;

    bool getline(std::string &line);
    bool error() const;
    bool eof() const;
    bool is_compressed() const;

private:
    struct State;
    std::unique_ptr<State> s_;
};

std::unique_ptr<StreamingGzipReader> make_streaming_reader(std::istream &in);
std::unique_ptr<StreamingGzipReader> make_streaming_reader(const std::string &path, std::ifstream &fileStream);

}  // namespace vcfx

#endif  // VCFX_CORE_H
