// vcfx_core.cpp -- libvcfx_core: the host-side VCFX core API (include/vcfx_core.h).
//
// Behaviour kept from the reference (src/vcfx_core.cpp):
//   trim / split                 :11-29   (split has getline semantics: no empty last field)
//   flag_present / print_*       :31-44
//   read_maybe_compressed        :~95-130 (gzip magic sniff; inflate window 15+32 = gzip or
//                                          zlib; stops at the END of the first member, false
//                                          when the stream ends before it; the file variant
//                                          also accepts .gz/.bgz/.bgzf names and appends)
//   StreamingGzipReader          :~133-353 (64 KiB reads; "\r\n" -> line without '\r';
//                                          a final unterminated line is returned as is;
//                                          multi-member (BGZF) streams continue after each
//                                          member end)
// Kept quirk: a one-byte input reads as empty.  Differences: a gzip stream truncated
// mid-member ends the reader (eof) where the reference spins; buffers live behind a pimpl.
#include "vcfx_core.h"

#include <zlib.h>

#include <sstream>

namespace vcfx {

namespace {
constexpr size_t kChunk = 64 * 1024;
const char *const kSpace = " \t\n\r";

bool sniff_gzip(std::istream &in) {
    const int a = in.get();
    if (a == EOF) return false;
    const int b = in.get();
    if (b == EOF) {
        // kept quirk: the reference ungets on a stream already at EOF, which fails, so a
        // one-byte input reads as empty (src/vcfx_core.cpp stream_has_gzip_magic)
        in.unget();
        return false;
    }
    in.putback((char)b);
    in.putback((char)a);
    return a == 0x1f && b == 0x8b;
}

// inflate the first gzip/zlib member of `in`, appending to out
bool inflate_first_member(std::istream &in, std::string &out) {
    z_stream z;
    std::memset(&z, 0, sizeof z);
    if (inflateInit2(&z, 15 + 32) != Z_OK) return false;
    std::vector<char> ib(kChunk), ob(kChunk);
    int rc = Z_OK;
    bool done = false;
    while (!done) {
        in.read(ib.data(), (std::streamsize)ib.size());
        const size_t got = (size_t)in.gcount();
        if (got == 0) break;  // input ended before the member did
        z.next_in = reinterpret_cast<Bytef *>(ib.data());
        z.avail_in = (uInt)got;
        do {
            z.next_out = reinterpret_cast<Bytef *>(ob.data());
            z.avail_out = (uInt)ob.size();
            rc = inflate(&z, Z_NO_FLUSH);
            if (rc == Z_NEED_DICT || rc == Z_DATA_ERROR || rc == Z_MEM_ERROR || rc == Z_STREAM_ERROR) {
                inflateEnd(&z);
                return false;
            }
            out.append(ob.data(), ob.size() - z.avail_out);
            if (rc == Z_STREAM_END) done = true;
        } while (!done && z.avail_out == 0);
    }
    inflateEnd(&z);
    return rc == Z_STREAM_END;
}

bool ends_with(const std::string &s, const char *suf) {
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}
}  // namespace

std::string trim(const std::string &str) {
    const size_t a = str.find_first_not_of(kSpace);
    if (a == std::string::npos) return std::string();
    const size_t b = str.find_last_not_of(kSpace);
    return str.substr(a, b - a + 1);
}

std::vector<std::string> split(const std::string &str, char delimiter) {
    std::vector<std::string> v;
    size_t p = 0;
    while (p < str.size()) {
        const size_t e = str.find(delimiter, p);
        if (e == std::string::npos) {
            v.emplace_back(str, p);
            break;
        }
        v.emplace_back(str, p, e - p);
        p = e + 1;
    }
    return v;
}

bool flag_present(int argc, char *argv[], const char *long_flag, const char *short_flag) {
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], long_flag)) return true;
        if (short_flag && !std::strcmp(argv[i], short_flag)) return true;
    }
    return false;
}

void print_error(const std::string &msg, std::ostream &os) { os << "Error: " << msg << '\n'; }

void print_version(const std::string &tool, const std::string &version, std::ostream &os) {
    os << tool << " version " << version << '\n';
}

bool read_maybe_compressed(std::istream &in, std::string &out) {
    out.clear();
    if (sniff_gzip(in)) return inflate_first_member(in, out);
    std::ostringstream ss;
    ss << in.rdbuf();
    out = ss.str();
    return true;
}

bool read_file_maybe_compressed(const std::string &path, std::string &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return false;
    const bool named = ends_with(path, ".gz") || ends_with(path, ".bgz") || ends_with(path, ".bgzf");
    if (named || sniff_gzip(f)) return inflate_first_member(f, out);
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// ------------------------------------------------------------------------------------------
struct StreamingGzipReader::State {
    std::istream &in;
    bool compressed = false, at_end = false, failed = false;
    z_stream *z = nullptr;
    std::vector<char> ib, ob;
    std::string pending;  // bytes not yet returned, from `head`
    size_t head = 0;
    explicit State(std::istream &s) : in(s), ib(kChunk), ob(kChunk) {}
    ~State() {
        if (z) {
            inflateEnd(z);
            delete z;
        }
    }
    // more bytes into `pending`; false at the end of the input or on error
    bool refill() {
        if (head > kChunk && head * 2 > pending.size()) {  // drop consumed bytes now and then
            pending.erase(0, head);
            head = 0;
        }
        if (!compressed) {
            if (!in.good()) return false;
            in.read(ob.data(), (std::streamsize)ob.size());
            const size_t got = (size_t)in.gcount();
            pending.append(ob.data(), got);
            return got > 0;
        }
        if (z->avail_in == 0) {
            if (!in.good()) return false;  // the input ended (possibly mid-member)
            in.read(ib.data(), (std::streamsize)ib.size());
            const size_t got = (size_t)in.gcount();
            if (got == 0) return false;
            z->next_in = reinterpret_cast<Bytef *>(ib.data());
            z->avail_in = (uInt)got;
        }
        z->next_out = reinterpret_cast<Bytef *>(ob.data());
        z->avail_out = (uInt)ob.size();
        const int rc = inflate(z, Z_NO_FLUSH);
        if (rc == Z_NEED_DICT || rc == Z_DATA_ERROR || rc == Z_MEM_ERROR || rc == Z_STREAM_ERROR) {
            failed = true;
            return false;
        }
        pending.append(ob.data(), ob.size() - z->avail_out);
        if (rc == Z_STREAM_END) {
            if (z->avail_in > 0 || in.good()) inflateReset(z);  // next BGZF / gzip member
            else at_end = true;
        }
        return true;
    }
};

StreamingGzipReader::StreamingGzipReader(std::istream &in) : s_(new State(in)) {
    const int a = in.peek();
    if (a == EOF) {
        s_->at_end = true;
        return;
    }
    s_->compressed = sniff_gzip(in);
    if (s_->compressed) {
        s_->z = new z_stream;
        std::memset(s_->z, 0, sizeof(z_stream));
        if (inflateInit2(s_->z, 15 + 32) != Z_OK) {
            delete s_->z;
            s_->z = nullptr;
            s_->failed = true;
        }
    }
}

StreamingGzipReader::~StreamingGzipReader() = default;
StreamingGzipReader::StreamingGzipReader(StreamingGzipReader &&other) noexcept = default;
StreamingGzipReader &StreamingGzipReader::operator=(StreamingGzipReader &&other) noexcept = default;

bool StreamingGzipReader::getline(std::string &line) {
    line.clear();
    State &s = *s_;
    if (s.failed) return false;
    for (;;) {
        const size_t nl = s.pending.find('\n', s.head);
        if (nl != std::string::npos) {
            size_t e = nl;
            if (e > s.head && s.pending[e - 1] == '\r') --e;
            line.assign(s.pending, s.head, e - s.head);
            s.head = nl + 1;
            return true;
        }
        if (s.at_end || !s.refill()) {
            if (s.failed) return false;
            s.at_end = true;
            if (s.head < s.pending.size()) {
                line.assign(s.pending, s.head, std::string::npos);
                s.pending.clear();
                s.head = 0;
                return true;
            }
            return false;
        }
    }
}

bool StreamingGzipReader::error() const { return s_->failed; }
bool StreamingGzipReader::eof() const { return s_->at_end && s_->head >= s_->pending.size(); }
bool StreamingGzipReader::is_compressed() const { return s_->compressed; }

std::unique_ptr<StreamingGzipReader> make_streaming_reader(std::istream &in) {
    std::unique_ptr<StreamingGzipReader> r(new StreamingGzipReader(in));
    if (r->error()) return nullptr;
    return r;
}

std::unique_ptr<StreamingGzipReader> make_streaming_reader(const std::string &path, std::ifstream &fileStream) {
    fileStream.open(path, std::ios::binary);
    if (!fileStream.is_open()) return nullptr;
    return make_streaming_reader(fileStream);
}

}  // namespace vcfx
