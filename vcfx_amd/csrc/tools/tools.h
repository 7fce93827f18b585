// tools.h -- in-process entry points of the VCFX_<tool> drop-ins (libvcfx_tools.so).
// Each has the tool's exact CLI contract; binaries are thin main()s over these, and tests
// call them in-process to reuse one GPU context across many cases.
#pragma once
#include <stdio.h>
#include <stdlib.h>

#include <getopt.h>

#include <mutex>
#include <string>
#include <vector>

#include "hostio.h"

#include "vcfx_tools.h"

namespace vcfxh {

// compiled record_filter criterion (FilterCriterion, VCFX_record_filter.h:37-44)
struct Criterion {
    std::string name, str;
    int op = 0, target = 0;
    bool numeric = false;
    double value = 0.0;
};
bool compile_filter(const std::string &all, std::vector<Criterion> &out, Out &err);
// the drop-ins' help texts (the library interfaces' printHelp)
const char *rf_help_text();
const char *gq_help_text();
std::vector<vcfxg_criterion> to_abi(const std::vector<Criterion> &cs);

// getopt_long prints its diagnostics on the C stderr stream; route them to the tool's
// err fd (identical text to the reference's getopt messages).
// getopt_long's state (optind, optarg) and the stderr swap are process-wide: the argument
// phase of the tools is serialised (the ranks of an in-process multi-GPU run parse at once).
std::recursive_mutex &getopt_mutex();
struct GetoptStderr {
    Out &err;
    std::unique_lock<std::recursive_mutex> lk;
    FILE *saved = nullptr, *mem = nullptr;
    char *buf = nullptr;
    size_t len = 0;
    explicit GetoptStderr(Out &e) : err(e), lk(getopt_mutex()) {
        fflush(stderr);
        mem = open_memstream(&buf, &len);
        saved = stderr;
        stderr = mem;
    }
    int next = 0;  // optind when the argument phase ended (read it, not optind, afterwards)
    void done() {
        if (lk.owns_lock()) next = optind;
        if (mem) {
            fflush(mem);
            stderr = saved;
            fclose(mem);
            mem = nullptr;
            if (len) err.put(buf, len);
            free(buf);
            buf = nullptr;
        }
        if (lk.owns_lock()) lk.unlock();
    }
    ~GetoptStderr() { done(); }
};
}  // namespace vcfxh
