// genotype_query_api.cpp -- the reference's VCFX_genotype_query library interface
// (include/vcfx_genotype_query.h) over the MI355X engine.
//
//   parseArguments       VCFX_genotype_query.cpp:379-428
//   printHelp            :350-373
//   genotypeQuery        :522-525
//   genotypeQueryStream  :527-617: the drop-in's stream path (the records matched on the GPU)
//                        on the istream's bytes, its output copied to the ostream
#include <getopt.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

#include <iterator>
#include <string>
#include <vector>

#include "hostio.h"
#include "tools.h"
#include "vcfx_genotype_query.h"

using namespace vcfxh;

void printHelp() { std::cout << gq_help_text(); }

bool parseArguments(int argc, char *argv[], std::string &genotype_query, bool &strictCompare, std::string &inputFile,
                    bool &quiet) {
    genotype_query.clear();
    inputFile.clear();
    strictCompare = false;
    quiet = false;
    static struct option lo[] = {{"genotype-query", required_argument, nullptr, 'g'},
                                 {"input", required_argument, nullptr, 'i'},
                                 {"strict", no_argument, nullptr, 's'},
                                 {"quiet", no_argument, nullptr, 'q'},
                                 {"help", no_argument, nullptr, 'h'},
                                 {"version", no_argument, nullptr, 'v'},
                                 {nullptr, 0, nullptr, 0}};
    int opt;
    while ((opt = getopt_long(argc, argv, "g:i:qhv", lo, nullptr)) != -1) {
        switch (opt) {
        case 'g': genotype_query = optarg; break;
        case 'i': inputFile = optarg; break;
        case 's': strictCompare = true; break;
        case 'q': quiet = true; break;
        case 'h':
            printHelp();
            std::exit(0);
        case 'v':
            std::cout << "VCFX_genotype_query version 1.0\n";
            std::exit(0);
        default: return false;
        }
    }
    if (optind < argc && inputFile.empty()) inputFile = argv[optind];
    return !genotype_query.empty();
}

void genotypeQuery(std::istream &in, std::ostream &out, const std::string &genotype_query, bool strictCompare) {
    genotypeQueryStream(in, out, genotype_query, strictCompare, false);
}

void genotypeQueryStream(std::istream &in, std::ostream &out, const std::string &genotype_query, bool strictCompare,
                         bool quiet) {
    const std::string buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    // the tool's stdin path over the bytes (memory files: no disk, no copy back through a pipe)
    const int fi = memfd_create("vcfx_gq_in", 0), fo = memfd_create("vcfx_gq_out", 0);
    if (fi < 0 || fo < 0) {
        if (fi >= 0) close(fi);
        if (fo >= 0) close(fo);
        std::cerr << "Error: vcfx_amd: memfd_create failed\n";
        return;
    }
    write_all(fi, buf.data(), buf.size());
    lseek(fi, 0, SEEK_SET);
    std::vector<std::string> args = {"VCFX_genotype_query", "--genotype-query", genotype_query};
    if (strictCompare) args.push_back("--strict");
    if (quiet) args.push_back("--quiet");
    std::vector<char *> argv;
    for (auto &a : args) argv.push_back(&a[0]);
    argv.push_back(nullptr);
    std::cerr.flush();
    vcfx_tool_genotype_query((int)args.size(), argv.data(), fi, fo, 2);
    const off_t n = lseek(fo, 0, SEEK_END);
    if (n > 0) {
        void *m = mmap(nullptr, (size_t)n, PROT_READ, MAP_PRIVATE, fo, 0);
        if (m != MAP_FAILED) {
            out.write((const char *)m, (std::streamsize)n);
            munmap(m, (size_t)n);
        }
    }
    close(fi);
    close(fo);
}
