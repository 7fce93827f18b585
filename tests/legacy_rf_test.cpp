// legacy_rf_test.cpp -- exercises the VCFX_record_filter library interface (parseCriteria,
// recordPasses, processVCF; VCFX_record_filter.h:99-102) and prints every observable result.
// Built by tests/test_legacy_api.py against build/libvcfx_record_filter.so and against the
// reference's own src/VCFX_record_filter/VCFX_record_filter.cpp (its main renamed); the outputs
// must be identical.
//   legacy_rf_test records CRITERIA_FILE RECORDS_FILE      parseCriteria + recordPasses
//   legacy_rf_test process CRITERIA_FILE VCF_FILE          processVCF (stdout; warnings on stderr)
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#ifdef VCFX_OURS
#include "vcfx_record_filter.h"
#else
#include "VCFX_record_filter.h"
#endif

static std::vector<std::string> lines_of(const char *path) {
    std::ifstream f(path, std::ios::binary);
    std::vector<std::string> v;
    std::string l;
    while (std::getline(f, l)) v.push_back(l);
    return v;
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    const std::string mode = argv[1];
    const auto crits = lines_of(argv[2]);
    for (const auto &cs : crits) {
        std::vector<FilterCriterion> c;
        const bool ok = parseCriteria(cs, c);
        std::cout << "criteria <" << cs << "> ok=" << ok << " n=" << c.size() << "\n";
        for (const auto &f : c)
            std::cout << "  name=<" << f.fieldName << "> op=" << (int)f.op << " num=" << f.numericValue << " str=<"
                      << f.stringValue << "> type=" << (int)f.fieldType << " target=" << (int)f.target << "\n";
        if (!ok) continue;
        for (int logic = 1; logic >= 0; logic--) {
            if (mode == "records") {
                std::string bits;
                for (const auto &r : lines_of(argv[3])) bits += recordPasses(r, c, logic == 1) ? '1' : '0';
                std::cout << (logic ? "  and " : "  or  ") << bits << "\n";
            } else {
                std::ifstream in(argv[3], std::ios::binary);
                std::ostringstream out;
                processVCF(in, out, c, logic == 1);
                std::cout << (logic ? "  and:\n" : "  or:\n") << out.str() << "  --\n";
            }
        }
    }
    return 0;
}
