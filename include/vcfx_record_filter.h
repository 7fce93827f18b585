/*
 * vcfx_record_filter.h -- the VCFX_record_filter library interface of the reference
 * (src/VCFX_record_filter/VCFX_record_filter.h:14-102): the compiled criterion types and the
 * legacy free functions parseCriteria / recordPasses / processVCF / printHelp, served by
 * build/libvcfx_record_filter.so over the MI355X engine (include/vcfx_gpu.h).
 *
 * processVCF evaluates every record on the GPU (vcfxg_record_filter_ex with the legacy
 * semantics: lines keep their '\r', OR-mode QUAL lenient).  recordPasses is the per-record
 * predicate: one record is evaluated on the host (a device round trip per record would cost
 * ~20x the evaluation); processVCF hands it only the lines the device flags
 * (VCFXG_LINE_RECHECK: an OR-mode QUAL that needs strtod's prefix value).
 */
#ifndef VCFX_RECORD_FILTER_H
#define VCFX_RECORD_FILTER_H

#include <cstdint>
#include <iostream>
#include <string>
#include <vector>

enum class FilterOp : uint8_t { GT, GE, LT, LE, EQ, NE };
enum class FieldType : uint8_t { NUMERIC, STRING };
enum class TargetField : uint8_t { POS, QUAL, FILTER, INFO_KEY };

struct FilterCriterion {
    std::string fieldName;
    FilterOp op;
    double numericValue;
    std::string stringValue;
    FieldType fieldType;
    TargetField target;
};

// Legacy API (VCFX_record_filter.h:99-102; VCFX_record_filter.cpp:663-812)
bool parseCriteria(const std::string &criteriaStr, std::vector<FilterCriterion> &criteria);
bool recordPasses(const std::string &record, const std::vector<FilterCriterion> &criteria, bool useAndLogic);
void processVCF(std::istream &in, std::ostream &out, const std::vector<FilterCriterion> &criteria, bool useAndLogic);
void printHelp();

#endif
