/*
 * vcfx_genotype_query.h -- the VCFX_genotype_query library interface of the reference
 * (src/VCFX_genotype_query/VCFX_genotype_query.h:9-24), served by
 * build/libvcfx_genotype_query.so over the MI355X engine (include/vcfx_gpu.h):
 * genotypeQuery / genotypeQueryStream run the drop-in's stream path (records matched on the
 * GPU), parseArguments / printHelp are the CLI's.
 */
#ifndef VCFX_GENOTYPE_QUERY_H
#define VCFX_GENOTYPE_QUERY_H

#include <iostream>
#include <string>

bool parseArguments(int argc, char *argv[], std::string &genotype_query, bool &strictCompare, std::string &inputFile,
                    bool &quiet);
void printHelp();
void genotypeQuery(std::istream &in, std::ostream &out, const std::string &genotype_query, bool strictCompare);
void genotypeQueryStream(std::istream &in, std::ostream &out, const std::string &genotype_query, bool strictCompare,
                         bool quiet);

#endif
