// Drop-in for the reference's include/isoform_assignment.h (:24-27, :41-44): the EM and the read
// assignment over sparse_chain's string-keyed results. Definitions in libskq.so (csrc/skq_dropin.cpp,
// over skq_em / skq_assign: the same arithmetic as src/isoform_assignment.cpp:9-97, summed in a
// fixed order instead of unordered_map order, so pi and the counts agree to rounding, not bits).
#ifndef ISOFORM_ASSIGNMENT_H
#define ISOFORM_ASSIGNMENT_H

#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "data_io.h"

std::unordered_map<std::string, double> estimate_isoform_abundance_em(
    const std::unordered_map<std::string, std::vector<std::pair<std::string, int>>>& homologous_segments,
    const std::unordered_map<std::string, Transcript>& transcripts,
    int max_iterations, double convergence_threshold);

std::unordered_map<std::string, double> assign_reads_to_isoforms(
    const std::unordered_map<std::string, std::vector<std::pair<std::string, int>>>& homologous_segments,
    const std::unordered_map<std::string, double>& pi,
    const std::unordered_map<std::string, Transcript>& transcripts);

#endif  // ISOFORM_ASSIGNMENT_H
