// realign.hpp -- the indel realigner's regions on the host (realign.cpp) and the device's indel genotyping
// inputs (kernels.hip KI).  Internal to libngsep_amd.so.
//
// A region is the reach of the reference's IndelRealignerPileupListener around alignments with indels
// (discovery/IndelRealignerPileupListener.java:85-526): inside it the listener edits alignments (moves indel
// starts, realigns and trims alignment ends) while the pileup sweep goes on, so every pileup of the region is
// taken from the alignments as edited so far.  realign_region replays that sweep over the region's admitted
// alignments and returns, per position with a pileup, its reference span, its span-1 column (PileupRecord
// .getAlleleCalls(1)) and, where the span is longer, the span's allele calls clustered into the candidate alleles
// (AlleleCallClustersBuilder.clusterAlleleCalls).  Genotyping (KP for the columns, KI for the indel sites) runs on
// the device; the listener's sequential rules (lastIndelEnd / embedded, the SNV fallback) are applied afterwards
// by the host over the device's results (engine.cpp resolve_regions).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ngsep {

// an admitted alignment as the realigner needs it (ReadAlignment fields)
struct RawRead {
    int32_t first = 0, last = 0, flags = 0;
    std::vector<int32_t> ops;          // NGSEP CIGAR codes len * 8 + op
    std::string chars;                 // upper case (empty: no characters)
    std::string quals;                 // phred + 33 (empty: no qualities)
    bool has_chars = false, has_quals = false;
    int16_t ignore_start = 0, ignore_end = 0;   // bases to ignore at the alignment's start / end (ignore5/3 by strand)
};

// one allele call of an indel site (PileupAlleleCall with span > 1)
struct ICall {
    int32_t off;                       // chars / quals offset in the site's text
    int32_t len;
    int32_t neg;
};

// what one position of a region contributes
struct RegionPos {
    int32_t pos = 0;                   // 1-based
    int32_t span = 1;                  // the realigner's reference span
    bool str = false, new_str = false;
    int32_t col_off = -1, col_len = 0; // span-1 column (u16 entries) in RegionOut::cols (-1: no non-reference call: hom-ref)
    int32_t indel = -1;                // index of its indel site (span > 1 and calls present)
};

// an indel site for KI: the clustered alleles (reference first) and the span's allele calls in pileup order
struct IndelSite {
    int32_t pos = 0;
    std::vector<std::string> alleles;
    std::string text;                  // the calls' alleles, then their qualities
    std::vector<ICall> calls;
};

struct RegionOut {
    int32_t seq_id = -1;
    int64_t first = 0, last = 0;       // the region (1-based, inclusive)
    std::vector<RegionPos> pos;        // positions with a pileup, ascending
    std::vector<uint16_t> cols;        // the columns, each padded to a multiple of 4 entries
    std::vector<IndelSite> sites;
};

struct RealignParams {
    int32_t max_base_qs = 30;          // -maxBaseQS (byte, as the listener passes it)
    bool ignore_lowercase = false;     // the column's reference code (non-callable lower case: no column)
};

// replays AlignmentsPileupGenerator + IndelRealignerPileupListener over [first, last] of one sequence; `reads` are
// the admitted alignments overlapping it in pending-list order (edited in place)
void realign_region(const std::string& ref, int32_t seq_id, int64_t first, int64_t last, std::vector<RawRead>& reads,
                    const RealignParams& p, RegionOut& out);

}  // namespace ngsep
