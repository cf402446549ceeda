// realign.hpp -- the indel realigner's regions on the host (realign.cpp).  Internal to libngsep_amd.so.
//
// A region is the reach of the reference's IndelRealignerPileupListener around alignments with indels
// (discovery/IndelRealignerPileupListener.java:85-526): inside it the listener edits alignments (moves indel
// starts, realigns and trims alignment ends) while the pileup sweep goes on, so every pileup of the region is
// taken from the alignments as edited so far.  replay_region replays that sweep over the region's admitted
// alignments and returns, per position with a pileup, its reference span, its span-1 column (PileupRecord
// .getAlleleCalls(1), the device's u16 column entries: genotyped by KP like every other position) and, where the
// span is longer, the span's indel call (AlleleCallClustersBuilder + CountsHelper indel counts + callIndel: a few
// sites per kilobase of region, genotyped here).  resolve_region then applies the listener's sequential rules
// (SingleSampleVariantPileupListener.onPileup :146-161, discoverVariant :213-273: lastIndelEnd, embedded SNVs,
// the SNV fallback of a span whose alleles made no call) over the device's SNV calls.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace ngsep {

// an admitted alignment as the realigner needs it (ReadAlignment fields), in admission (pending-list) order
// the bytes of a run of kept alignments (engine.cpp keep_raw: one block per slice of reads, shared by their RawReads)
struct RawBlock {
    std::unique_ptr<char[]> bytes;
};
struct RawRead {
    int32_t first = 0, last = 0, flags = 0;
    int32_t n_ops = 0, len = 0;        // CIGAR items; read characters (and qualities) held
    const int32_t* ops = nullptr;      // NGSEP CIGAR codes len * 8 + op
    const char* chars = nullptr;       // read characters (nullptr: getReadCharacters() == null)
    const char* quals = nullptr;       // phred + 33 (nullptr: '*')
    int32_t ignore_start = 0, ignore_end = 0;   // setBasesToIgnore5P/3P by strand (ReadAlignment.java:613-644)
    int16_t sample = -1;               // multisample: the sample of the read group (-1: none), and the read group's rank
    uint8_t rank = 0;                  //   in the sample's HashSet order (PileupRecord.getAlleleCalls(span, readGroups))
    std::shared_ptr<const RawBlock> hold;   // keeps ops / chars / quals alive (a copy is a view, not a deep copy)
};

struct RealignParams {
    int32_t max_base_qs = 30;          // -maxBaseQS
    int32_t min_quality = 40;          // -minQuality
    int32_t ploidy = 2;
    double het_rate = 0.001;           // -h
    bool ignore_lowercase = false;     // -ignoreLowerCaseRef
    int32_t n_samples = 0;             // > 0: MultisampleVariantsDetector's listener (population mode)
    bool known = false;                // -knownVariants: the listeners genotype the input variants (no discovery)
};

// a decided indel / STR call (callIndel + the listener's filters), its VCF line already formatted
struct IndelCall {
    int32_t pos = 0, last = 0;         // first, first + |REF| - 1
    std::string line;                  // without the sequence name: "POS\t.\tREF\tALT\t..." + '\n'
};

// what one position of a region contributes
struct RegionPos {
    int32_t pos = 0;                   // 1-based
    int32_t span = 1;                  // the realigner's reference span
    bool str = false, new_str = false; // input STR = str && !new_str (PileupRecord.isInputSTR)
    bool var_embedded = false;         // inside an input STR past its first position (the realigner's setEmbedded)
    int32_t col_off = 0, col_len = 0;  // span-1 column: u16 entries code | negative strand << 8 in RegionOut::cols
    int32_t indel = -1;                // span > 1: index into RegionOut::indels of the span's call (-1: none)
    bool blocked = false;              // no call at all (span past the sequence end, lower-case reference ignored)
    bool nonref = false;               // the span-1 column holds a valid call of another allele than the reference base
    int32_t pcol = -1;                 // population mode: its span-1 columns, samples 0 .. S - 1 then the reads of no
                                       // sample: RegionOut::pcodes[poff[pcol + s] .. poff[pcol + s + 1])
    int32_t pindel = -1;               // population mode, span > 1: index into RegionOut::pindels when
                                       // discoverPopulationVariantWithSpan found an indel variant (-1: null)
};

// MultisampleVariantsDetector's indel / STR variant at a span (discoverPopulationIndel non-null): genotyped again by
// onPileup (genotypeVariant, :532) -- written iff its QS passes, and never followed by the SNV fallback
struct PopIndel {
    bool pass = false;                 // QS > 0 and >= minQuality (MultisampleVariantsDetector.java:533)
    int32_t qs = 0, last = 0;          // the variant QS; first + |REF| - 1 (lastIndelEnd when written)
    std::string line;                  // the record without the sequence name: "POS\t.\tREF\tALT\t..." + '\n'
};

// -knownVariants: a genotyped input indel / MNP / other non-SNV record (a GenomicVariantImpl of VCFFileReader
// .loadGenomicVariant, :249-253) -- its record, written whatever the genotype (the known index orders records that
// share a position)
struct KnownCall {
    int32_t pos = 0;
    int64_t known = 0;                 // index of the input variant in the context's sorted list
    std::string line;                  // without the sequence name
};

struct RegionOut {
    int64_t first = 0, last = 0;       // the region (1-based, inclusive)
    std::vector<RegionPos> pos;        // positions with a pileup, ascending
    std::vector<uint16_t> cols;
    std::vector<IndelCall> indels;
    std::vector<uint8_t> pcodes;       // population mode: the positions' per-sample span-1 codes (engine.hpp codes)
    std::vector<uint32_t> poff;        //   S + 2 offsets per position
    std::vector<PopIndel> pindels;
    std::vector<KnownCall> kcalls;     // -knownVariants: the region's non-SNV input variants, genotyped (position order)
};

// an input variant of the indel realigner (IndelRealignerPileupListener.setInputVariants): a -knownSTRs region
// (SingleSampleVariantsDetector.makeNonRedundantSTRs, TYPE_STR) or a -knownVariants record (findSNVS :897-905,
// MultisampleVariantsDetector.run :432-438); 1-based [first, last]
struct StrVar {
    int32_t first, last;
    bool str = true;                   // TYPE_STR: the pileup at `first` gets the STR flag (:92)
    bool event = true;                 // opens a realigner region (an STR, or a known record that is not an SNV)
    int64_t known = -1;                // -knownVariants, not an SNV: its index in the context's list (genotyped in the region)
    int32_t rec = -1;                  //   and its KnownRecord
};

// the input variants of one sequence in GenomicRegionPositionComparator order (first, then last; stable) and the
// prefix maximum of `last`, so intersectWithVariants' index can be found at any position (replay_region)
struct InputVars {
    std::vector<StrVar> v;
    std::vector<int32_t> pmax;
    void finish() {
        pmax.resize(v.size());
        int32_t m = INT32_MIN;
        for (size_t i = 0; i < v.size(); i++) { m = v[i].last > m ? v[i].last : m; pmax[i] = m; }
    }
};

// a -knownVariants record that is not an SNV, as replay_region genotypes it
struct KnownRecord {
    std::vector<std::string> alleles;  // reference first (upper case)
    std::string id;                    // "" for '.'
    int16_t qs = 0;
    int8_t type = 0;                   // INFO TYPE id (GenomicVariant.TYPE_*): printed when 2-5
};

// replays AlignmentsPileupGenerator + IndelRealignerPileupListener over [first, last] of one sequence (`seq`: the
// reference as loaded, case kept); `reads` are the admitted alignments overlapping it in pending-list order
// (read only); `inputs`: the sequence's realigner input variants (may be null); `knowns`: the records their
// `known` indexes name (p.known)
void replay_region(const std::string& seq, int64_t first, int64_t last, std::vector<RawRead>& reads, const RealignParams& p,
                   const InputVars* inputs, const std::vector<KnownRecord>* knowns, RegionOut& out);

// the listener's decisions over a replayed region, position by position: kind 0 nothing, 1 the position's SNV
// call (flag embedded: TYPE=EMBEDDED), 2 the indel call out.indels[idx].  last_indel_end is the listener's
// lastIndelEnd (per sequence, carried across regions)
struct RegionDecision {
    int32_t pos;
    int8_t kind;
    bool embedded;
    int32_t idx;
};
void resolve_region(const RegionOut& out, const std::vector<uint8_t>& has_snv_call, bool call_embedded, int32_t* last_indel_end,
                    std::vector<RegionDecision>& dec);
// MultisampleVariantsDetector.onPileup's rules (:522-538) over a replayed region in population mode: kind 1 the
// position's population SNV record (has_snv_record: the device wrote one; flag embedded: TYPE=EMBEDDED), 2 the
// indel / STR record out.pindels[idx]
void resolve_population_region(const RegionOut& out, const std::vector<uint8_t>& has_snv_record, bool call_embedded,
                               int32_t* last_indel_end, std::vector<RegionDecision>& dec);

}  // namespace ngsep
