// cli.cpp -- `ngsep-amd SingleSampleVariantsDetector ...`: same option names and defaults as
// `java -jar NGSEPcore.jar SingleSampleVariantsDetector` (main/CommandsDescriptor.xml:565-703,
// SingleSampleVariantsDetector.main/run :583-656).  Options of the SV/CNV analyses
// (-runRD, -runRP, -runRep, -runLongReadSVs, ...) are outside this build and rejected.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ngsep_gpu.h"

// regions around indel-bearing alignments that the device path left uncalled (ngsep_fetch_carved_regions):
// written as BED next to the output for the caller's own indel path, with a warning
static void report_carved(ngsep_ctx* c, const std::string& prefix) {
    int64_t n = 0;
    ngsep_fetch_carved_regions(c, nullptr, nullptr, nullptr, 0, &n);
    if (n == 0) return;
    std::vector<int32_t> sid((size_t)n);
    std::vector<int64_t> a((size_t)n), b((size_t)n);
    ngsep_fetch_carved_regions(c, sid.data(), a.data(), b.data(), n, &n);
    const std::string path = prefix + ".carved.bed";
    FILE* f = std::fopen(path.c_str(), "w");
    int64_t total = 0;
    for (int64_t k = 0; k < n; k++) {
        if (f) std::fprintf(f, "%s\t%lld\t%lld\n", ngsep_sequence_name(c, sid[(size_t)k]), (long long)a[(size_t)k] - 1, (long long)b[(size_t)k]);
        total += b[(size_t)k] - a[(size_t)k] + 1;
    }
    if (f) std::fclose(f);
    std::fprintf(stderr, "warning: %lld regions (%lld bp) around alignments with indels were not called on the GPU "
                 "(the indel realigner's reach); listed in %s\n", (long long)n, (long long)total, path.c_str());
}

static int usage(const char* argv0) {
    std::fprintf(stderr,
                 "usage: %s SingleSampleVariantsDetector -i <alignments.bam> -r <reference.fa> -o <output prefix> [options]\n"
                 "options: -sampleId S -ploidy N -psp -minMQ N -maxAlnsPerStartPos N -p -s -ignore5 N -ignore3 N\n"
                 "         -h RATE -maxBaseQS N -minQuality N -ignoreLowerCaseRef -embeddedSNVs -csb\n"
                 "         -querySeq SEQ -first N -last N -knownVariants VCF -device N\n", argv0);
    return 2;
}

// `ngsep-amd MultisampleVariantsDetector -r REF -o OUT.vcf [options] BAM...`
// (MultisampleVariantsDetector.main/run, discovery/MultisampleVariantsDetector.java:412-459)
static int main_mvd(int argc, char** argv, int i) {
    ngsep_params p;
    ngsep_params_default(&p);
    p.multisample = 1;
    const char *ref = nullptr, *outp = "variants.vcf", *known = nullptr, *strs = nullptr;
    int device = 0;
    std::vector<const char*> bams;
    for (; i < argc; i++) {
        const char* a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
        auto takes = [&](const char* name) { if (std::strcmp(a, name) == 0 && v) { i++; return true; } return false; };
        if (takes("-r")) ref = v;
        else if (takes("-o")) outp = v;
        else if (takes("-ploidy")) p.ploidy = std::atoi(v);
        else if (takes("-minMQ")) p.min_mq = std::atoi(v);
        else if (takes("-maxAlnsPerStartPos")) p.max_alns_per_start = std::atoi(v);
        else if (takes("-ignore5")) p.ignore5 = std::atoi(v);
        else if (takes("-ignore3")) p.ignore3 = std::atoi(v);
        else if (takes("-h")) { p.het_rate = std::atof(v); p.het_rate_set = 1; }
        else if (takes("-maxBaseQS")) p.max_base_qs = std::atoi(v);
        else if (takes("-minQuality")) p.min_quality = std::atoi(v);
        else if (takes("-minAlleleDepthFrequency")) p.min_allele_depth_freq = std::atof(v);
        else if (takes("-querySeq")) std::snprintf(p.query_seq, sizeof p.query_seq, "%s", v);
        else if (takes("-first")) p.query_first = std::atoi(v);
        else if (takes("-last")) p.query_last = std::atoi(v);
        else if (takes("-device")) device = std::atoi(v);
        else if (takes("-knownVariants")) known = v;    // MultisampleVariantsDetector.setKnownVariantsFile (:193-195)
        else if (takes("-knownSTRs")) strs = v;         // the realigner's input STRs without -knownVariants (:439-446)
        else if (!std::strcmp(a, "-embeddedSNVs")) p.call_embedded = 1;
        else if (!std::strcmp(a, "-psp")) p.print_sample_ploidy = 1;
        else if (!std::strcmp(a, "-p")) p.process_nonunique = 1;
        else if (!std::strcmp(a, "-s")) p.process_secondary = 1;
        else if (!std::strcmp(a, "-ignoreLowerCaseRef")) p.ignore_lowercase_ref = 1;
        else if (a[0] == '-') { std::fprintf(stderr, "unknown or unsupported option %s\n", a); return 2; }
        else bams.push_back(a);
    }
    if (!ref || bams.empty()) {
        std::fprintf(stderr, "usage: ngsep-amd MultisampleVariantsDetector -r <reference.fa> -o <out.vcf> [options] <BAM>...\n");
        return 2;
    }
    ngsep_ctx* c = nullptr;
    int rc = ngsep_open(device, &p, &c);
    if (rc == NGSEP_OK) rc = ngsep_load_fasta(c, ref);
    if (rc == NGSEP_OK && known) rc = ngsep_set_known_variants(c, known);
    else if (rc == NGSEP_OK && strs) rc = ngsep_set_known_strs(c, strs);
    if (rc == NGSEP_OK) rc = ngsep_call_population_bams(c, bams.data(), (int32_t)bams.size(), outp);
    if (rc != NGSEP_OK) { std::fprintf(stderr, "error %d: %s\n", rc, c ? ngsep_last_error(c) : "open failed"); if (c) ngsep_close(c); return 1; }
    ngsep_stats st;
    ngsep_get_stats(c, &st);
    std::fprintf(stderr, "alignments=%lld admitted=%lld positions=%lld candidates=%lld variants=%lld\n",
                 (long long)st.alignments_in, (long long)st.alignments_admitted, (long long)st.positions_genotyped,
                 (long long)st.candidates, (long long)st.sites_called);
    report_carved(c, outp);
    ngsep_close(c);
    return 0;
}

// `ngsep-amd CoverageStats -i BAM [-o OUT] [-r REF] [-minMQ N]`
// (CoverageStatisticsCalculator.main/run, discovery/CoverageStatisticsCalculator.java:93-122,
// main/CommandsDescriptor.xml:458-477): writes to standard output unless -o is given
static int main_coverage(int argc, char** argv, int i) {
    ngsep_params p;
    ngsep_params_default(&p);
    p.coverage_stats = 1;
    p.process_secondary = 1;
    p.max_alns_per_start = 100;
    const char *in = nullptr, *ref = nullptr, *outp = "-";
    int device = 0;
    for (; i < argc; i++) {
        const char* a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
        auto takes = [&](const char* name) { if (std::strcmp(a, name) == 0 && v) { i++; return true; } return false; };
        if (takes("-i")) in = v;
        else if (takes("-o")) outp = v;
        else if (takes("-r")) ref = v;
        else if (takes("-minMQ")) p.min_mq = std::atoi(v);
        else if (takes("-device")) device = std::atoi(v);
        else { std::fprintf(stderr, "unknown or unsupported option %s\n", a); return 2; }
    }
    if (!in) {
        std::fprintf(stderr, "The alignments input file is a required parameter\n"
                             "usage: ngsep-amd CoverageStats -i <alignments.bam> [-o <out.txt>] [-r <reference.fa>] [-minMQ N]\n");
        return 2;
    }
    ngsep_ctx* c = nullptr;
    int rc = ngsep_open(device, &p, &c);
    if (rc == NGSEP_OK && ref) rc = ngsep_load_fasta(c, ref);
    if (rc == NGSEP_OK) rc = ngsep_coverage_bam(c, in, outp);
    if (rc != NGSEP_OK) { std::fprintf(stderr, "error %d: %s\n", rc, c ? ngsep_last_error(c) : "open failed"); if (c) ngsep_close(c); return 1; }
    ngsep_close(c);
    return 0;
}

// `ngsep-amd RelativeAlleleCounts -i BAM [-o OUT] [-r REF] [-minRD N] [-maxRD N] [-minBQ N] [-s]`
// (RelativeAlleleCountsCalculator.main/run, discovery/RelativeAlleleCountsCalculator.java:175-211):
// writes to standard output unless -o is given
static int main_rac(int argc, char** argv, int i) {
    ngsep_params p;
    ngsep_params_default(&p);
    p.relative_allele_counts = 1;
    p.max_alns_per_start = 1000;            // DEF_MAX_RD
    const char *in = nullptr, *ref = nullptr, *outp = "-";
    int device = 0;
    for (; i < argc; i++) {
        const char* a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
        auto takes = [&](const char* name) { if (std::strcmp(a, name) == 0 && v) { i++; return true; } return false; };
        if (takes("-i")) in = v;
        else if (takes("-o")) outp = v;
        else if (takes("-r")) ref = v;
        else if (takes("-minRD")) p.rac_min_rd = std::atoi(v);
        else if (takes("-maxRD")) p.max_alns_per_start = std::atoi(v);
        else if (takes("-minBQ")) p.rac_min_bq = std::atoi(v);
        else if (std::strcmp(a, "-s") == 0) p.process_secondary = 1;
        else if (takes("-device")) device = std::atoi(v);
        else { std::fprintf(stderr, "unknown or unsupported option %s\n", a); return 2; }
    }
    if (!in) {
        std::fprintf(stderr, "The alignments input file is a required parameter\n"
                             "usage: ngsep-amd RelativeAlleleCounts -i <alignments.bam> [-o <out.txt>] [-r <reference.fa>] [-minRD N] [-maxRD N] [-minBQ N] [-s]\n");
        return 2;
    }
    ngsep_ctx* c = nullptr;
    int rc = ngsep_open(device, &p, &c);
    if (rc == NGSEP_OK && ref) rc = ngsep_load_fasta(c, ref);
    if (rc == NGSEP_OK) rc = ngsep_rac_bam(c, in, outp);
    if (rc != NGSEP_OK) { std::fprintf(stderr, "error %d: %s\n", rc, c ? ngsep_last_error(c) : "open failed"); if (c) ngsep_close(c); return 1; }
    ngsep_close(c);
    return 0;
}

int main(int argc, char** argv) {
    ngsep_params p;
    ngsep_params_default(&p);
    const char *in = nullptr, *ref = nullptr, *outp = nullptr, *known = nullptr, *strs = nullptr;
    int device = 0;
    int i = 1;
    if (i < argc && std::strcmp(argv[i], "MultisampleVariantsDetector") == 0) return main_mvd(argc, argv, i + 1);
    if (i < argc && std::strcmp(argv[i], "CoverageStats") == 0) return main_coverage(argc, argv, i + 1);
    if (i < argc && std::strcmp(argv[i], "RelativeAlleleCounts") == 0) return main_rac(argc, argv, i + 1);
    if (i < argc && std::strcmp(argv[i], "SingleSampleVariantsDetector") == 0) i++;
    else if (i < argc && argv[i][0] != '-') { std::fprintf(stderr, "unsupported command %s\n", argv[i]); return usage(argv[0]); }
    for (; i < argc; i++) {
        const char* a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
        auto takes = [&](const char* name) { if (std::strcmp(a, name) == 0 && v) { i++; return true; } return false; };
        if (takes("-i")) in = v;
        else if (takes("-r")) ref = v;
        else if (takes("-o")) outp = v;
        else if (takes("-sampleId")) std::snprintf(p.sample_id, sizeof p.sample_id, "%s", v);
        else if (takes("-ploidy")) p.ploidy = std::atoi(v);
        else if (takes("-minMQ")) p.min_mq = std::atoi(v);
        else if (takes("-maxAlnsPerStartPos")) p.max_alns_per_start = std::atoi(v);
        else if (takes("-ignore5")) p.ignore5 = std::atoi(v);
        else if (takes("-ignore3")) p.ignore3 = std::atoi(v);
        else if (takes("-h")) { p.het_rate = std::atof(v); p.het_rate_set = 1; }
        else if (takes("-maxBaseQS")) p.max_base_qs = std::atoi(v);
        else if (takes("-minQuality")) p.min_quality = std::atoi(v);
        else if (takes("-querySeq")) std::snprintf(p.query_seq, sizeof p.query_seq, "%s", v);
        else if (takes("-first")) p.query_first = std::atoi(v);
        else if (takes("-last")) p.query_last = std::atoi(v);
        else if (takes("-device")) device = std::atoi(v);
        else if (takes("-knownVariants")) known = v;
        else if (takes("-knownSTRs")) strs = v;
        else if (!std::strcmp(a, "-psp")) p.print_sample_ploidy = 1;
        else if (!std::strcmp(a, "-p")) p.process_nonunique = 1;
        else if (!std::strcmp(a, "-s")) p.process_secondary = 1;
        else if (!std::strcmp(a, "-ignoreLowerCaseRef")) p.ignore_lowercase_ref = 1;
        else if (!std::strcmp(a, "-embeddedSNVs")) p.call_embedded = 1;
        else if (!std::strcmp(a, "-csb")) p.calc_strand_bias = 1;
        else { std::fprintf(stderr, "unknown or unsupported option %s\n", a); return usage(argv[0]); }
    }
    if (!in || !ref || !outp) return usage(argv[0]);
    ngsep_ctx* c = nullptr;
    int rc = ngsep_open(device, &p, &c);
    if (rc != NGSEP_OK) { std::fprintf(stderr, "error: %s\n", c ? ngsep_last_error(c) : "open failed"); return 1; }
    rc = ngsep_load_fasta(c, ref);
    if (rc == NGSEP_OK && known) rc = ngsep_set_known_variants(c, known);
    else if (rc == NGSEP_OK && strs) rc = ngsep_set_known_strs(c, strs);   // (:897-912: -knownVariants first)
    std::string vcf = std::string(outp) + ".vcf";
    if (rc == NGSEP_OK) rc = ngsep_call_bam(c, in, vcf.c_str());
    if (rc != NGSEP_OK) { std::fprintf(stderr, "error %d: %s\n", rc, ngsep_last_error(c)); ngsep_close(c); return 1; }
    ngsep_stats st;
    ngsep_get_stats(c, &st);
    std::fprintf(stderr, "alignments=%lld admitted=%lld positions=%lld candidates=%lld variants=%lld\n",
                 (long long)st.alignments_in, (long long)st.alignments_admitted, (long long)st.positions_genotyped,
                 (long long)st.candidates, (long long)st.sites_called);
    report_carved(c, outp);
    ngsep_close(c);
    return 0;
}
