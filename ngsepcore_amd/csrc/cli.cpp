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

// -devices 0,1,...: one context per device, the windows of ngsep_call_bam_multi / ngsep_call_population_bams_multi
// (SURVEY.md 8(e)); empty: the single -device
static std::vector<int> parse_devices(const char* v) {
    std::vector<int> d;
    for (const char* t = v; t && *t;) {
        d.push_back(std::atoi(t));
        t = std::strchr(t, ',');
        if (t) t++;
    }
    return d;
}

// opens one context per device (the first loads the reference and the input variants; the others take them from it)
static int open_contexts(const std::vector<int>& devices, const ngsep_params& p, const char* ref, const char* known,
                         const char* strs, std::vector<ngsep_ctx*>& ctxs) {
    int rc = NGSEP_OK;
    for (int d : devices) {
        ngsep_ctx* c = nullptr;
        rc = ngsep_open(d, &p, &c);
        if (c) ctxs.push_back(c);
        if (rc != NGSEP_OK) return rc;
    }
    rc = ngsep_load_fasta(ctxs[0], ref);
    if (rc == NGSEP_OK && known) rc = ngsep_set_known_variants(ctxs[0], known);
    else if (rc == NGSEP_OK && strs) rc = ngsep_set_known_strs(ctxs[0], strs);   // (:897-912: -knownVariants first)
    return rc;
}

static void print_stats(const std::vector<ngsep_ctx*>& ctxs) {
    long long a = 0, b = 0, q = 0, cnd = 0, v = 0;
    for (ngsep_ctx* c : ctxs) {
        ngsep_stats st;
        ngsep_get_stats(c, &st);
        a += st.alignments_in; b += st.alignments_admitted; q += st.positions_genotyped; cnd += st.candidates; v += st.sites_called;
    }
    std::fprintf(stderr, "alignments=%lld admitted=%lld positions=%lld candidates=%lld variants=%lld\n", a, b, q, cnd, v);
}

static int usage(const char* argv0) {
    std::fprintf(stderr,
                 "usage: %s SingleSampleVariantsDetector -i <alignments.bam> -r <reference.fa> -o <output prefix> [options]\n"
                 "options: -sampleId S -ploidy N -psp -minMQ N -maxAlnsPerStartPos N -p -s -ignore5 N -ignore3 N\n"
                 "         -h RATE -maxBaseQS N -minQuality N -ignoreLowerCaseRef -embeddedSNVs -csb\n"
                 "         -querySeq SEQ -first N -last N -knownVariants VCF -knownSTRs FILE -device N\n"
                 "         -devices N,N,... [-window BP]   (several GPUs of this process: windows from one queue)\n", argv0);
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
    std::vector<int> devices;
    long long window = 4 << 20;
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
        else if (takes("-devices")) devices = parse_devices(v);
        else if (takes("-window")) window = std::atoll(v);
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
    if (devices.empty()) devices.push_back(device);
    std::vector<ngsep_ctx*> ctxs;
    int rc = open_contexts(devices, p, ref, known, strs, ctxs);
    if (rc == NGSEP_OK)
        rc = ctxs.size() == 1 ? ngsep_call_population_bams(ctxs[0], bams.data(), (int32_t)bams.size(), outp)
                              : ngsep_call_population_bams_multi(ctxs.data(), (int32_t)ctxs.size(), bams.data(),
                                                                 (int32_t)bams.size(), outp, window);
    if (rc != NGSEP_OK) {
        std::fprintf(stderr, "error %d: %s\n", rc, ctxs.empty() ? "open failed" : ngsep_last_error(ctxs[0]));
        for (ngsep_ctx* c : ctxs) ngsep_close(c);
        return 1;
    }
    print_stats(ctxs);
    report_carved(ctxs[0], outp);
    for (ngsep_ctx* c : ctxs) ngsep_close(c);
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
    std::vector<int> devices;
    long long window = 4 << 20;
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
        else if (takes("-devices")) devices = parse_devices(v);
        else if (takes("-window")) window = std::atoll(v);
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
    if (devices.empty()) devices.push_back(device);
    if (devices.size() > 1 && p.query_seq[0]) {
        std::fprintf(stderr, "-devices runs the whole file (windows over every sequence): without -querySeq\n");
        return 2;
    }
    std::vector<ngsep_ctx*> ctxs;
    int rc = open_contexts(devices, p, ref, known, strs, ctxs);
    std::string vcf = std::string(outp) + ".vcf";
    if (rc == NGSEP_OK)
        rc = ctxs.size() == 1 ? ngsep_call_bam(ctxs[0], in, vcf.c_str())
                              : ngsep_call_bam_multi(ctxs.data(), (int32_t)ctxs.size(), in, vcf.c_str(), window);
    if (rc != NGSEP_OK) {
        std::fprintf(stderr, "error %d: %s\n", rc, ctxs.empty() ? "open failed" : ngsep_last_error(ctxs[0]));
        for (ngsep_ctx* c : ctxs) ngsep_close(c);
        return 1;
    }
    print_stats(ctxs);
    report_carved(ctxs[0], outp);
    for (ngsep_ctx* c : ctxs) ngsep_close(c);
    return 0;
}
