/*
 * ngsep_oracle.h -- CPU restatement of NGSEP's SNV pileup-calling path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X product path (libngsep_amd.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * Parity pin: the reference (Java, NGSEPcore 4.3.2) cannot be compiled or run
 * in this image (no JDK/JRE).  The restatement is pinned by
 *   - the CountsHelperTest inputs (test/ngsep/discovery/test/CountsHelperTest.java:12-87)
 *     with the expected values derived in SURVEY.md section 4,
 *   - closed-form known-answer tests (all-Q30 pileups),
 *   - a plausibility fixture extracted from training/yeastDemo_*.vcf.gz.
 * See DESIGN.md "Oracle" for what this does and does not pin.
 */
#ifndef NGSEP_ORACLE_H
#define NGSEP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGO_MAX_ALLELES 16

/* Mirrors SingleSampleVariantsDetector / AlignmentsPileupGenerator options.
 * Defaults: SingleSampleVariantsDetector.java:65-78, CountsHelper.java:42-48,
 * AlignmentsPileupGenerator.java:40,53-58. */
typedef struct ngo_params {
    int32_t min_mq;                /* -minMQ (20) */
    int32_t max_alns_per_start;    /* -maxAlnsPerStartPos (5) */
    int32_t ignore5;               /* -ignore5 (0) */
    int32_t ignore3;               /* -ignore3 (0) */
    int32_t max_base_qs;           /* -maxBaseQS (30) */
    int32_t min_quality;           /* -minQuality (40) */
    int32_t ploidy;                /* -ploidy (2) */
    int32_t process_nonunique;     /* -p */
    int32_t process_secondary;     /* -s */
    int32_t ignore_lowercase_ref;  /* -ignoreLowerCaseRef */
    int32_t call_embedded;         /* -embeddedSNVs */
    int32_t calc_strand_bias;      /* -csb */
    int32_t print_sample_ploidy;   /* -psp */
    int32_t het_rate_set;          /* 1 if -h was given */
    double  het_rate;              /* -h (0.001; 1e-6 for haploids if not set) */
    const char* sample_id;         /* -sampleId ("Sample") */
    const char* query_seq;         /* -querySeq (NULL) */
    int32_t query_first;           /* -first (0) */
    int32_t query_last;            /* -last (1e9) */
    int32_t indel_passthrough;     /* 1: reads with I/D are admitted and the indel realigner is a pass-through
                                      (IndelRealignerPileupListener.java:85-126 without its events): the SNV
                                      calls are the reference's only outside the realigner's windows -- what
                                      the GPU path's carved regions leave (tests/test_gpu_indels.py) */
    const char* known_vcf;         /* -knownVariants (NULL): genotype these biallelic SNVs instead of discovering */
    const char* known_strs;        /* -knownSTRs (NULL): regions "seq first last" given to the indel realigner as input
                                      STR variants (SingleSampleVariantsDetector.findSNVS :906-912); ignored with
                                      -knownVariants, as there */
} ngo_params;

void ngo_params_default(ngo_params* p);

/* ---- CountsHelper restatement (CountsHelper.java:40-251,410-495) ---- */
typedef struct ngo_counts {
    int n_alleles;
    int f, g;                 /* heterozygous-proportion bins (CountsHelper.java:212-213) */
    int max_base_qs;
    int total_count;
    int low_bq_count;
    int counts[NGO_MAX_ALLELES];
    int counts_strand[NGO_MAX_ALLELES][2];
    double allele_error_log_probs[NGO_MAX_ALLELES];
    double logc[NGO_MAX_ALLELES][NGO_MAX_ALLELES];
} ngo_counts;

void ngo_counts_init(ngo_counts* c, int n_alleles, double het_proportion, int max_base_qs);
/* allele_idx < 0 means "not one of the helper's alleles" (e.g. N) */
void ngo_counts_update(ngo_counts* c, int allele_idx, int qual_score, int negative_strand);
/* 16-event posterior, CountsHelper.getPosteriorProbabilities(h) for n alleles */
void ngo_counts_posteriors(const ngo_counts* c, double het_rate, double* post /* n*n row-major */);
/* PhredScoreHelper.calculatePhredScore (math/PhredScoreHelper.java:31-40) */
int ngo_phred(double p);
/* Java Math.round for doubles */
int64_t ngo_java_round(double x);
/* FisherExactTest.calculatePValue (math/FisherExactTest.java:65-101) */
double ngo_fisher_pvalue(int a, int b, int c, int d);
/* logProbCache tables (CountsHelper.java:135-187) for n alleles, het bin f */
double ngo_table_error(int q, int j);
double ngo_table_gt(int f, int q, int j);

/* ---- whole path: SAM + FASTA -> VCF (SingleSampleVariantsDetector.findSNVS) ---- */
typedef struct ngo_stats {
    int64_t alignments_read;
    int64_t alignments_admitted;
    int64_t positions_genotyped;   /* pileups with >=1 overlapping admitted alignment */
    int64_t variants_called;
    double  seconds;
} ngo_stats;

/* Returns 0 on success. out_vcf may be "-" for stdout.
 * dump_path (optional, may be NULL): per-position TSV dump of the sufficient statistics
 * (pos, DP, counts[4], logc upper triangle) for every genotyped position with totalCount>0. */
int ngo_run_ssvd(const char* fasta, const char* sam, const char* out_vcf,
                 const char* dump_path, const ngo_params* p, ngo_stats* stats);

/* MultisampleVariantsDetector (discovery/MultisampleVariantsDetector.java:421-693), SNV-only inputs,
 * samples from the @RG SM tags of one SAM file (the generator's merge of per-sample files).
 * p->min_quality is -minQuality; per-sample calls use the fresh listener's DEF_MIN_QUALITY 40. */
int ngo_run_mvd(const char* fasta, const char* sam, const char* out_vcf, const ngo_params* p,
                double min_allele_depth_freq, ngo_stats* stats);

/* CoverageStatisticsCalculator (discovery/CoverageStatisticsCalculator.java:108-216): per-position
 * numAlignments / numUniqueAlns histograms; out_txt gets printCoverageStats' text ("-" = stdout). */
typedef struct ngo_coverage {
    int max_coverage;              /* maxCoverage (300) */
    int64_t* counts;               /* coverageCounts[max_coverage] */
    int64_t* counts_unique;        /* coverageCountUniqueAlignments[max_coverage] */
    int64_t high, high_unique;     /* highCoverageCount, highCoverageCountUniqueAlignments */
} ngo_coverage;
int ngo_run_coverage(const char* fasta, const char* sam, const char* out_txt, int min_mq, int max_coverage,
                     int64_t* counts, int64_t* counts_unique, int64_t* high, int64_t* high_unique, ngo_stats* stats);

/* RelativeAlleleCountsCalculator (discovery/RelativeAlleleCountsCalculator.java:183-331): printResults' text
 * into out_txt ("-" = stdout).  Defaults: min_rd 10, max_rd 1000 (maxAlnsPerStartPos), min_bq 20. */
int ngo_run_rac(const char* fasta, const char* sam, const char* out_txt, int min_rd, int max_rd, int min_bq,
                int secondary, ngo_stats* stats);

/* DecimalFormat("##0.0#") with HALF_EVEN (main/io/ParseUtils.java:29) */
int ngo_java_fmt2(double x, char* buf, int cap);
/* INFO of a population record: NS, AN, AFS, OH, MAF (biallelic) from the calls' (n_called, called[2], acn[4]) */
int ngo_population_info(int n_calls, const int* n_called, const int* called, const int* acn, int n_alleles,
                        char* buf, int cap);

#ifdef __cplusplus
}
#endif
#endif
