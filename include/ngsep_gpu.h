/*
 * ngsep_gpu.h -- C ABI of the MI355X-native NGSEP SNV pileup caller (libngsep_amd.so).
 *
 * Drop-in boundary for the reference's SingleSampleVariantsDetector path:
 *   Java caller (JNI shim) or the bundled CLI/Python host
 *        |  plain pointers + sizes, caller-owned buffers, int status codes
 *        v
 *   host admission sweep + reference projection (C++)  ->  HBM-resident read SoA
 *        v
 *   HIP kernels on gfx950 (K1 candidate scan, K2 SNVQ genotyping)
 *
 * Every entry point names the reference interface it replaces
 * (paths relative to src/ngsep/ of acastem15/NGSEPcore 4.3.2).
 *
 * Conventions: 0 = success, negative = error (see NGSEP_E_*); after an error
 * ngsep_last_error(ctx) returns a message.  One context per device per host
 * thread; contexts are independent (re-entrant across contexts).
 */
#ifndef NGSEP_GPU_H
#define NGSEP_GPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGSEP_ABI_VERSION 12

#define NGSEP_OK 0
#define NGSEP_E_INVALID (-1)      /* bad argument / state */
#define NGSEP_E_IO (-2)           /* file cannot be read or written */
#define NGSEP_E_FORMAT (-3)       /* malformed BAM / FASTA */
#define NGSEP_E_DEVICE (-4)       /* HIP runtime error or no device */
#define NGSEP_E_UNSUPPORTED (-5)  /* input outside the implemented path (ploidy > 128, > 255 samples, ...) */
#define NGSEP_E_NOMEM (-6)

typedef struct ngsep_ctx ngsep_ctx;

/* Options of SingleSampleVariantsDetector (main/CommandsDescriptor.xml:565-703);
 * defaults are the DEF_* constants (SingleSampleVariantsDetector.java:65-78,
 * CountsHelper.java:42-48, AlignmentsPileupGenerator.java:40,53-58). */
typedef struct ngsep_params {
    int32_t min_mq;               /* -minMQ                 20 */
    int32_t max_alns_per_start;   /* -maxAlnsPerStartPos    5  */
    int32_t ignore5;              /* -ignore5               0  */
    int32_t ignore3;              /* -ignore3               0  */
    int32_t max_base_qs;          /* -maxBaseQS             30 */
    int32_t min_quality;          /* -minQuality            40 */
    int32_t ploidy;               /* -ploidy                2  */
    int32_t process_nonunique;    /* -p                     0  */
    int32_t process_secondary;    /* -s                     0  */
    int32_t ignore_lowercase_ref; /* -ignoreLowerCaseRef    0  */
    int32_t call_embedded;        /* -embeddedSNVs          0  */
    int32_t calc_strand_bias;     /* -csb                   0  */
    int32_t print_sample_ploidy;  /* -psp                   0  */
    int32_t het_rate_set;         /* 1 if -h was given (haploid default switch, :591-593) */
    double  het_rate;             /* -h                     0.001 */
    int32_t query_first;          /* -first                 0 (used only with query_seq) */
    int32_t query_last;           /* -last                  1e9 */
    char    query_seq[256];       /* -querySeq              "" = all */
    char    sample_id[256];       /* -sampleId              "Sample" */
    /* engine knobs (no reference counterpart) */
    int32_t prune_candidates;     /* 1: exact non-candidate pruning (DESIGN.md "K1"), 0: genotype every position */
    int32_t dump_all_positions;   /* 1: ngsep_fetch_sites returns a record for every position with DP>0 */
    int32_t window_positions;     /* max positions per device window (0 = whole contig) */
    /* MultisampleVariantsDetector (discovery/MultisampleVariantsDetector.java:54-95) */
    int32_t multisample;          /* 1: population calling over the samples of ngsep_set_samples */
    double  min_allele_depth_freq;/* -minAlleleDepthFrequency 0 (setMinAlleleDepthFrequency, :398-403) */
    /* CoverageStatisticsCalculator (discovery/CoverageStatisticsCalculator.java:37-51,108-122): the caller
     * also sets process_secondary = 1 and max_alns_per_start = 100 as its processFile does */
    int32_t coverage_stats;       /* 1: the alignments feed the coverage histograms instead of the variant caller */
    int32_t max_coverage;         /* maxCoverage 300 (setMaxCoverage): bins [0, max_coverage) + "More"; <= 1024 */
    /* RelativeAlleleCountsCalculator (discovery/RelativeAlleleCountsCalculator.java:28-52,183-211): the caller
     * also sets max_alns_per_start = maxRD (1000) and process_secondary = secondaryAlns as its runProcess does */
    int32_t relative_allele_counts; /* 1: the pileups feed the allele-proportion distributions */
    int32_t rac_min_rd;           /* -minRD 10 */
    int32_t rac_min_bq;           /* -minBQ 20 (4..30 here: the pile's codes keep qualities clamped to 30) */
    /* ABI 5: what a biallelic SNV record carries back from the device.  0 (default): what the reference's
     * CalledSNV keeps (variants/CalledSNV.java:42-45,259-265) -- logc only at (ref,ref), (ref,alt), (alt,alt)
     * and strand_counts only for the reference and alternative alleles, the other entries 0; 1: the whole
     * CountsHelper state (all ten log-conditionals, every strand count).  Multi-allelic, pool and
     * dump_all_positions records are always whole. */
    int32_t full_records;
    /* ABI 6: the indel realigner and indel / STR discovery (IndelRealignerPileupListener + VariantDiscovery-
     * SNVQAlgorithm.callIndel, single-sample discovery at ploidy < 3, streamed runs; ABI 8: also
     * MultisampleVariantsDetector, discoverPopulationIndel; ABI 9: also with -knownVariants, whose records are the
     * realigner's input variants, and at ploidy >= 3 -- the pool algorithm's indel branch, genotypeVariantPool).
     * 0 (default): regions around alignments with indels are realigned and called here (indel / STR records,
     * TYPE=EMBEDDED SNVs with call_embedded); 1: pass-through -- no call inside those regions, which are returned
     * by ngsep_fetch_carved_regions for the caller's own indel path (the ABI 5 behaviour). */
    int32_t indel_passthrough;
} ngsep_params;

/* Alignments as AlignmentsPileupGenerator.processAlignment receives them
 * (AlignmentsPileupGenerator.java:377-403): already filtered by the reader,
 * coordinate-sorted.  Mirrors the ReadAlignment fields the JNI side copies out
 * (alignments/ReadAlignment.java:87-122). */
typedef struct ngsep_read_batch {
    int64_t n_reads;
    const int32_t* seq_id;      /* index of the reference sequence (order of ngsep_set_reference) */
    const int32_t* first;       /* 1-based first aligned reference position (getFirst) */
    const int32_t* flags;       /* SAM flags (0x10 strand, 0x100 secondary are used) */
    const int32_t* read_group;  /* caller's read-group index, -1 = DEF_READ_GROUP "" */
    const int64_t* cigar_off;   /* offset of the read's CIGAR items in cigar[] */
    const int32_t* cigar_n;     /* number of CIGAR items */
    const int32_t* cigar;       /* NGSEP encoding len*8+op, op: H0 D1 I2 M3 P4 N5 S6 X7 (ReadAlignment.java:60-67,1180-1198) */
    const int64_t* seq_off;     /* offset of the read's characters in bases[] and quals[] */
    const int32_t* seq_len;     /* read length; 0 = no read characters (getReadCharacters()==null) */
    const char*    bases;       /* read characters, upper case */
    const char*    quals;       /* phred+33 quality characters (NULL = no qualities for any read) */
    const uint8_t* has_quals;   /* per read: 0 = quality string absent ('*'), may be NULL = all present */
} ngsep_read_batch;

/* One called variant = one VCF data line of SingleSampleVariantsDetector
 * (CalledSNV / triallelic CalledGenomicVariantImpl, VariantDiscoverySNVQAlgorithm.java:100-222). */
typedef struct ngsep_site_out {
    int32_t seq_id;
    int32_t pos;             /* 1-based */
    int8_t  ref;             /* upper-case reference base 'A','C','G','T' */
    int8_t  n_alleles;       /* 2 = biallelic CalledSNV, 3 = MULTISNV (called 1/2) */
    int8_t  alt;             /* DNA index (0=A,1=C,2=G,3=T) of ALT (first ALT if triallelic) */
    int8_t  third;           /* DNA index of the second ALT, or -1 */
    int8_t  genotype;        /* 0 hom-ref (dump mode only), 1 het, 2 hom-alt, 3 het alt/third, -1 none */
    int8_t  strand_bias;     /* FS phred score (-csb) or -1 */
    int16_t gq;              /* genotype quality, PhredScoreHelper.calculatePhredScore(1-maxP) */
    int16_t qual;            /* variant QS, phred(P[ref][ref]) */
    int8_t  is_call;         /* bit 0: passes the listener filters (always set unless dump_all_positions);
                              * bit 2: an SNV inside a called indel (INFO TYPE=EMBEDDED, params.call_embedded);
                              * bit 3: an indel / STR record (ABI 9: or a -knownVariants record that is not an
                              * SNV) -- its fields here are 0 except seq_id / pos, its VCF line comes from
                              * ngsep_site_vcf_line (ABI 6) */
    uint8_t pool;            /* ploidy >= 3 (SingleSampleVariantPileupListener.genotypeVariantPool, :402-503):
                              * bits 0-3 = the variant's alleles as DNA-index bits (reference included; the
                              * alleles are the reference, then the others in A,C,G,T order), bit 4 = the call
                              * report (PL / ADP) is present; 0 = an SNVQ record.  In a pool record n_alleles =
                              * the variant's allele count, genotype = number of called alleles (0 undecided,
                              * 1 homozygous, 2 heterozygous), alt / third = DNA indexes of the called alleles
                              * (-1 when absent), logc = the report's log-conditionals over the variant's alleles
                              * (upper triangle, i <= j < n_alleles, row-major), dp = the pool call's read depth;
                              * ABI 9, -knownVariants: strand_bias = the copy number genotypeVariantPool gave the
                              * first called allele of a heterozygous call (-1 otherwise) */
    int32_t dp;              /* CountsHelper.getTotalCount() */
    int32_t counts[4];       /* A,C,G,T base counts (BSDP) */
    int32_t strand_counts[4][2]; /* [allele][0=negative,1=positive] (CountsHelper.countsStrand); biallelic SNV
                              * records without full_records: the reference and alternative rows only */
    double  logc[10];        /* log10 P(data|genotype) upper triangle: 00 01 02 03 11 12 13 22 23 33; biallelic
                              * SNV records without full_records: (ref,ref), (ref,alt), (alt,alt) only */
} ngsep_site_out;

/* One population VCF line of MultisampleVariantsDetector (VCFRecord.createDefaultPopulationVCFRecord,
 * vcf/VCFRecord.java:277-301): the variant and n_samples ngsep_sample_call records. */
typedef struct ngsep_popsite_out {
    int32_t seq_id;
    int32_t pos;             /* 1-based */
    int8_t  n_alleles;       /* 2..4 (0 for an indel / STR record) */
    int8_t  alleles[4];      /* DNA indexes (0=A..3=T): reference first, then alternatives in A,C,G,T order */
    int8_t  multisnv_type;   /* 1: the pooled multi-allelic SNV kept all its alleles -> INFO TYPE=MULTISNV;
                              * 2 (ABI 8): an SNV inside an indel / STR (-embeddedSNVs) -> TYPE=EMBEDDED;
                              * 3 (ABI 8): an indel / STR record of the realigner's regions (discoverPopulationIndel,
                              * MultisampleVariantsDetector.java:599-634; ABI 9: or a -knownVariants record that is
                              * not an SNV): its alleles and sample calls are only in its VCF line
                              * (ngsep_population_site_vcf_line); its calls[] entries are zeroed */
    int16_t qual;            /* variant QS: max GQ over decided non-reference sample calls (:674-693) */
    int16_t pad;
} ngsep_popsite_out;

/* One sample's genotype call at a population site: CalledSNV (biallelic) or
 * CalledGenomicVariantImpl (multi-allelic / no data), as VCFFileWriter.printGenotypeInfo prints it. */
typedef struct ngsep_sample_call {
    int8_t  kind;            /* 0 CalledSNV, 1 CalledGenomicVariantImpl */
    int8_t  n_called;        /* 0 = undecided ("./."), 1 homozygous, 2 heterozygous */
    int8_t  called[2];       /* indexes into the site's alleles */
    int16_t gq;
    int16_t total_cn;        /* getCopyNumber (ACN "." when 0) */
    int32_t dp;              /* CountsHelper.getTotalCount() of the sample */
    int32_t counts[4];       /* BSDP A,C,G,T */
    int16_t acn[4];          /* getAllelesCopyNumber over the site's alleles */
    int32_t pl[10];          /* PL in VCF order (j-major, i<=j over the site's alleles) */
} ngsep_sample_call;

typedef struct ngsep_stats {
    int64_t alignments_in;          /* alignments received */
    int64_t alignments_admitted;    /* after the maxAlnsPerStartPos cap */
    int64_t positions_genotyped;    /* positions with >=1 overlapping admitted alignment */
    int64_t candidates;             /* positions sent to K2 */
    int64_t sites_called;
    int64_t read_bases;             /* projected read bytes resident in HBM */
    int64_t slot_bytes;             /* multisample: bytes of the population kernel's per-sample pile (incl. padding) */
    double  kernel_ms;              /* host wall time of the last device run (kernels + D2H) */
    double  scan_ms;                /* device time of the tile scan (KT) */
    double  genotype_ms;            /* device time of the posterior kernel */
    int32_t tile_positions;         /* positions per pileup tile (T) */
    int32_t tile_rows_max;          /* largest tile depth (rows of the tile-blocked pileup matrix) */
    int32_t slot_size;              /* bytes per read slot of the read-major SoA */
    int32_t hard_sites;             /* candidates that needed the exact tally + posterior */
    int64_t pile_bytes;             /* bytes of the pileup streamed by the scan (multisample: candidate-column bytes) */
    int64_t exact_bound_passes;     /* wavefront passes of the scan's exact integer hom-ref bound */
    int64_t global_positions;       /* positions of the device coordinate (windows + halos, whole tiles) */
    int64_t n_tiles;                /* pileup tiles (multisample: scan groups of 64 candidate columns) */
    double  layout_ms;              /* host time to build the device layout of the last staged run */
    double  upload_ms;              /* host time of its H2D upload */
    int64_t carved_positions;       /* covered positions inside carved indel regions (not called here) */
    int64_t other_allele_calls;     /* entries of the scan's other-allele lists (valid non-reference calls) */
    double  realign_ms;             /* ABI 10: host wall time of the indel realigner's region replays, summed */
    int64_t realign_regions;        /* ABI 10: realigner regions replayed */
    /* ABI 11: where the indel path's host time goes (path B, single sample; wall times, summed over windows) */
    double  keep_raw_ms;            /* the reader thread keeping the raw alignments a region can need (keep_raw) */
    double  region_setup_ms;        /* the regions' device queue built from the replays (window worker) */
    double  region_device_ms;       /* the regions' span-1 columns genotyped on the device (one more KP run per window) */
    double  region_merge_ms;        /* the listener's span rules and the merge of the region records into the window's */
    double  window_wait_ms;         /* the reader thread waiting for a free window worker (device + regions behind) */
    double  region_gather_ms;       /* the regions' kept alignments gathered for the worker (reader thread) */
} ngsep_stats;

/* ---- -knownVariants (SingleSampleVariantsDetector.findSNVS :896-906, MultisampleVariantsDetector.run :432-438) ---- */
/* Genotype the records of this VCF (VCFFileReader.loadVariants(file, true, true): ALT '.' and structural records
 * skipped) at their covered first positions instead of discovering variants (SingleSampleVariantPileupListener.onPileup
 * with input variants, :158-176; MultisampleVariantsDetector.onPileup :539-551): every input variant with a pileup gets
 * a record (hom-ref, het, hom-alt or undecided; ID, alleles and INFO TYPE kept; QUAL the input's, or the population
 * QS).  Biallelic SNVs are genotyped on the device (genotypeSNV / the pool algorithm); ABI 9: indels, MNPs and other
 * records that are not SNVs are accepted -- they are the indel realigner's fixed events (IndelRealignerPileupListener
 * .setInputVariants, findSNVS :904) and are genotyped in their realigner regions by callIndel with the variant given
 * (genotypeVariantSample :377-386), or by genotypeVariantPool at ploidy >= 3.  Multi-allelic SNVs and records that
 * repeat an allele: E_UNSUPPORTED.  Call after the reference is loaded; NULL or "" returns
 * to discovery; a file with no usable record also discovers (inputVariants.size() == 0, :148).  Once a file is set,
 * ngsep_set_known_strs is ignored (the reference's else-if, :906). */
int  ngsep_set_known_variants(ngsep_ctx* c, const char* vcf_path);   /* ngsep_set_known_variants(c, NULL) clears it */

/* ---- -knownSTRs (ABI 7; SingleSampleVariantsDetector.findSNVS :906-912, makeNonRedundantSTRs :843-894) ----
 * Regions "sequence first last" (1-based, space or tab separated; SimpleGenomicRegionFileHandler.loadRegions) merged
 * into the indel realigner's input STR variants [first - 1, last + 1]: at an STR's first position the pileup takes the
 * STR's span and is genotyped as an STR (TYPE=STR whatever its allele lengths), inside it the pileup is embedded.  Every
 * STR opens a realigner region like an alignment with an indel (ngsep_fetch_carved_regions' geometry).  Single-sample
 * discovery only; -knownVariants takes precedence, as in the reference.  Call after the reference is loaded; NULL or ""
 * clears them. */
int  ngsep_set_known_strs(ngsep_ctx* c, const char* path);

/* ---- RelativeAlleleCountsCalculator (params.relative_allele_counts) ---- */
/* RelativeAlleleCountsCalculator.runProcess + printResults (:183-244) on a BAM: the report text to out_path */
int  ngsep_rac_bam(ngsep_ctx* c, const char* bam_path, const char* out_path);
/* the distributions so far: prop[51] (bins 0, 0.01, .., 0.5), n_alleles[10] (bins 1..10), moments[6] =
 * proportion count, sum, sum of squares, number-of-alleles count, sum, sum of squares (any may be NULL) */
int  ngsep_fetch_rac(ngsep_ctx* c, double* prop, double* n_alleles, double* moments);
/* printResults' text ("-" = stdout) */
int  ngsep_write_rac(ngsep_ctx* c, const char* out_path);
int  ngsep_clear_rac(ngsep_ctx* c);

/* ---- context ---- */
int  ngsep_abi_version(void);
void ngsep_params_default(ngsep_params* p);
/* device: HIP ordinal.  Replaces `new SingleSampleVariantsDetector()` + option setters */
int  ngsep_open(int device, const ngsep_params* params, ngsep_ctx** out);
int  ngsep_close(ngsep_ctx* ctx);
const char* ngsep_last_error(ngsep_ctx* ctx);
int  ngsep_get_stats(ngsep_ctx* ctx, ngsep_stats* out);
int  ngsep_device_count(void);

/* ---- reference: ReferenceGenome(filename, keepLowerCase=true) (genome/ReferenceGenome.java:40-62) ---- */
int ngsep_set_reference(ngsep_ctx* ctx, const char* seq_name, const char* bases, int64_t len);
int ngsep_load_fasta(ngsep_ctx* ctx, const char* path);
int ngsep_n_sequences(ngsep_ctx* ctx);
const char* ngsep_sequence_name(ngsep_ctx* ctx, int seq_id);

/* ---- path A: alignments pushed by the host (AlignmentsPileupGenerator.processAlignments, :334-361) ---- */
int ngsep_process_alignments(ngsep_ctx* ctx, const ngsep_read_batch* batch);
/* AlignmentsPileupGenerator.notifyEndOfAlignments (:447-452): flushes the last sequence */
int ngsep_notify_end(ngsep_ctx* ctx);
/* Calls accumulated so far (SingleSampleVariantPileupListener.getCalledVariants, :139-141), in
 * (sequence, position) order.  n_out receives the number available; at most cap are copied. */
int ngsep_fetch_sites(ngsep_ctx* ctx, ngsep_site_out* out, int64_t cap, int64_t* n_out);
int ngsep_clear_sites(ngsep_ctx* ctx);
/* Alignments with insertions/deletions (CIGAR I/D) go through IndelRealignerPileupListener in the
 * reference (discovery/IndelRealignerPileupListener.java:85-526), which realigns the alignments around
 * each indel event and calls indels.  Every admitted alignment with an I/D item opens a region
 * [first - R, last + indel bases + R], R = the largest alignment span + 100 (the reach of an event's
 * realignment: every alignment overlapping it), merged per sequence.  With params.indel_passthrough = 0
 * (ABI 6, the default for single-sample runs at ploidy < 3 in streamed runs; ABI 8: MultisampleVariantsDetector at
 * ploidy < 3, outside the staged measurement entry points; ABI 9: with -knownVariants too)
 * the regions are realigned and called here: indel / STR records (is_call bit 3; population records with
 * multisnv_type 3) and the SNVs of the realigned alignments join the other calls, and no region is listed below.  Otherwise (pass-through, and
 * every other mode) no call is made inside a region; outside them the calls are the reference's; the regions
 * are returned here, in processing order, for the caller's own path (the JNI host runs the Java listener
 * chain on them): sequence ids, 1-based first and last positions.  n_out receives the number available. */
int ngsep_fetch_carved_regions(ngsep_ctx* ctx, int32_t* seq_id, int64_t* first, int64_t* last, int64_t cap, int64_t* n_out);
int ngsep_clear_carved_regions(ngsep_ctx* ctx);

/* ---- VCF text, VCFFileWriter.printHeader / printVCFRecord (vcf/VCFFileWriter.java:44-68,309-311) ---- */
int ngsep_write_vcf_header(ngsep_ctx* ctx, const char* path);
int ngsep_append_vcf_records(ngsep_ctx* ctx, const char* path);   /* all fetched sites, then clears them */
int64_t ngsep_format_site(ngsep_ctx* ctx, const ngsep_site_out* site, char* buf, int64_t cap);
/* ABI 6: the VCF line of fetched site i (any record kind, indel / STR records included); returns its length,
 * copies at most cap - 1 characters and a terminating 0 (VCFFileWriter.printVCFRecord) */
int64_t ngsep_site_vcf_line(ngsep_ctx* ctx, int64_t i, char* buf, int64_t cap);

/* ---- MultisampleVariantsDetector (discovery/MultisampleVariantsDetector.java:421-693) ----
 * Samples in VCF column order (loadSamplesFromAlignmentHeaders: TreeMap by id, :499-523).
 * rg_sample[g] = sample of read group g (the read_group index of ngsep_read_batch; -1 = none: the
 * read still counts in the pooled allele counts); rg_rank[g] = position of g in its sample's read
 * group set iteration (Sample.getReadGroups, variants/Sample.java:36-67), the order in which
 * PileupRecord.getAlleleCalls(span, readGroups) (:104-111) visits them. */
int ngsep_set_samples(ngsep_ctx* ctx, int32_t n_samples, const char* const* sample_ids,
                      int32_t n_read_groups, const int32_t* rg_sample, const int32_t* rg_rank);
/* Population sites in (sequence, position) order; calls[i * n_samples + s] is sample s at site i. */
int ngsep_fetch_population_sites(ngsep_ctx* ctx, ngsep_popsite_out* sites, ngsep_sample_call* calls,
                                 int64_t cap, int64_t* n_out);
/* MultisampleVariantsDetector output: VCF header with the samples, then every fetched site */
int ngsep_write_population_vcf(ngsep_ctx* ctx, const char* path);
/* ABI 8: the VCF line of population site i (any record kind, indel / STR records included); returns its length,
 * copies at most cap - 1 characters and a terminating 0 (VCFFileWriter.printVCFRecord of
 * VCFRecord.createDefaultPopulationVCFRecord, vcf/VCFRecord.java:277-282) */
int64_t ngsep_population_site_vcf_line(ngsep_ctx* ctx, int64_t i, char* buf, int64_t cap);
/* path B of the multisample detector: `MultisampleVariantsDetector -r REF -o OUT.vcf BAM...`
 * (MultisampleVariantsDetector.main/run, :412-459): samples from the BAM headers' @RG SM tags,
 * files merged as AlignmentsPileupGenerator.processFiles does (:201-266, chooseNextAln :268-289) */
int ngsep_call_population_bams(ngsep_ctx* ctx, const char* const* bam_paths, int32_t n_files, const char* out_vcf_path);
/* the same restricted to seq:first-last (1-based, inclusive; -querySeq -first -last), every file read from the region's
 * BAI chunks; the context (reference, -knownVariants, device) is reused by the next call -- one context per rank in the
 * sharded population caller (MultisampleVariantsDetector.run per sequence, :421-459) */
int ngsep_call_population_region_bams(ngsep_ctx* ctx, const char* const* bam_paths, int32_t n_files, const char* seq,
                                      int64_t first, int64_t last, const char* out_vcf_path);

/* ---- path B: the whole SingleSampleVariantsDetector.findSNVS on a BAM file (:896-931) ----
 * BGZF blocks inflate on the host threads (NGSEP_THREADS / OMP_NUM_THREADS) while records are decoded;
 * with params.query_seq set the reader seeks through the BAI index (path.bai) when one exists. */
int ngsep_call_bam(ngsep_ctx* ctx, const char* bam_path, const char* out_vcf_path);
/* findSNVS restricted to seq:first-last (1-based, inclusive) -- `-querySeq seq -first first -last last`
 * (SingleSampleVariantsDetector options, AlignmentsPileupGenerator.java:242-254,342-354) -- reading only
 * the region's BGZF blocks through the BAI index (htsjdk SamReader.query's role in
 * ReadAlignmentFileReader.java:171-183).  Writes the VCF header and the region's calls to out_vcf_path. */
int ngsep_call_region_bam(ngsep_ctx* ctx, const char* bam_path, const char* seq, int64_t first, int64_t last,
                          const char* out_vcf_path);
/* ABI 9: a window boundary for the sharded drivers: the first position *cut >= pos of seq that no
 * indel realigner event can reach -- outside [first - M, last + indel bases + M] of every alignment with I/D in the
 * files (and of every region-opening input variant), M = 2 x the longest alignment span around pos + 100 -- and
 * *lead = M + that span.  A region run of seq:(cut_k - lead_k)..(cut_k+1 - 1) (ngsep_call_region_bam /
 * ngsep_call_population_region_bams) calls every position in [cut_k, cut_k+1) as the whole-file run does
 * (IndelRealignerPileupListener's state and the listeners' lastIndelEnd are fresh there; AlignmentsPileupGenerator's
 * querySeq admission, :310-322, differs only before cut_k).  *cut = the sequence length + 1 when no such position
 * exists.  Reads the files' BAI indexes; deterministic in (files, seq, pos). */
int ngsep_clean_cut(ngsep_ctx* ctx, const char* const* bam_paths, int32_t n_files, const char* seq, int64_t pos,
                    int64_t* cut, int64_t* lead);

/* ABI 11: several devices from ONE process -- the drop-in's multi-GPU run of
 * SingleSampleVariantsDetector.findSNVS (:896-931) / MultisampleVariantsDetector.run (:421-459).  ctxs[0..n_ctx) are
 * open contexts, one per device (ngsep_open(device_k, params), the same params); the first holds the reference (and the
 * -knownVariants / -knownSTRs inputs); a later context without a reference takes the first one's.  Every header
 * sequence of the (first) BAM is cut into windows of about `window` bp at ngsep_clean_cut boundaries (window <= 0, or
 * indel pass-through mode: whole sequences); one host thread per context takes windows from an in-process queue and
 * runs each as a region (ngsep_call_region_bam / ngsep_call_population_region_bams from the cut minus its lead-in:
 * AlignmentsPileupGenerator.java:242-254,310-322), on its own device, streams and pinned buffers, keeping the records
 * inside the window; out_vcf_path gets the header and the windows' records in (sequence, window) order -- the
 * one-context VCF.  Temporary files out_vcf_path.part<k> are removed.  Errors are reported on ctxs[0]; in pass-through
 * mode every context's carved regions end up on ctxs[0] (ngsep_fetch_carved_regions).  Host memory: a context without
 * a reference receives a copy of the first one's (sequences and input variants), so N contexts hold N copies of the
 * reference (a 3.1 Gb genome: ~3 GB each) on top of the per-context read buffers. */
int ngsep_call_bam_multi(ngsep_ctx* const* ctxs, int32_t n_ctx, const char* bam_path, const char* out_vcf_path,
                         int64_t window);
int ngsep_call_population_bams_multi(ngsep_ctx* const* ctxs, int32_t n_ctx, const char* const* bam_paths, int32_t n_files,
                                     const char* out_vcf_path, int64_t window);
/* the windows those drivers (and ngsepcore_amd/sharding.py) run: for i < min(*n_out, cap), sequence seq_id[i] positions
 * first[i]..last[i], run from first[i] - lead[i]; every header sequence the reference holds is covered once, in order
 * (host only: reads the BAM header and the BAI neighbourhoods of the nominal cuts) */
int ngsep_plan_windows(ngsep_ctx* ctx, const char* const* bam_paths, int32_t n_files, int64_t window, int32_t* seq_id,
                       int64_t* first, int64_t* last, int64_t* lead, int64_t cap, int64_t* n_out);

/* ---- CoverageStatisticsCalculator (discovery/CoverageStatisticsCalculator.java:108-216) ----
 * path A: params.coverage_stats = 1, alignments through ngsep_process_alignments, ngsep_notify_end runs
 * the device histogram (the PileupListener.onPileup -> processPileup loop, :124-131,177-190) over every
 * sequence received; the staged entry points (ngsep_stage_*, ngsep_run_staged) run it on resident reads.
 * ngsep_fetch_coverage returns getCoverageCounts() and the unique-alignment counts for i in [1, max_coverage)
 * (entry 0 is set to 0: the reference's bin 0 counts empty pileups, which are never printed) and the two
 * "More" counts; ngsep_write_coverage prints printCoverageStats (:209-215).  Counts accumulate over runs
 * until ngsep_clear_coverage. */
int ngsep_fetch_coverage(ngsep_ctx* ctx, int64_t* counts, int64_t* counts_unique, int64_t* high, int64_t* high_unique);
int ngsep_write_coverage(ngsep_ctx* ctx, const char* path);   /* "-" = stdout */
int ngsep_clear_coverage(ngsep_ctx* ctx);
/* path B: `CoverageStats -i BAM -o OUT [-minMQ N]` (CoverageStatisticsCalculator.processFile, :99-122) */
int ngsep_coverage_bam(ngsep_ctx* ctx, const char* bam_path, const char* out_path);

/* ---- BAM reading (ReadAlignmentFileReader semantics, alignments/io/ReadAlignmentFileReader.java:219-354) ---- */
typedef struct ngsep_bam ngsep_bam;
int  ngsep_bam_open(ngsep_ctx* ctx, const char* path, ngsep_bam** out);
/* reads up to max_reads filtered alignments; the batch arrays stay valid until the next call */
int  ngsep_bam_next_batch(ngsep_bam* bam, int64_t max_reads, ngsep_read_batch* batch);
/* positions the reader at the first BGZF chunk that can hold alignments overlapping seq:first-last (BAI
 * index, SAM spec 5.2); next_batch then returns records in file order and stops after the last record
 * of seq starting at or before last.  NGSEP_E_IO when the BAM has no index. */
int  ngsep_bam_set_region(ngsep_bam* bam, const char* seq_name, int64_t first, int64_t last);
int  ngsep_bam_close(ngsep_bam* bam);
/* ABI 12: BGZF decompression on the context's device -- htsjdk BlockCompressedInputStream's role for the BAM readers
 * (ReadAlignmentFileReader.java:171-183).  Every BGZF block of in[0, n) (which ends on a block boundary) is inflated
 * (RFC 1951) into out; *out_n = the decoded bytes (the sum of the blocks' ISIZE).  NGSEP_E_INVALID with *out_n set
 * when cap is too small, NGSEP_E_FORMAT for a malformed block or one that does not inflate to its ISIZE.  The
 * single-sample BAM readers (ngsep_bam_open with no samples set) inflate this way when NGSEP_GPU_INFLATE is set. */
int  ngsep_bgzf_inflate(ngsep_ctx* ctx, const uint8_t* in, int64_t n, uint8_t* out, int64_t cap, int64_t* out_n);

/* ---- measurement entry points (bench.py): split staging (pack + H2D) from the device run ---- */
int ngsep_stage_alignments(ngsep_ctx* ctx, const ngsep_read_batch* batch);  /* pack + upload, keep resident */
int ngsep_stage_finish(ngsep_ctx* ctx);
/* one pass of K1+K2 (+ D2H of the calls) over every resident window; returns elapsed ms (host wall, synchronized) */
int ngsep_run_staged(ngsep_ctx* ctx, double* elapsed_ms);
int ngsep_release_staged(ngsep_ctx* ctx);
/* the same pass split in two: submit enqueues the kernels and the result copies and returns at once;
 * collect waits for the oldest submitted pass and makes its calls the context's result
 * (ngsep_fetch_sites).  At most two passes in flight: the copies and host work of one overlap the
 * kernels of the next (a streaming caller's pipeline over windows). */
int ngsep_submit_staged(ngsep_ctx* ctx);
int ngsep_collect_staged(ngsep_ctx* ctx, double* elapsed_ms);

#ifdef __cplusplus
}
#endif
#endif
