/*
 * ngsep_synth.h -- seeded synthetic genomes and reads for parity tests and bench.py
 * (SURVEY.md section 8(d)).  Test/bench data infrastructure, not part of the product.
 *
 * The reference's own simulators are unseeded (simulation/SingleIndividualSimulator.java:282)
 * so reproducible fixtures come from this generator instead.
 */
#ifndef NGSEP_SYNTH_H
#define NGSEP_SYNTH_H
#include <stdint.h>
#include "../../include/ngsep_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { NGS_GENOME_YEAST = 0, NGS_GENOME_HUMAN = 1, NGS_GENOME_CUSTOM = 2 };

typedef struct ngs_synth_params {
    int32_t genome;          /* NGS_GENOME_* */
    int32_t contig_first;    /* first contig index to keep (yeast/human tables) */
    int32_t n_contigs;       /* number of contigs to keep (<=0: all from contig_first) */
    int64_t custom_len;      /* NGS_GENOME_CUSTOM: one contig "chrS" of this length */
    double  depth;           /* 30 */
    int32_t read_len;        /* 150 */
    uint64_t seed;           /* per-config seed (C1 1, C2 2, C3 3, ...) */
    double  snv_rate;        /* 1e-3 */
    double  dup_rate;        /* 0.002 PCR duplicate copies */
    double  lower_frac;      /* fraction of lower-case reference positions (0 or 0.01) */
    double  n_frac;          /* fraction of read bases replaced by N at Q2 (0.001) */
    int32_t sample_idx;      /* RG/SM = S%03d */
    int32_t quality_model;   /* 0: {2:2%,12:3%,25:10%,33:35%,37:50%}; 1: all Q30 ('?') ; 2: uniform 0..40 */
    double  secondary_rate;  /* fraction of extra secondary (0x100) records */
    double  lowmq_rate;      /* fraction of reads with MAPQ 5 */
    double  noqual_rate;     /* fraction of reads whose QUAL is '*' */
    double  softclip_rate;   /* fraction of reads with a 5-20 bp soft clip at one end */
    int32_t n_samples;       /* >1: a population of diploid samples S%03d (sample_idx..), depth per sample,
                                population SNVs at snv_rate with AF U(0.02,0.98) in HWE (multisample config C5) */
    int64_t trunc_len;       /* >0: every contig truncated to this length (bounded CPU-baseline samples) */
    int32_t rng_per_contig;  /* 1: each contig's donor/reads from its own seeded stream, so a contig generated
                                alone (one rank's shard, contig_first=k, n_contigs=1) equals it in the whole genome */
    double  indel_rate;      /* donor indels (1-10 bp insertions/deletions) per bp; reads across them carry I/D */
    int64_t hot_first;       /* hot_depth > 0: extra reads starting in [hot_first, hot_first + hot_len - read_len] */
    int64_t hot_len;         /*   (1-based; a collapsed repeat: every sample hot_depth deeper there) */
    double  hot_depth;
} ngs_synth_params;

typedef struct ngs_synth ngs_synth;

void ngs_synth_default(ngs_synth_params* p);
ngs_synth* ngs_synth_create(const ngs_synth_params* p);
void ngs_synth_free(ngs_synth* s);
int ngs_synth_n_contigs(const ngs_synth* s);
const char* ngs_synth_contig_name(const ngs_synth* s, int i);
int64_t ngs_synth_contig_len(const ngs_synth* s, int i);
const char* ngs_synth_contig_seq(const ngs_synth* s, int i);
int64_t ngs_synth_n_reads(const ngs_synth* s);
int64_t ngs_synth_n_bases(const ngs_synth* s);
/* reads after the reader's filters (unmapped/secondary/multiple, consecutive duplicates), as
 * AlignmentsPileupGenerator.processAlignment would receive them with default options */
int ngs_synth_batch(ngs_synth* s, ngsep_read_batch* out);
int ngs_synth_write_fasta(const ngs_synth* s, const char* path);
int ngs_synth_write_sam(const ngs_synth* s, const char* path);
int ngs_synth_write_bam(const ngs_synth* s, const char* path);   /* also writes path + ".bai" */
int ngs_synth_write_bam_sample(const ngs_synth* s, const char* path, int sample);
int ngs_synth_write_truth(const ngs_synth* s, const char* path);
/* SAM text -> BAM (header verbatim, records in file order, aux tags A/i/f/Z) */
int ngs_sam_to_bam(const char* sam_path, const char* bam_path);

#ifdef __cplusplus
}
#endif
#endif
