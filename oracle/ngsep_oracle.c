/*
 * ngsep_oracle.c -- CPU restatement of NGSEP 4.3.2's SNV pileup-calling path.
 *
 * TEST INFRASTRUCTURE ONLY (see ngsep_oracle.h).  Written as a line-by-line
 * restatement of the Java reference so that the HIP product can be checked
 * against it; it is deliberately simple and single-threaded, like the
 * reference's pileup thread.  Every function cites the Java it follows
 * (paths relative to src/ngsep/ of acastem15/NGSEPcore).
 *
 * Scope restated: SAM text + FASTA -> VCF for SingleSampleVariantsDetector with
 * ploidy 1/2, SNV-only alignments (no I/D CIGAR operations: the indel realigner
 * is then a pass-through, discovery/IndelRealignerPileupListener.java:85-126).
 * Inputs outside that scope make ngo_run_ssvd() return NGO_UNSUPPORTED.
 */
#define _GNU_SOURCE
#include "ngsep_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <ctype.h>

#define NGO_OK 0
#define NGO_ERR_IO 1
#define NGO_ERR_FORMAT 2
#define NGO_UNSUPPORTED 3

/* ------------------------------------------------------------------ */
/* Java numerics                                                        */
/* ------------------------------------------------------------------ */

/* java.lang.Math.round(double): closest long, ties toward +infinity, NaN -> 0 */
int64_t ngo_java_round(double x) {
    if (isnan(x)) return 0;
    double f = floor(x);
    double r = (x - f >= 0.5) ? f + 1.0 : f;
    if (r >= 9.2233720368547758e18) return INT64_MAX;
    if (r <= -9.2233720368547758e18) return INT64_MIN;
    return (int64_t)r;
}

/* math/PhredScoreHelper.java:31-40 */
int ngo_phred(double p) {
    if (p == 0) return 255;
    double score = -10 * log10(p);
    if (score > 255) return 255;           /* NaN > 255 is false, as in Java */
    return (int16_t)ngo_java_round(score);  /* (short)Math.round(score) */
}

/* math/PhredScoreHelper.java:46-51 */
static double phred_prob(int q) {
    if (q >= 255) return 0;
    return pow(10.0, -0.1 * q);
}

/* ------------------------------------------------------------------ */
/* CountsHelper probability caches, CountsHelper.java:135-187           */
/* ------------------------------------------------------------------ */
#define NGO_M 31          /* DEF_MAX_BASE_QS+1 */
#define NGO_NCOL 18       /* covers allele lists up to 16 (+1) */
#define NGO_NFREQ 501     /* DEF_NUM_FREQUENCIES */
static double g_err[NGO_M][NGO_NCOL];
static double (*g_gt)[NGO_M][NGO_NCOL];
static int g_tables_ready = 0;

static void ensure_tables(void) {
    if (g_tables_ready) return;
    memset(g_err, 0, sizeof(g_err));
    /* CountsHelper.java:147-154 (entries q < DEF_MIN_BASE_QS stay 0) */
    for (int i = 3; i < NGO_M; i++) {
        g_err[i][0] = -0.1 * i;
        for (int j = 2; j < NGO_NCOL; j++) g_err[i][j] = g_err[i][0] - log10((double)(j - 1));
    }
    g_gt = calloc(NGO_NFREQ, sizeof(*g_gt));
    /* CountsHelper.java:168-187 */
    for (int f = 0; f < NGO_NFREQ; f++) {
        double af = (double)f / (NGO_NFREQ - 1);
        for (int i = 3; i < NGO_M; i++) {
            double errorProb = phred_prob(i);
            double successProb = 1 - errorProb;
            g_gt[f][i][0] = log10(successProb);
            for (int j = 2; j < NGO_NCOL; j++) {
                double hetProb = af * successProb + (1 - af) * errorProb / (j - 1);
                g_gt[f][i][j] = log10(hetProb);
            }
        }
    }
    g_tables_ready = 1;
}

double ngo_table_error(int q, int j) { ensure_tables(); return g_err[q][j]; }
double ngo_table_gt(int f, int q, int j) { ensure_tables(); return g_gt[f][q][j]; }

/* CountsHelper.java:86-89,110-112,125-134,191-202 */
void ngo_counts_init(ngo_counts* c, int n_alleles, double het_proportion, int max_base_qs) {
    ensure_tables();
    memset(c, 0, sizeof(*c));
    c->n_alleles = n_alleles;
    c->max_base_qs = 30;                                  /* DEF_MAX_BASE_QS */
    if ((int8_t)max_base_qs > 0) c->max_base_qs = (int8_t)max_base_qs;   /* byte field */
    c->f = (int)ngo_java_round(het_proportion * (NGO_NFREQ - 1));        /* :212 */
    c->g = (int)ngo_java_round((1 - het_proportion) * (NGO_NFREQ - 1));  /* :213 */
}

/* CountsHelper.updateCounts, CountsHelper.java:209-251 */
void ngo_counts_update(ngo_counts* c, int index, int qualScore, int negativeStrand) {
    c->total_count++;
    int8_t q = (int8_t)qualScore;
    if (q <= 3) { c->low_bq_count++; return; }           /* DEF_MIN_BASE_QS */
    else if (q > c->max_base_qs) q = (int8_t)c->max_base_qs;
    if (index < 0) return;
    int n = c->n_alleles;
    c->counts[index]++;
    c->allele_error_log_probs[index] += g_err[q][0];
    if (negativeStrand) c->counts_strand[index][0]++;
    else c->counts_strand[index][1]++;
    for (int i = 0; i < n; i++) {
        if (i == index) c->logc[i][i] += g_gt[c->f][q][0];
        else c->logc[i][i] += g_err[q][n];
        for (int j = 0; j < n; j++) {
            if (i != j) {
                if (j == index) c->logc[i][j] += g_gt[c->f][q][n];
                else if (i == index) c->logc[i][j] += g_gt[c->g][q][n];
                else c->logc[i][j] += g_err[q][n];
            }
        }
    }
}

/* CountsHelper.calculatePosteriorProbabilities, CountsHelper.java:472-495 */
static void calc_posteriors(double* ev, int m) {
    double logMax = 1;
    for (int i = 0; i < m; i++)
        if (logMax > 0 || logMax < ev[i]) logMax = ev[i];
    double totalProb = 0;
    for (int i = 0; i < m; i++) {
        ev[i] -= logMax;
        if (ev[i] < -20) ev[i] = 0.0;
        else ev[i] = pow(10.0, ev[i]);
        totalProb += ev[i];
    }
    for (int i = 0; i < m; i++) ev[i] = ev[i] / totalProb;
}

/* CountsHelper.getPosteriorProbabilities(double), CountsHelper.java:410-443 */
void ngo_counts_posteriors(const ngo_counts* c, double hetRate, double* post) {
    int n = c->n_alleles;
    int heteroGenotypes = n * (n - 1);
    double logPriorHetero = log10(hetRate / heteroGenotypes);
    double logPriorHomo = log10((1 - hetRate) / n);
    double ev[NGO_MAX_ALLELES * NGO_MAX_ALLELES];
    int k = 0;
    for (int i = 0; i < n; i++) {
        ev[k++] = c->logc[i][i] + logPriorHomo;
        for (int j = 0; j < n; j++)
            if (i != j) ev[k++] = c->logc[i][j] + logPriorHetero;
    }
    calc_posteriors(ev, n * n);
    k = 0;
    for (int i = 0; i < n; i++) {
        post[i * n + i] = ev[k++];
        for (int j = 0; j < n; j++)
            if (i != j) post[i * n + j] = ev[k++];
    }
}

/* math/FisherExactTest.java:65-134 (quick mode is the static default, :31) */
static double* g_logfact = NULL;
static int g_logfact_n = 0;
static double fisher_exact(int a, int b, int c, int d) {
    int n = a + b + c + d;
    if (!g_logfact || g_logfact_n <= n) {
        int m = n < 10000 ? 10000 : n;
        free(g_logfact);
        g_logfact = malloc(sizeof(double) * (m + 1));
        g_logfact[0] = g_logfact[1] = 0;
        for (int i = 2; i <= m; i++) g_logfact[i] = g_logfact[i - 1] + log10((double)i);
        g_logfact_n = m + 1;
    }
    double ans = g_logfact[a + b];
    ans += g_logfact[c + d];
    ans += g_logfact[a + c];
    ans += g_logfact[b + d];
    ans -= g_logfact[a];
    ans -= g_logfact[b];
    ans -= g_logfact[c];
    ans -= g_logfact[d];
    ans -= g_logfact[n];
    return pow(10.0, ans);
}
double ngo_fisher_pvalue(int a, int b, int c, int d) {
    if (a > b) { int t = a; a = b; b = t; t = c; c = d; d = t; }
    if (a > c) { int t = a; a = c; c = t; t = b; b = d; d = t; }
    int e = a < d ? a : d;
    double answer = 0;
    while (a >= 0 && d >= 0) {
        double p = fisher_exact(a, b, c, d);
        if (e >= 10 && answer > (double)(100 * e) * p) break;
        answer += p;
        a--; b++; c++; d--; e++;
    }
    return answer;
}

/* CountsHelper.getScoreStrandBiasFisher, CountsHelper.java:563-576 */
static int strand_bias_score(const ngo_counts* c, int i1, int i2) {
    double pv = ngo_fisher_pvalue(c->counts_strand[i1][0], c->counts_strand[i2][0],
                                  c->counts_strand[i1][1], c->counts_strand[i2][1]);
    int s = ngo_phred(pv);
    if (s > 100) s = 100;          /* MAX_STRAND_BIAS_SCORE */
    return (int8_t)s;
}

void ngo_params_default(ngo_params* p) {
    memset(p, 0, sizeof(*p));
    p->min_mq = 20;
    p->max_alns_per_start = 5;
    p->max_base_qs = 30;
    p->min_quality = 40;
    p->ploidy = 2;
    p->het_rate = 0.001;
    p->sample_id = "Sample";
    p->query_first = 0;
    p->query_last = 1000000000;
}

/* ------------------------------------------------------------------ */
/* Reference genome (genome/ReferenceGenome.java, FastaFileReader with   */
/* keepLowerCase=true, DNAMaskedSequence alphabet "AaCcNngGtT")          */
/* ------------------------------------------------------------------ */
typedef struct { char* name; char* seq; int64_t len; } ngo_seq;
typedef struct { ngo_seq* s; int n, cap; } ngo_genome;

static char mask_base(char c) {
    switch (c) {
        case 'A': case 'a': case 'C': case 'c': case 'N': case 'n':
        case 'G': case 'g': case 'T': case 't': return c;
        default: return 'N';
    }
}

static int load_fasta(const char* path, ngo_genome* g) {
    FILE* f = fopen(path, "r");
    if (!f) return NGO_ERR_IO;
    memset(g, 0, sizeof(*g));
    char* line = NULL; size_t lcap = 0; ssize_t l;
    ngo_seq* cur = NULL; int64_t scap = 0;
    while ((l = getline(&line, &lcap, f)) >= 0) {
        while (l > 0 && (line[l - 1] == '\n' || line[l - 1] == '\r')) line[--l] = 0;
        if (l > 0 && line[0] == '>') {
            if (g->n == g->cap) { g->cap = g->cap ? 2 * g->cap : 16; g->s = realloc(g->s, sizeof(ngo_seq) * g->cap); }
            cur = &g->s[g->n++];
            size_t e = 1; while (line[e] && line[e] != ' ' && line[e] != '\t') e++;
            cur->name = strndup(line + 1, e - 1);
            scap = 1 << 20; cur->seq = malloc(scap); cur->len = 0;
        } else if (cur) {
            if (cur->len + l + 1 > scap) { while (cur->len + l + 1 > scap) scap *= 2; cur->seq = realloc(cur->seq, scap); }
            for (ssize_t i = 0; i < l; i++) cur->seq[cur->len++] = mask_base(line[i]);
            cur->seq[cur->len] = 0;
        }
    }
    free(line); fclose(f);
    return NGO_OK;
}
static int genome_find(const ngo_genome* g, const char* name) {
    for (int i = 0; i < g->n; i++) if (strcmp(g->s[i].name, name) == 0) return i;
    return -1;
}

/* ------------------------------------------------------------------ */
/* ReadAlignment (alignments/ReadAlignment.java)                        */
/* ------------------------------------------------------------------ */
enum { OP_H = 0, OP_D = 1, OP_I = 2, OP_M = 3, OP_P = 4, OP_N = 5, OP_S = 6, OP_X = 7 };  /* :60-67 */
#define FLAG_UNMAPPED 0x4
#define FLAG_REVERSE 0x10
#define FLAG_SECONDARY 0x100
#define FLAG_MULTIPLE 0x1000

typedef struct ngo_aln {
    int seq;                 /* genome index */
    int first, last, read_length, flags, rg;
    int n_ops; int* ops;     /* len*8+op, ReadAlignment.java:1180-1198 */
    char* chars;             /* NULL if '*' */
    uint8_t* quals;          /* NULL if '*' */
    int ignore_start, ignore_end;
    int16_t* acl;            /* alleleCallLength, :747-834 */
    int has_indel;
} ngo_aln;

static void aln_free(ngo_aln* a) { free(a->ops); free(a->chars); free(a->quals); free(a->acl); free(a); }

/* ReadAlignment.updateAlleleCallsInfo, ReadAlignment.java:747-834 (indel-call map omitted:
 * SNV-only inputs never populate it) */
static void update_allele_calls(ngo_aln* a) {
    free(a->acl);
    a->acl = calloc(a->read_length > 0 ? a->read_length : 1, sizeof(int16_t));
    int refPos = a->first, readPos = 0, prevIndel = 0;
    const int closeIndel = 2;  /* basesToIgnoreCloseToIndel, :115 */
    for (int i = 0; i < a->n_ops; i++) {
        int len = a->ops[i] / 8, op = a->ops[i] & 7;
        int cRef = op & 1, cRead = (op & 2) != 0;
        int nextOp = -1, nextLen = 0, nextIsIndel = 0, nextReadCons = 0;
        if (i < a->n_ops - 1) {
            nextOp = a->ops[i + 1] & 7; nextLen = a->ops[i + 1] / 8;
            nextIsIndel = (nextOp == OP_D || nextOp == OP_I);
            nextReadCons = (nextOp & 2) ? nextLen : 0;
        }
        if (cRef) {
            if (cRead) {
                for (int j = 0; j < len; j++) {
                    int skip = readPos < a->ignore_start;
                    skip = skip || (a->read_length - readPos) <= a->ignore_end;
                    skip = skip || (prevIndel && j < closeIndel);
                    skip = skip || (nextIsIndel && j < len - 1 && j >= len - closeIndel);
                    skip = skip || (nextIsIndel && j == len - 1 &&
                                    (readPos < closeIndel || a->read_length - readPos - nextReadCons < closeIndel));
                    int readPosAfterIndel = readPos + nextReadCons + 1;
                    skip = skip || (nextIsIndel && j == len - 1 && (a->read_length - readPosAfterIndel < a->ignore_end));
                    if (!skip && readPos < a->read_length) {
                        if (j == len - 1 && nextIsIndel) a->acl[readPos] = (nextOp == OP_I) ? (int16_t)(nextLen + 2) : 2;
                        else a->acl[readPos] = 1;
                    }
                    refPos++; readPos++;
                }
            } else refPos += len;
        } else if (cRead) readPos += len;
        prevIndel = (op == OP_D || op == OP_I);
    }
}

/* ReadAlignment.getAlignedReadPosition, ReadAlignment.java:842-871 */
static int aligned_read_pos(const ngo_aln* a, int refPos) {
    int curRef = a->first, curRead = 0;
    if (refPos < a->first || refPos > a->last) return -1;
    for (int i = 0; i < a->n_ops; i++) {
        int len = a->ops[i] / 8, op = a->ops[i] & 7;
        int cRef = op & 1, cRead = (op & 2) != 0;
        if (cRef && cRead) {
            if (refPos < curRef) return -1;
            else if (curRef + len > refPos) {
                int ans = curRead + refPos - curRef;
                if (ans < 0 || ans >= a->read_length) return -1;
                return ans;
            }
        }
        if (cRef) curRef += len;
        if (cRead) curRead += len;
    }
    return -1;
}

/* ReadAlignment.setBasesToIgnore5P/3P, ReadAlignment.java:613-644 */
static void set_ignore(ngo_aln* a, int i5, int i3) {
    if (a->flags & FLAG_REVERSE) { a->ignore_end = i5; a->ignore_start = i3; }
    else { a->ignore_start = i5; a->ignore_end = i3; }
}

/* ------------------------------------------------------------------ */
/* SAM record parsing (the role htsjdk plays in                         */
/* alignments/io/ReadAlignmentFileReader.java:219-354)                  */
/* ------------------------------------------------------------------ */
typedef struct { char** ids; int n, cap; } ngo_strlist;
static int strlist_get(ngo_strlist* l, const char* s, int add) {
    for (int i = 0; i < l->n; i++) if (strcmp(l->ids[i], s) == 0) return i;
    if (!add) return -1;
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 8; l->ids = realloc(l->ids, sizeof(char*) * l->cap); }
    l->ids[l->n] = strdup(s);
    return l->n++;
}

typedef struct {
    char* qname; int flag; int start; int paired, first_of_pair;
} ngo_rawkey;

/* parse CIGAR into NGSEP codes with collapseEqualEvents; returns -1 if malformed */
static int parse_cigar(const char* s, int** ops_out, int* n_out) {
    static const char* codes = "HDIMPNSX";     /* ALIGNMENT_CHAR_CODES, :69 */
    int cap = 8, n = 0; int* ops = malloc(sizeof(int) * cap);
    long len = 0; int have = 0;
    for (const char* p = s; *p; p++) {
        if (isdigit((unsigned char)*p)) { len = len * 10 + (*p - '0'); have = 1; continue; }
        if (!have) { free(ops); return -1; }
        const char* q = strchr(codes, *p);
        int op;
        if (q) op = (int)(q - codes);
        else if (*p == '=') op = OP_M;
        else { free(ops); return -1; }
        if (n > 0 && (ops[n - 1] & 7) == op) ops[n - 1] += (int)len * 8;   /* collapseEqualEvents */
        else { if (n == cap) { cap *= 2; ops = realloc(ops, sizeof(int) * cap); } ops[n++] = (int)len * 8 + op; }
        len = 0; have = 0;
    }
    *ops_out = ops; *n_out = n;
    return 0;
}

/* ------------------------------------------------------------------ */
/* Listener output: called SNVs (variants/CalledSNV.java,              */
/* variants/CalledGenomicVariantImpl.java) and the VCF writer          */
/* (vcf/VCFFileWriter.java:44-308)                                      */
/* ------------------------------------------------------------------ */
typedef struct ngo_call {
    int pos;
    char ref;
    int n_alleles;            /* 2 = CalledSNV, 3 = triallelic CalledGenomicVariantImpl */
    int idx[3];               /* DNA indexes of ref, alt, third */
    int genotype;             /* CalledSNV: 1 het, 2 homalt */
    int gq, qual, dp;
    int counts[4];
    double logc[4][4];
    int strand_bias;          /* -1 invalid */
    int ploidy;
} ngo_call;

typedef struct { ngo_call* c; int n, cap; } ngo_calls;

static const char* BASES = "ACGT";
static int base_idx(char c) { const char* p = strchr(BASES, c); return (c && p) ? (int)(p - BASES) : -1; }

static void print_header(FILE* out, const ngo_params* p) {
    /* vcf/VCFFileHeader.java:46-71 (attribute order ID,Number,Type,Description per VCFHeaderLine.java:43-50), :219-245 */
    static const char* lines[][5] = {
        {"INFO", "CNV", "\"Number of samples with CNVs around this variant\"", "1", "Integer"},
        {"INFO", "TA", "\"Variant annotation based on a gene model\"", "1", "String"},
        {"INFO", "TID", "\"Id of the transcript related to the variant annotation\"", "1", "String"},
        {"INFO", "TGN", "\"Name of the gene related to the variant annotation\"", "1", "String"},
        {"INFO", "TCO", "\"One based codon position of the start of the variant. The decimal is the codon position\"", "1", "Float"},
        {"INFO", "TACH", "\"Description of the aminoacid change produced by a non-synonymous mutation. String encoded as reference aminoacid, position and mutated aminoacid\"", "1", "String"},
        {"INFO", "NS", "\"Number of samples genotyped\"", "1", "Integer"},
        {"INFO", "MAF", "\"Minor allele frequency\"", "1", "Float"},
        {"INFO", "OH", "\"Observed heterozygosity\"", "1", "Float"},
        {"INFO", "AN", "\"Number of alleles in called genotypes\"", "1", "Integer"},
        {"INFO", "AFS", "\"Allele counts over the population for all alleles, including the reference\"", "R", "Integer"},
        {"INFO", "TYPE", "\"Type of variant\"", "1", "String"},
        {"INFO", "FS", "\"Phred-scaled p-value using Fisher's exact test to detect strand bias\"", "1", "Float"},
        {"INFO", "END", "\"End position of the structural variant\"", "1", "Integer"},
        {"INFO", "SVTYPE", "\"Type of SV:DEL=Deletion, INS=Insertion, DUP=Duplication, INV=Inversion\"", "1", "String"},
        {"INFO", "SVLEN", "\"Difference in length between REF and ALT alleles\"", "1", "Integer"},
        {"FORMAT", "GT", "\"Genotype\"", "1", "String"},
        {"FORMAT", "PL", "\"Phred-scaled genotype likelihoods rounded to the closest integer\"", "G", "Integer"},
        {"FORMAT", "GQ", "\"Genotype quality\"", "1", "Integer"},
        {"FORMAT", "DP", "\"Read depth\"", "1", "Integer"},
        {"FORMAT", "ADP", "\"Counts for observed alleles, including the reference allele\"", "R", "Integer"},
        {"FORMAT", "BSDP", "\"Number of base calls (depth) for the 4 nucleotides in called SNVs sorted as A,C,G,T\"", "4", "Integer"},
        {"FORMAT", "ACN", "\"Predicted copy number of each allele taking into account the prediction of number of copies of the region surrounding the variant\"", "R", "Integer"},
    };
    fprintf(out, "##fileformat=VCFv4.2\n");
    for (size_t i = 0; i < sizeof(lines) / sizeof(lines[0]); i++)
        fprintf(out, "##%s=<ID=%s,Number=%s,Type=%s,Description=%s>\n", lines[i][0], lines[i][1], lines[i][3], lines[i][4], lines[i][2]);
    if (p->print_sample_ploidy) fprintf(out, "##SAMPLE=<ID=%s,PL=%d>\n", p->sample_id, p->ploidy);
    fprintf(out, "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t%s\n", p->sample_id);
}

/* one VCF line per call: VCFFileWriter.printVCFRecord + printGenotypeInfo */
static void print_call(FILE* out, const char* seqName, const ngo_call* c) {
    fprintf(out, "%s\t%d\t.\t%c\t", seqName, c->pos, c->ref);
    if (c->n_alleles == 2) fprintf(out, "%c", BASES[c->idx[1]]);
    else fprintf(out, "%c,%c", BASES[c->idx[1]], BASES[c->idx[2]]);
    fprintf(out, "\t%d\t.\t", c->qual);
    /* INFO: FS (SingleSampleVariantsDetector.java:957, CalledSNV only) then TYPE (VCFFileWriter.java:47-49) */
    int printed = 0;
    if (c->n_alleles == 2 && c->strand_bias != -1) { fprintf(out, "FS=%d", c->strand_bias); printed = 1; }
    if (c->n_alleles == 3) { fprintf(out, "%sTYPE=MULTISNV", printed ? ";" : ""); printed = 1; }
    if (!printed) fprintf(out, ".");
    fprintf(out, "\tGT:PL:GQ:DP:BSDP:ACN\t");
    int ploidy = c->ploidy;
    if (c->n_alleles == 2) {
        /* CalledSNV: GT */
        if (c->genotype == 2) { fprintf(out, "1"); if (ploidy > 1) fprintf(out, "/1"); }
        else fprintf(out, "0/1");
        fprintf(out, ":");
        /* PL from float log-conds (CalledSNV.java:259-265, :413-435; VCFFileWriter.java:200-212) */
        float hr = (float)c->logc[c->idx[0]][c->idx[0]];
        float ha = (float)c->logc[c->idx[1]][c->idx[1]];
        float ra = (float)c->logc[c->idx[0]][c->idx[1]];
        float ar = (float)c->logc[c->idx[1]][c->idx[0]];
        double lc[2][2] = {{hr, ra}, {ar, ha}};
        int present = (hr + ra + ar + ha) != 0;
        for (int j = 0; j < 2; j++)
            for (int i = 0; i <= j; i++) {
                if (i > 0 || j > 0) fprintf(out, ",");
                int v = present ? (int)ngo_java_round(-10 * lc[i][j]) : 0;
                fprintf(out, "%d", v);
            }
        fprintf(out, ":%d:%d:%d,%d,%d,%d:", c->gq, c->dp, c->counts[0], c->counts[1], c->counts[2], c->counts[3]);
        /* ACN: CalledSNV.updateAllelesCopyNumberFromCounts(ploidy), CalledSNV.java:134-168 */
        int total = ploidy, refcn = 0;
        if (c->genotype == 2) refcn = 0;
        else if (total <= 2) { total = 2; refcn = 1; }
        else {
            double cr = c->counts[c->idx[0]], sum = cr + c->counts[c->idx[1]];
            double prop = sum > 0 ? cr / sum : 0.5;
            refcn = (int16_t)ngo_java_round(prop * total);
            if (refcn == 0) refcn = 1; else if (refcn >= total) refcn = total - 1;
        }
        if (total == 0) fprintf(out, ".");
        else fprintf(out, "%d,%d", refcn, total - refcn);
    } else {
        /* triallelic CalledGenomicVariantImpl with called alleles {1,2} */
        fprintf(out, "1/2:");
        for (int j = 0; j < 3; j++)
            for (int i = 0; i <= j; i++) {
                if (i > 0 || j > 0) fprintf(out, ",");
                fprintf(out, "%d", (int)ngo_java_round(-10 * c->logc[c->idx[i]][c->idx[j]]));
            }
        fprintf(out, ":%d:%d:%d,%d,%d,%d:", c->gq, c->dp, c->counts[0], c->counts[1], c->counts[2], c->counts[3]);
        /* CalledGenomicVariantImpl.java:228-240: totalCopyNumber <= nCalled(2) -> 1 per called allele */
        if (ploidy <= 2) fprintf(out, "0,1,1");
        else {
            int cnt[2], tot = 0;
            for (int i = 0; i < 2; i++) { cnt[i] = c->counts[c->idx[i + 1]]; if (!cnt[i]) cnt[i] = 1; tot += cnt[i]; }
            int cn[3] = {0, 0, 0}, tc = 0;
            for (int i = 0; i < 2; i++) {
                int64_t r = ngo_java_round((double)ploidy * cnt[i] / tot);
                cn[i + 1] = (int)(r < 1 ? 1 : r); tc += cn[i + 1];
            }
            if (tc < ploidy) cn[1] += ploidy - tc;
            else { int ex = tc - ploidy; for (int i = 2; ex > 0 && i >= 1; i--) { int rm = ex < cn[i] - 1 ? ex : cn[i] - 1; cn[i] -= rm; ex -= rm; } }
            fprintf(out, "%d,%d,%d", cn[0], cn[1], cn[2]);
        }
    }
    fprintf(out, "\n");
}

/* ------------------------------------------------------------------ */
/* VariantDiscoverySNVQAlgorithm.discoverSNV (:100-222) and the        */
/* SingleSampleVariantPileupListener filters (:213-232)                */
/* ------------------------------------------------------------------ */
static void indexes_max_genotype(const double* post, int idxDefault, int* oi, int* oj) {
    /* VariantDiscoverySNVQAlgorithm.java:223-243 */
    if (idxDefault < 0 || idxDefault >= 4) idxDefault = 0;
    int bi = idxDefault, bj = idxDefault;
    double probMax = post[idxDefault * 4 + idxDefault];
    for (int i = 0; i < 4; i++)
        for (int j = i; j < 4; j++) {
            double gp = post[i * 4 + j];
            if (i != j) gp += post[j * 4 + i];
            if (gp > probMax + 0.01) { probMax = gp; bi = i; bj = j; }
        }
    *oi = bi; *oj = bj;
}

/* returns 1 if a call is kept */
static int discover_snv(const ngo_counts* h, int pos, char refBase, const ngo_params* p, double hetRate, ngo_call* out) {
    if (h->total_count == 0) return 0;
    int indexRef = base_idx(refBase);
    if (indexRef < 0) return 0;
    double post[16];
    ngo_counts_posteriors(h, hetRate, post);
    int I, J;
    indexes_max_genotype(post, indexRef, &I, &J);
    double refProb = post[indexRef * 4 + indexRef];
    double maxP = post[I * 4 + J];
    if (I != J) maxP += post[J * 4 + I];
    int gq = ngo_phred(1 - maxP);
    memset(out, 0, sizeof(*out));
    out->pos = pos; out->ref = refBase; out->gq = gq; out->dp = h->total_count;
    out->qual = ngo_phred(refProb);
    out->strand_bias = -1;
    out->ploidy = p->ploidy;
    memcpy(out->counts, h->counts, sizeof(out->counts));
    for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) out->logc[i][j] = h->logc[i][j];
    if (I != J && I != indexRef && J != indexRef) {
        /* triallelic, :128-177 */
        int alt, third;
        if (post[I * 4 + I] > post[J * 4 + J] + 0.01) { alt = I; third = J; }
        else { alt = J; third = I; }
        out->n_alleles = 3; out->idx[0] = indexRef; out->idx[1] = alt; out->idx[2] = third;
        /* strand bias of a triallelic call is never printed (SingleSampleVariantsDetector.java:956-958) */
    } else if (I != J) {
        out->n_alleles = 2; out->idx[0] = indexRef; out->idx[1] = (indexRef != I) ? I : J;
        out->genotype = 1;
    } else if (indexRef != I) {
        out->n_alleles = 2; out->idx[0] = indexRef; out->idx[1] = I; out->genotype = 2;
    } else {
        return 0;   /* homozygous reference: dropped by SingleSampleVariantPileupListener.java:223 */
    }
    if (out->n_alleles == 2 && p->calc_strand_bias)
        out->strand_bias = strand_bias_score(h, out->idx[0], out->idx[1]);
    /* undecided / homRef / minQuality > GQ -> dropped (SingleSampleVariantPileupListener.java:223) */
    if ((int16_t)p->min_quality > gq) return 0;
    return 1;
}

/* ------------------------------------------------------------------ */
/* AlignmentsPileupGenerator sweep (discovery/AlignmentsPileupGenerator.java:377-504) */
/* ------------------------------------------------------------------ */
typedef struct { ngo_aln** a; int n, cap; } ngo_alist;
static void alist_push(ngo_alist* l, ngo_aln* a) {
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 64; l->a = realloc(l->a, sizeof(ngo_aln*) * l->cap); }
    l->a[l->n++] = a;
}

typedef struct {
    const ngo_params* p;
    double het_rate;
    ngo_genome* g;
    FILE* out;
    FILE* dump;
    int cur_seq;               /* -1: none */
    int cur_pos, cur_last, last_start;
    ngo_alist pending, ss_primary, ss_secondary, retired;
    ngo_calls calls;
    ngo_stats* st;
    int unsupported;
} ngo_gen;

static void on_sequence_end(ngo_gen* G) {
    /* SingleSampleVariantsDetector.saveSequenceVariants, :933-968: calls are already in position order */
    for (int i = 0; i < G->calls.n; i++) print_call(G->out, G->g->s[G->cur_seq].name, &G->calls.c[i]);
    G->st->variants_called += G->calls.n;
    G->calls.n = 0;
}

/* processCurrentPosition + listeners for one position, AlignmentsPileupGenerator.java:475-498 */
static int process_current_position(ngo_gen* G) {
    if (G->pending.n == 0) { G->cur_pos++; return 0; }
    const ngo_params* p = G->p;
    if (p->query_seq && (G->cur_pos < p->query_first || G->cur_pos > p->query_last)) { G->cur_pos++; return 0; }
    int pos = G->cur_pos;
    int numAlignments = 0;
    ngo_counts h;
    ngo_counts_init(&h, 4, 0.5, p->max_base_qs);     /* CountsHelper.calculateCountsSNV(calls, maxBaseQS, 0.5) */
    for (int k = 0; k < G->pending.n; k++) {
        ngo_aln* a = G->pending.a[k];
        if (a->first > pos || a->last < pos) continue;   /* PileupRecord.addAlignment, :154-167 */
        numAlignments++;
        /* PileupRecord.getAlleleCalls(1,null), :126-152 */
        if (!a->chars) continue;
        int rp = aligned_read_pos(a, pos);
        if (rp < 0) continue;
        int len = a->acl[rp];
        if (len == 0) continue;
        if (len > 1) continue;
        int qc = a->quals ? a->quals[rp] : '+';
        int q = qc - 33; if (q > 30) q = 30;              /* CountsHelper.java:91 */
        ngo_counts_update(&h, base_idx(a->chars[rp]), (int8_t)q, (a->flags & FLAG_REVERSE) != 0);
    }
    if (numAlignments > 0) G->st->positions_genotyped++;
    /* SingleSampleVariantPileupListener.onPileup -> calculateReferenceAlleleDiscovery (:191-206) */
    const ngo_seq* s = &G->g->s[G->cur_seq];
    if (numAlignments > 0 && pos >= 1 && pos <= s->len) {
        char r = s->seq[pos - 1];
        if (G->dump && h.total_count > 0) {
            fprintf(G->dump, "%s\t%d\t%c\t%d\t%d,%d,%d,%d", s->name, pos, r, h.total_count, h.counts[0], h.counts[1], h.counts[2], h.counts[3]);
            for (int i = 0; i < 4; i++) for (int j = i; j < 4; j++) fprintf(G->dump, "\t%.17g", h.logc[i][j]);
            fprintf(G->dump, "\n");
        }
        if (!(p->ignore_lowercase_ref && islower((unsigned char)r))) {
            char R = (char)toupper((unsigned char)r);
            ngo_call c;
            if (discover_snv(&h, pos, R, p, G->het_rate, &c)) {
                if (G->calls.n == G->calls.cap) { G->calls.cap = G->calls.cap ? 2 * G->calls.cap : 1024; G->calls.c = realloc(G->calls.c, sizeof(ngo_call) * G->calls.cap); }
                G->calls.c[G->calls.n++] = c;
            }
        }
    }
    G->cur_pos++;
    return numAlignments > 0;
}

/* updatePendingAlns, :464-471 */
static void update_pending(ngo_gen* G) {
    int k = 0;
    for (int i = 0; i < G->pending.n; i++) {
        ngo_aln* a = G->pending.a[i];
        if (a->last >= G->cur_pos) G->pending.a[k++] = a;
        else alist_push(&G->retired, a);
    }
    G->pending.n = k;
    for (int i = 0; i < G->retired.n; i++) aln_free(G->retired.a[i]);
    G->retired.n = 0;
}

/* processPileups, :453-462 */
static void process_pileups(ngo_gen* G, int alignmentStart) {
    if (alignmentStart == G->cur_pos) return;
    while (G->cur_pos < alignmentStart) {
        if (!process_current_position(G)) {
            update_pending(G);
            if (G->pending.n == 0) G->cur_pos = alignmentStart;
        }
    }
    update_pending(G);
}

/* processSameStartAlns, :407-433 */
static void process_same_start(ngo_gen* G) {
    int posStart = 0;
    if (G->ss_primary.n > 0) posStart = G->ss_primary.a[0]->first;
    else if (G->ss_secondary.n > 0) posStart = G->ss_secondary.a[0]->first;
    if (posStart == 0) return;
    ngo_alist all = {0};
    for (int i = 0; i < G->ss_primary.n; i++) alist_push(&all, G->ss_primary.a[i]);
    for (int i = 0; i < G->ss_secondary.n; i++) alist_push(&all, G->ss_secondary.a[i]);
    G->ss_primary.n = G->ss_secondary.n = 0;
    /* Map<String,Integer> alnsPerReadGroup */
    int rgcap = 16; int* rgcnt = calloc(rgcap, sizeof(int));
    for (int i = 0; i < all.n; i++) {
        ngo_aln* a = all.a[i];
        if (a->rg + 1 >= rgcap) { int nc = (a->rg + 1) * 2; rgcnt = realloc(rgcnt, sizeof(int) * nc); memset(rgcnt + rgcap, 0, sizeof(int) * (nc - rgcap)); rgcap = nc; }
        int* cnt = &rgcnt[a->rg + 1];
        if (*cnt == 0) *cnt = 1;
        else if (G->p->max_alns_per_start <= 0 || *cnt < G->p->max_alns_per_start) (*cnt)++;
        else { aln_free(a); continue; }
        set_ignore(a, G->p->ignore5, G->p->ignore3);
        update_allele_calls(a);
        alist_push(&G->pending, a);
        G->st->alignments_admitted++;
    }
    free(rgcnt); free(all.a);
}

/* processAlignment, :377-403 */
static void process_alignment(ngo_gen* G, ngo_aln* a) {
    if (G->cur_seq >= 0) {
        int same = (G->cur_seq == a->seq);
        if (!same || G->last_start != a->first) {
            process_same_start(G);
            if (!same) {
                process_pileups(G, G->cur_last + 1);
                on_sequence_end(G);
                G->cur_seq = -1;
            } else process_pileups(G, a->first);
        }
    }
    if (G->cur_seq < 0) {   /* startSequence, :435-444 */
        G->cur_seq = a->seq; G->cur_pos = a->first; G->cur_last = a->last;
    }
    if (a->last > G->cur_last) G->cur_last = a->last;
    if (a->flags & FLAG_SECONDARY) alist_push(&G->ss_secondary, a);
    else alist_push(&G->ss_primary, a);
    G->last_start = a->first;
}

/* notifyEndOfAlignments, :447-452 */
static void notify_end(ngo_gen* G) {
    process_same_start(G);
    int lim = G->p->query_last < G->cur_last ? G->p->query_last : G->cur_last;
    process_pileups(G, lim + 1);
    if (G->cur_seq >= 0) on_sequence_end(G);
    G->cur_seq = -1;
}

/* ------------------------------------------------------------------ */
/* driver: ReadAlignmentFileReader iterator + SingleSampleVariantsDetector.findSNVS */
/* ------------------------------------------------------------------ */
static char* split_tab(char** s) {
    char* b = *s; if (!b) return NULL;
    char* t = strchr(b, '\t');
    if (t) { *t = 0; *s = t + 1; } else *s = NULL;
    return b;
}

int ngo_run_ssvd(const char* fasta, const char* sam, const char* out_vcf,
                 const char* dump_path, const ngo_params* p, ngo_stats* stats) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    ngo_stats st_local; ngo_stats* st = stats ? stats : &st_local;
    memset(st, 0, sizeof(*st));
    if (p->ploidy >= 3) return NGO_UNSUPPORTED;   /* pool algorithm (SingleSampleVariantPileupListener.java:240-254) */
    ngo_genome g;
    if (load_fasta(fasta, &g) != NGO_OK) return NGO_ERR_IO;
    FILE* in = fopen(sam, "r");
    if (!in) return NGO_ERR_IO;
    FILE* out = strcmp(out_vcf, "-") == 0 ? stdout : fopen(out_vcf, "w");
    if (!out) { fclose(in); return NGO_ERR_IO; }
    FILE* dump = dump_path ? fopen(dump_path, "w") : NULL;

    ngo_gen G; memset(&G, 0, sizeof(G));
    G.p = p; G.g = &g; G.out = out; G.dump = dump; G.cur_seq = -1; G.st = st;
    /* SingleSampleVariantsDetector.run, :591-593 */
    G.het_rate = p->het_rate;
    if (!p->het_rate_set && p->ploidy == 1) G.het_rate = 1e-6;
    print_header(out, p);

    int filterFlags = FLAG_UNMAPPED;          /* AlignmentsPileupGenerator.createReader, :367-372 */
    if (!p->process_secondary) {
        filterFlags |= FLAG_SECONDARY;
        if (!p->process_nonunique) filterFlags |= FLAG_MULTIPLE;
    }
    ngo_strlist rgs = {0};
    char* line = NULL; size_t lcap = 0; ssize_t l;
    char* last_qname = NULL; int last_start = -1, last_paired = 0, last_fop = 0, have_last = 0;
    int rc = NGO_OK;
    int query_found = 0;
    while ((l = getline(&line, &lcap, in)) >= 0) {
        while (l > 0 && (line[l - 1] == '\n' || line[l - 1] == '\r')) line[--l] = 0;
        if (l == 0) continue;
        if (line[0] == '@') {
            if (strncmp(line, "@RG", 3) == 0) {
                char* id = strstr(line, "\tID:");
                if (id) { id += 4; char* e = strchr(id, '\t'); char save = 0; if (e) { save = *e; *e = 0; } strlist_get(&rgs, id, 1); if (e) *e = save; }
            }
            continue;
        }
        char* cur = line;
        char* f[11];
        int nf = 0;
        for (; nf < 11; nf++) { f[nf] = split_tab(&cur); if (!f[nf]) break; }
        if (nf < 11) continue;   /* malformed record skipped (ReadAlignmentFileReader.java:330-335) */
        char* tags = cur;
        st->alignments_read++;
        int flag = atoi(f[1]);
        int start = atoi(f[3]);
        int paired = (flag & 1) != 0, fop = (flag & 0x40) != 0;
        /* isSameAlignment, ReadAlignmentFileReader.java:292-306 */
        if (have_last && last_start == start && last_paired == paired && (!paired || last_fop == fop) && strcmp(last_qname, f[0]) == 0) continue;
        free(last_qname); last_qname = strdup(f[0]); last_start = start; last_paired = paired; last_fop = fop; have_last = 1;
        /* loadAlignment, :219-272 */
        int nh = 0, nh_present = 0, rg = -1;
        for (char* t = tags; t && *t;) {
            char* tag = split_tab(&t);
            if (strncmp(tag, "NH:i:", 5) == 0) { nh = atoi(tag + 5); nh_present = 1; }
            /* htsjdk getReadGroup() is null for ids missing from the header -> DEF_READ_GROUP "" */
            else if (strncmp(tag, "RG:Z:", 5) == 0) rg = strlist_get(&rgs, tag + 5, 0);
        }
        int mapq = atoi(f[4]);
        int flags = flag;
        /* isMultiple, :284-291 */
        int multiple;
        if (flag & FLAG_SECONDARY) multiple = 1;
        else if (nh_present && nh > 1) multiple = 1;
        else if (nh_present && nh == 1) multiple = 0;
        else multiple = mapq < p->min_mq;
        if (multiple) flags += FLAG_MULTIPLE;
        if (flag & FLAG_UNMAPPED) continue;
        int seq = genome_find(&g, f[2]);
        if (seq < 0) continue;   /* sequence not in the reference: loadAlignment throws, record skipped */
        ngo_aln* a = calloc(1, sizeof(ngo_aln));
        a->seq = seq; a->first = start; a->flags = flags; a->rg = rg;
        int seqlen = strcmp(f[9], "*") == 0 ? 0 : (int)strlen(f[9]);
        a->read_length = seqlen;
        if (strcmp(f[5], "*") == 0 || parse_cigar(f[5], &a->ops, &a->n_ops) != 0) { aln_free(a); continue; }
        int expRead = 0, expEnd = start;
        for (int i = 0; i < a->n_ops; i++) {
            int op = a->ops[i] & 7, len = a->ops[i] / 8;
            if (op & 2) expRead += len;
            if (op & 1) expEnd += len;
            if (op == OP_D || op == OP_I) a->has_indel = 1;
        }
        a->last = expEnd - 1;     /* htsjdk getAlignmentEnd == setCigarString's expected end */
        a->read_length = expRead;
        if (seqlen > 0) {
            if (seqlen != a->read_length) { aln_free(a); continue; }   /* setReadCharacters throws */
            a->chars = malloc(seqlen + 1);
            for (int i = 0; i < seqlen; i++) { char c = (char)toupper((unsigned char)f[9][i]); a->chars[i] = c == '.' ? 'N' : c; }
            a->chars[seqlen] = 0;
            if (strcmp(f[10], "*") != 0) {
                /* setQualityScores, ReadAlignment.java:581-595 */
                a->quals = malloc(a->read_length);
                memset(a->quals, 38, a->read_length);
                int ql = (int)strlen(f[10]);
                for (int i = 0; i < ql && i < a->read_length; i++) { int sig = (unsigned char)f[10][i]; a->quals[i] = (uint8_t)(sig > 127 ? 127 : sig); }
            }
        }
        if ((flags & filterFlags) != 0) { aln_free(a); continue; }
        /* querySeq handling, AlignmentsPileupGenerator.java:310-322 */
        if (p->query_seq) {
            if (strcmp(p->query_seq, g.s[seq].name) == 0) {
                query_found = 1;
                if (a->first > p->query_last) { aln_free(a); break; }
                if (p->query_first > a->last) { aln_free(a); continue; }
            } else if (query_found) { aln_free(a); break; }
            else { aln_free(a); continue; }
        }
        if (a->has_indel) { G.unsupported = 1; aln_free(a); rc = NGO_UNSUPPORTED; break; }
        process_alignment(&G, a);
    }
    if (rc == NGO_OK) notify_end(&G);
    free(line); free(last_qname); fclose(in);
    if (out != stdout) fclose(out); else fflush(out);
    if (dump) fclose(dump);
    for (int i = 0; i < G.pending.n; i++) aln_free(G.pending.a[i]);
    for (int i = 0; i < G.ss_primary.n; i++) aln_free(G.ss_primary.a[i]);
    for (int i = 0; i < G.ss_secondary.n; i++) aln_free(G.ss_secondary.a[i]);
    free(G.pending.a); free(G.ss_primary.a); free(G.ss_secondary.a); free(G.retired.a); free(G.calls.c);
    for (int i = 0; i < g.n; i++) { free(g.s[i].name); free(g.s[i].seq); }
    free(g.s);
    for (int i = 0; i < rgs.n; i++) free(rgs.ids[i]);
    free(rgs.ids);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    st->seconds = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    return rc;
}
