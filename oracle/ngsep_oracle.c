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
 * ploidy 1/2 (SNVQ) and >= 3 (the pool algorithm), SNV-only alignments (no I/D CIGAR operations: the indel realigner
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
#define NGO_ERR_ARG 4

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

/* an indel call of an alignment: GenomicVariantImpl(seq, refPos, refLast, TYPE_INDEL) with setLength(opLen),
 * keyed by refPos = the reference position of the base before the event (ReadAlignment.java:798-815) */
typedef struct { int first, last, len; } ngo_indel;

typedef struct ngo_aln {
    int seq;                 /* genome index */
    int first, last, read_length, flags, rg;
    int n_ops; int* ops;     /* len*8+op, ReadAlignment.java:1180-1198 */
    char* chars;             /* NULL if '*' */
    uint8_t* quals;          /* NULL if '*' */
    int ignore_start, ignore_end;
    int16_t* acl;            /* alleleCallLength, :747-834 */
    int id;                  /* the record's ordinal among the SAM's alignment lines (the realigner trace's key) */
    int has_indel;
    int n_indel, cap_indel;  /* indelCalls (TreeMap by refPos: ascending), rebuilt with acl */
    ngo_indel* indel;
} ngo_aln;

static void aln_free(ngo_aln* a) { free(a->ops); free(a->chars); free(a->quals); free(a->acl); free(a->indel); free(a); }

/* ReadAlignment.updateAlleleCallsInfo, ReadAlignment.java:747-834: alleleCallLength per read position and the
 * indel calls (recomputed after every change of the alignment or of the bases to ignore, which is when the
 * reference's lazy alleleCallsUpdated flag would trigger it) */
static void update_allele_calls(ngo_aln* a) {
    free(a->acl);
    a->acl = calloc(a->read_length > 0 ? a->read_length : 1, sizeof(int16_t));
    a->n_indel = 0;
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
                        if (j == len - 1 && nextIsIndel) {
                            a->acl[readPos] = (nextOp == OP_I) ? (int16_t)(nextLen + 2) : 2;
                            int refLast = refPos + 1;
                            if (nextOp != OP_I) refLast += nextLen;
                            if (a->n_indel == a->cap_indel) { a->cap_indel = a->cap_indel ? 2 * a->cap_indel : 4; a->indel = realloc(a->indel, sizeof(ngo_indel) * a->cap_indel); }
                            /* TreeMap.put: a later event at the same key replaces the earlier one */
                            if (a->n_indel > 0 && a->indel[a->n_indel - 1].first == refPos) a->n_indel--;
                            a->indel[a->n_indel].first = refPos; a->indel[a->n_indel].last = refLast; a->indel[a->n_indel].len = nextLen;
                            a->n_indel++;
                        } else a->acl[readPos] = 1;
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
    const char* id;           /* -knownVariants: the input variant's ID (NULL: '.') */
    int known;                /* 1: a genotyped input variant (genotype 0 hom-ref, -1 undecided allowed) */
    int logc_present;         /* 0: no log-conditionals (an undecided call without allele calls) */
    int embedded;             /* TYPE_EMBEDDED_SNV (-embeddedSNVs inside a called indel, :227) */
    struct ngo_indel_call_s* indel;   /* an indel / STR call instead of an SNV (ngsep_oracle_indel.inc) */
    struct ngo_kindel* kindel;        /* -knownVariants: a genotyped input indel / MNP (GenomicVariantImpl) instead */
    int known_type;                   /* -knownVariants: the input record's INFO TYPE id (printed when 2-5) */
    /* ploidy >= 3 (genotypeVariantPool): a CalledGenomicVariantImpl over the pool variant's alleles */
    int pool;                 /* 1: the fields below describe the call, logc[][] is over the variant alleles */
    int pool_n;               /* variant alleles: DNA indexes pool_dna[0..n) (reference first) */
    int pool_dna[4];
    int pool_multi;           /* TYPE_MULTIALLELIC_SNV (INFO TYPE=MULTISNV) */
    int pool_ncalled, pool_called[2];
    int pool_report;          /* VariantCallReport present (counts + log-conditionals) */
    int pool_counts[4];       /* report counts over the variant alleles (ADP) */
    int pool_acn[4], pool_total_cn;
} ngo_call;

typedef struct { ngo_call* c; int n, cap; } ngo_calls;

static const char* BASES = "ACGT";
/* GenomicVariantImpl.getVariantTypeName for the types a -knownVariants record can carry here (2-5) */
static const char* type_name(int t) {
    static const char* names[] = {NULL, NULL, "MULTISNV", "EMBEDDED", "INDEL", "STR"};
    return t >= 2 && t <= 5 ? names[t] : NULL;
}
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

/* VCFFileHeader.print with the samples of MultisampleVariantsDetector (vcf/VCFFileHeader.java:219-245) */
static void print_header_samples(FILE* out, const ngo_params* p, const char* const* ids, int n) {
    ngo_params q = *p;
    q.print_sample_ploidy = 0;
    q.sample_id = "";
    /* reuse the fixed lines; the sample part differs */
    FILE* tmp = out;
    static const char* tail = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT";
    char* buf = NULL; size_t len = 0;
    FILE* mem = open_memstream(&buf, &len);
    print_header(mem, &q);
    fclose(mem);
    char* cut = strstr(buf, "#CHROM");
    if (cut) *cut = 0;
    fputs(buf, tmp);
    free(buf);
    if (p->print_sample_ploidy)
        for (int i = 0; i < n; i++) fprintf(tmp, "##SAMPLE=<ID=%s,PL=%d>\n", ids[i], p->ploidy);
    fputs(tail, tmp);
    for (int i = 0; i < n; i++) fprintf(tmp, "\t%s", ids[i]);
    fputs("\n", tmp);
}

/* one VCF line per call: VCFFileWriter.printVCFRecord + printGenotypeInfo */
static void print_pool_call(FILE* out, const char* seqName, const ngo_call* c) {
    /* a CalledGenomicVariantImpl of genotypeVariantPool: FORMAT NGSEP_NOSNV (discovery: no getAllCounts) or
     * NGSEP_SNV (-knownVariants: setAllCounts), SingleSampleVariantsDetector.java:942-946 */
    const int n = c->pool_n;
    fprintf(out, "%s\t%d\t%s\t%c\t", seqName, c->pos, c->id ? c->id : ".", c->ref);
    for (int i = 1; i < n; i++) fprintf(out, "%s%c", i > 1 ? "," : "", BASES[c->pool_dna[i]]);
    if (c->embedded) fprintf(out, "\t%d\t.\tTYPE=EMBEDDED", c->qual);        /* an SNV inside an indel (:227) */
    else if (c->pool_multi) fprintf(out, "\t%d\t.\tTYPE=MULTISNV", c->qual);
    else if (type_name(c->known_type)) fprintf(out, "\t%d\t.\tTYPE=%s", c->qual, type_name(c->known_type));
    else fprintf(out, "\t%d\t.\t.", c->qual);
    fprintf(out, c->known ? "\tGT:PL:GQ:DP:BSDP:ACN\t" : "\tGT:PL:GQ:DP:ADP:ACN\t");
    if (c->pool_ncalled == 0) fprintf(out, "./.");
    else if (c->pool_ncalled == 1) fprintf(out, "%d/%d", c->pool_called[0], c->pool_called[0]);
    else fprintf(out, "%d/%d", c->pool_called[0], c->pool_called[1]);
    fprintf(out, ":");
    for (int j = 0; j < n; j++)
        for (int i = 0; i <= j; i++) {
            if (i > 0 || j > 0) fprintf(out, ",");
            fprintf(out, "%d", c->pool_report ? (int)ngo_java_round(-10 * c->logc[i][j]) : 0);
        }
    fprintf(out, ":%d:%d:", c->gq, c->dp);
    if (c->known) fprintf(out, "%d,%d,%d,%d", c->counts[0], c->counts[1], c->counts[2], c->counts[3]);
    else for (int i = 0; i < n; i++) fprintf(out, "%s%d", i ? "," : "", c->pool_report ? c->pool_counts[i] : 0);
    fprintf(out, ":");
    if (c->pool_total_cn == 0) fprintf(out, ".");
    else
        for (int j = 0; j < n; j++) {
            int v = c->pool_acn[j];
            if (c->pool_ncalled == 0 && j == 0) v = c->pool_total_cn;
            fprintf(out, "%s%d", j ? "," : "", v);
        }
    fprintf(out, "\n");
}

static void print_indel_call_any(FILE* out, const char* seqName, const ngo_call* c);
static void print_kindel(FILE* out, const char* seqName, const struct ngo_kindel* k);
static void free_kindel(struct ngo_kindel* k);
static void print_call(FILE* out, const char* seqName, const ngo_call* c) {
    if (c->indel) { print_indel_call_any(out, seqName, c); return; }
    if (c->kindel) { print_kindel(out, seqName, c->kindel); return; }
    if (c->pool) { print_pool_call(out, seqName, c); return; }
    fprintf(out, "%s\t%d\t%s\t%c\t", seqName, c->pos, c->id ? c->id : ".", c->ref);
    if (c->n_alleles == 2) fprintf(out, "%c", BASES[c->idx[1]]);
    else fprintf(out, "%c,%c", BASES[c->idx[1]], BASES[c->idx[2]]);
    fprintf(out, "\t%d\t.\t", c->qual);
    /* INFO: FS (SingleSampleVariantsDetector.java:957, CalledSNV only) then TYPE (VCFFileWriter.java:47-49) */
    int printed = 0;
    if (c->n_alleles == 2 && c->strand_bias != -1) { fprintf(out, "FS=%d", c->strand_bias); printed = 1; }
    if (c->embedded) { fprintf(out, "%sTYPE=EMBEDDED", printed ? ";" : ""); printed = 1; }
    else if (c->n_alleles == 3) { fprintf(out, "%sTYPE=MULTISNV", printed ? ";" : ""); printed = 1; }
    else if (type_name(c->known_type)) { fprintf(out, "%sTYPE=%s", printed ? ";" : "", type_name(c->known_type)); printed = 1; }
    if (!printed) fprintf(out, ".");
    fprintf(out, "\tGT:PL:GQ:DP:BSDP:ACN\t");
    int ploidy = c->ploidy;
    if (c->n_alleles == 2) {
        /* CalledSNV: GT (VCFFileWriter.java:168-197) */
        if (c->genotype == 2) { fprintf(out, "1"); if (ploidy > 1) fprintf(out, "/1"); }
        else if (c->genotype == 0) { fprintf(out, "0"); if (ploidy > 1) fprintf(out, "/0"); }
        else if (c->genotype == -1) { fprintf(out, "."); if (ploidy > 1) fprintf(out, "/."); }
        else fprintf(out, "0/1");
        fprintf(out, ":");
        /* PL from float log-conds (CalledSNV.java:259-265, :413-435; VCFFileWriter.java:200-212) */
        float hr = (float)c->logc[c->idx[0]][c->idx[0]];
        float ha = (float)c->logc[c->idx[1]][c->idx[1]];
        float ra = (float)c->logc[c->idx[0]][c->idx[1]];
        float ar = (float)c->logc[c->idx[1]][c->idx[0]];
        double lc[2][2] = {{hr, ra}, {ar, ha}};
        int present = c->logc_present && (hr + ra + ar + ha) != 0;
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
        else if (c->genotype == 0 || c->genotype == -1) refcn = total;   /* hom-ref; undecided: ACN[0] = total (:237) */
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
    out->logc_present = 1;
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
/* -knownVariants: SingleSampleVariantPileupListener.onPileup with input variants (:158-176) ->      */
/* genotypeVariantSample (:361-391) -> VariantDiscoverySNVQAlgorithm.genotypeSNV (:21-62), biallelic  */
/* SNVs as VCFFileReader.loadGenomicVariant makes them (vcf/VCFFileReader.java:196-260)               */
/* ------------------------------------------------------------------ */
typedef struct {
    int seq, pos, last;       /* last = pos + |REF| - 1 (GenomicVariantImpl(seq, first, alleles)) */
    char ref, alt;            /* a biallelic SNV (snv = 1): its bases */
    int qs; char* id;
    int snv;                  /* 1: an SNV object (two alleles of one base each, VCFFileReader.java:243-248) */
    int n_alleles; char** alleles;   /* a GenomicVariantImpl (snv = 0): its alleles, reference first */
    int type;                 /* INFO TYPE (VCFFileReader.loadInfoField :274-279): 0 undetermined, 2-5 */
} ngo_known;
static void genotype_known(const ngo_counts* h, const ngo_known* kv, const ngo_params* p, double hetRate, ngo_call* out) {
    memset(out, 0, sizeof(*out));
    out->pos = kv->pos; out->ref = kv->ref; out->n_alleles = 2; out->known = 1; out->id = kv->id;
    out->idx[0] = base_idx(kv->ref); out->idx[1] = base_idx(kv->alt);
    out->qual = kv->qs;                         /* the input variant's QS: genotypeSNV sets none */
    out->known_type = kv->type;
    out->strand_bias = -1;                      /* genotypeSNV(.., calcStrandBias = false) */
    out->ploidy = p->ploidy;
    out->dp = h->total_count;
    memcpy(out->counts, h->counts, sizeof(out->counts));
    if (h->total_count == 0) { out->genotype = -1; return; }   /* undecided, no log-conditionals (:23-27) */
    out->logc_present = 1;
    for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) out->logc[i][j] = h->logc[i][j];
    double post[16];
    ngo_counts_posteriors(h, hetRate, post);
    const int r = out->idx[0], a = out->idx[1];
    double pMax = post[r * 4 + r];
    int gt = 0;
    if (post[a * 4 + a] > pMax + 0.01) { pMax = post[a * 4 + a]; gt = 2; }
    const double pHet = post[r * 4 + a] + post[a * 4 + r];
    if (pHet > pMax + 0.01) { pMax = pHet; gt = 1; }
    int gq = ngo_phred(1 - pMax);
    if (gq == 0) gt = -1;
    if ((int16_t)p->min_quality > gq) { gt = -1; gq = 0; }   /* makeUndecided (:388) */
    out->genotype = gt;
    out->gq = gq;
}

/* ------------------------------------------------------------------ */
/* AlignmentsPileupGenerator sweep (discovery/AlignmentsPileupGenerator.java:377-504) */
/* ------------------------------------------------------------------ */
typedef struct { ngo_aln** a; int n, cap; } ngo_alist;
static void alist_push(ngo_alist* l, ngo_aln* a) {
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 64; l->a = realloc(l->a, sizeof(ngo_aln*) * l->cap); }
    l->a[l->n++] = a;
}

/* one PileupAlleleCall of span 1 as calculateCountsGTSNV reads it (CountsHelper.java:86-95) */
typedef struct { int base; int q; int neg; } ngo_acall;   /* base: DNA index or -1; q = min(30, qual-33) */
typedef struct { ngo_acall* c; int n, cap; } ngo_acalls;
static void acalls_push(ngo_acalls* l, int base, int q, int neg) {
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 64; l->c = realloc(l->c, sizeof(ngo_acall) * l->cap); }
    l->c[l->n].base = base; l->c[l->n].q = q; l->c[l->n].neg = neg; l->n++;
}

struct ngo_mvd;
typedef struct ngo_strv { int seq, first, last; } ngo_strv;   /* an input STR variant (-knownSTRs) */
typedef struct {
    const ngo_params* p;
    struct ngo_mvd* mvd;       /* MultisampleVariantsDetector listener instead of the single-sample one */
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
    ngo_coverage* cov;         /* CoverageStatisticsCalculator listener instead of the variant listeners */
    struct ngo_rac* rac;       /* RelativeAlleleCountsCalculator listener instead of the variant listeners */
    ngo_known* known;          /* -knownVariants (sequence order, then position, input order kept) */
    int n_known, known_next;   /* known_next: nextSIVIndex over the whole list */
    ngo_acalls acalls;         /* ploidy >= 3: the position's allele calls in pending order */
    int realign;               /* IndelRealignerPileupListener active (single-sample discovery, ploidy < 3) */
    int last_indel_end;        /* SingleSampleVariantPileupListener.lastIndelEnd, :143 */
    ngo_alist pileup;          /* the position's alignments (PileupRecord.getAlignments) */
    struct ngo_strv* strs;     /* -knownSTRs: the realigner's input STR variants (sequence order, then first, last) */
    int n_strs, str_next;      /* str_next: IndelRealignerPileupListener.idxNextVariant over the whole list */
    int rk_next;               /* -knownVariants: the realigner's idxNextVariant over `known` (its own index) */
} ngo_gen;

/* IndelRealignerPileupListener.intersectWithVariants (:141-157): the input variant at pos (first 0: none) -- the
 * -knownVariants records when given (SingleSampleVariantsDetector.java:897-905, MultisampleVariantsDetector.java:
 * 432-438), else the -knownSTRs (always TYPE_STR) */
static void realigner_input_at(ngo_gen* G, int pos, int* first, int* last, int* is_str) {
    *first = *last = *is_str = 0;
    if (G->known) {
        while (G->rk_next < G->n_known && G->known[G->rk_next].seq == G->cur_seq) {
            const ngo_known* v = &G->known[G->rk_next];
            if (pos < v->pos) break;
            if (pos <= v->last) { *first = v->pos; *last = v->last; *is_str = v->type == 5; return; }
            G->rk_next++;
        }
        return;
    }
    while (G->str_next < G->n_strs && G->strs[G->str_next].seq == G->cur_seq) {
        const ngo_strv* v = &G->strs[G->str_next];
        if (pos < v->first) break;
        if (pos <= v->last) { *first = v->first; *last = v->last; *is_str = 1; return; }
        G->str_next++;
    }
}

/* ------------------------------------------------------------------ */
/* RelativeAlleleCountsCalculator (discovery/RelativeAlleleCountsCalculator.java:246-331) with the     */
/* math.Distribution it fills (math/Distribution.java:52-93,301-345)                                    */
/* ------------------------------------------------------------------ */
#define RAC_PROP_BINS 51           /* Distribution(0, 0.5, 0.01): (int)((0.5 - 0) / 0.01) + 1 */
#define RAC_NALL_BINS 10           /* Distribution(1, 10, 1) */
typedef struct {
    double dist[RAC_PROP_BINS];
    double sum, sum_sq, count;
} rac_dist;
typedef struct ngo_rac {
    int min_rd, min_bq;
    rac_dist prop;
    double nall[RAC_NALL_BINS], nall_sum, nall_sum_sq, nall_count;
    int n_seq;                     /* sequences longer than 100000 bp (onSequenceStart, :312-322) */
    char** seq_names;
    rac_dist* seq_dist;
    rac_dist* cur;                 /* currentSequencePropDist (NULL for short sequences) */
    int64_t covered;               /* coveredGenomeSize */
} ngo_rac;

/* Distribution.processDatapoint(1, value) for the bins that cannot overflow here */
static void rac_point(rac_dist* d, double v) {
    d->sum += v;
    d->sum_sq += v * v;
    d->count += 1;
    d->dist[(int)((v - 0.0) / 0.01)] += 1;
}

/* onPileup (:246-294): calls = getAlleleCalls(1); alleles counted by their character when the call's
 * quality is >= minBaseQualityScore; the proportion of the second most frequent allele among the two
 * most frequent ones (TreeMap order, strict maxima: the first of equal counts wins, :296-308) */
static void rac_on_pileup(ngo_gen* G, int pos) {
    ngo_rac* R = G->rac;
    int ncalls = 0;
    int cnt[256];
    memset(cnt, 0, sizeof(cnt));
    for (int k = 0; k < G->pending.n; k++) {
        ngo_aln* a = G->pending.a[k];
        if (a->first > pos || a->last < pos) continue;
        if (!a->chars) continue;
        int rp = aligned_read_pos(a, pos);
        if (rp < 0) continue;
        if (a->acl[rp] != 1) continue;                  /* PileupRecord.getAlleleCalls(1), :126-152 */
        ncalls++;
        int qc = a->quals ? a->quals[rp] : '+';          /* getQualityScores: '+' without qualities */
        int qs = (int)(int8_t)(uint8_t)qc - 33;
        if (qs >= R->min_bq) cnt[(uint8_t)a->chars[rp]]++;
    }
    if (ncalls < R->min_rd) return;
    int n_all = 0;
    for (int c = 0; c < 256; c++) n_all += cnt[c] > 0;
    if (n_all == 0) return;
    {   /* distNumAlleles.processDatapoint(alleleCounts.size()) */
        double v = n_all;
        R->nall_sum += v; R->nall_sum_sq += v * v; R->nall_count += 1;
        R->nall[(int)((v - 1.0) / 1.0)] += 1;
    }
    int mx = -1, mc = -1;                               /* TreeMap iteration: ascending characters */
    for (int c = 0; c < 256; c++) if (cnt[c] > 0 && (mx < 0 || mc < cnt[c])) { mx = c; mc = cnt[c]; }
    int sc = 0, s2 = -1;
    for (int c = 0; c < 256; c++) if (c != mx && cnt[c] > 0 && (s2 < 0 || sc < cnt[c])) { s2 = c; sc = cnt[c]; }
    if (mc > 0) {
        double prop = (double)sc / (mc + sc);
        rac_point(&R->prop, prop);
        if (R->cur) rac_point(R->cur, prop);
    }
    R->covered++;
}

static void rac_on_sequence_start(ngo_gen* G, int seq) {
    ngo_rac* R = G->rac;
    if (G->g->s[seq].len > 100000) {
        R->seq_names = realloc(R->seq_names, sizeof(char*) * (R->n_seq + 1));
        R->seq_dist = realloc(R->seq_dist, sizeof(rac_dist) * (R->n_seq + 1));
        R->seq_names[R->n_seq] = G->g->s[seq].name;
        memset(&R->seq_dist[R->n_seq], 0, sizeof(rac_dist));
        R->n_seq++;
        R->cur = &R->seq_dist[R->n_seq - 1];
    } else {
        R->cur = NULL;
    }
}

static void rac_fmt(FILE* out, double x) { char b[64]; ngo_java_fmt2(x, b, sizeof b); fputs(b, out); }

/* Distribution.printDistribution (:301-345) of a distribution with no outliers */
static void rac_print_dist(FILE* out, const double* dist, int nbins, double min, double bin, double max, int integer,
                           double count, double sum, double sum_sq) {
    int maxIdx = (int)((max - min) / bin);
    for (int i = 0; i < nbins && i <= maxIdx; i++) {
        if (integer) fprintf(out, "%d\t%lld\n", (int)(min + i * bin), (long long)ngo_java_round(dist[i]));
        else { rac_fmt(out, min + i * bin); fputc('\t', out); rac_fmt(out, dist[i]); fputc('\n', out); }
    }
    fprintf(out, "Count\t%lld\n", (long long)ngo_java_round(count));
    if (integer) fprintf(out, "Sum\t%lld\n", (long long)ngo_java_round(sum));
    else { fputs("Sum\t", out); rac_fmt(out, sum); fputc('\n', out); }
    if (count > 0) { fputs("Average\t", out); rac_fmt(out, sum / count); fputc('\n', out); }
    if (count > 1) {
        double var = (sum_sq - sum * sum / count) / (count - 1);
        fputs("Variance\t", out); rac_fmt(out, var); fputc('\n', out);
        fputs("STDev\t", out); rac_fmt(out, sqrt(var)); fputc('\n', out);
    }
}

/* printResults (:213-244) */
static void rac_print(FILE* out, const ngo_rac* R) {
    fprintf(out, "Distribution of allele proportions\n");
    rac_print_dist(out, R->prop.dist, RAC_PROP_BINS, 0.0, 0.01, 0.5, 0, R->prop.count, R->prop.sum, R->prop.sum_sq);
    fprintf(out, "Distribution of number of alleles\n");
    rac_print_dist(out, R->nall, RAC_NALL_BINS, 1.0, 1.0, 10.0, 1, R->nall_count, R->nall_sum, R->nall_sum_sq);
    if (R->n_seq == 0) return;
    fprintf(out, "Distribution of allele proportions per sequence\n");
    fprintf(out, "Proportion");
    for (int i = 0; i < R->n_seq; i++) fprintf(out, "\t%s", R->seq_names[i]);
    fputc('\n', out);
    double min = 0;
    for (int b = 0; b < RAC_PROP_BINS; b++) {
        rac_fmt(out, min);
        for (int i = 0; i < R->n_seq; i++) { fputc('\t', out); rac_fmt(out, R->seq_dist[i].dist[b]); }
        fputc('\n', out);
        min += 0.01;
    }
}

static void free_indel_call(struct ngo_indel_call_s* c);
static void pool_known_first_cn(ngo_call* c, int ploidy);
static void on_sequence_end(ngo_gen* G) {
    /* SingleSampleVariantsDetector.saveSequenceVariants, :933-968: calls are already in position order.
     * intersectVariantsCNVs (:969-1008) calls updateAllelesCopyNumberFromCounts(normalPloidy) on the first call only
     * (with no CNV the index runs to the end and the loop breaks): it matters for the pool algorithm's input records,
     * whose ACN genotypeVariantPool set (setAllelesCopyNumber :498) */
    if (G->calls.n > 0) pool_known_first_cn(&G->calls.c[0], G->p->ploidy);
    for (int i = 0; i < G->calls.n; i++) {
        print_call(G->out, G->g->s[G->cur_seq].name, &G->calls.c[i]);
        if (G->calls.c[i].indel) free_indel_call(G->calls.c[i].indel);
        if (G->calls.c[i].kindel) free_kindel(G->calls.c[i].kindel);
    }
    G->st->variants_called += G->calls.n;
    G->calls.n = 0;
}

/* ------------------------------------------------------------------ */
/* MultisampleVariantsDetector, SNV-only (discovery/MultisampleVariantsDetector.java:522-693) */
/* ------------------------------------------------------------------ */
/* Java String.hashCode */
static int32_t java_string_hash(const char* s) {
    uint32_t h = 0;
    for (; *s; s++) h = 31u * h + (uint8_t)*s;
    return (int32_t)h;
}
/* Iteration order of a java.util.HashSet<String> filled in the given order (Sample.readGroups,
 * variants/Sample.java:36): buckets of the final table (16, doubled past 0.75 load), insertion
 * order inside a bucket.  Used for PileupRecord.getAlleleCalls(span, readGroups) (:104-111). */
static void java_hashset_order(char** ids, int* idx, int n) {
    int cap = 16;
    while (n > cap * 3 / 4) cap *= 2;
    int* bucket = malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        uint32_t h = (uint32_t)java_string_hash(ids[idx[i]]);
        bucket[i] = (int)((h ^ (h >> 16)) & (uint32_t)(cap - 1));
    }
    for (int i = 1; i < n; i++) {          /* stable insertion sort by bucket */
        int b = bucket[i], v = idx[i], j = i - 1;
        while (j >= 0 && bucket[j] > b) { bucket[j + 1] = bucket[j]; idx[j + 1] = idx[j]; j--; }
        bucket[j + 1] = b; idx[j + 1] = v;
    }
    free(bucket);
}

/* ------------------------------------------------------------------ */
/* Ploidy >= 3: SingleSampleVariantPileupListener.genotypeVariantPool (:402-503), the pool paths of   */
/* discoverSNV (:234-255), genotypeVariantSample (:361-391) and createSNVVariantPool (:297-332)       */
/* ------------------------------------------------------------------ */

typedef struct {
    int n_called, called[2];  /* indexes into the variant alleles, ascending */
    int gq, dp;               /* dp: setTotalReadDepth (0 for the low-count undecided call) */
    int report;               /* VariantCallReport present */
    int counts[4];            /* report counts over the variant alleles */
    double logc[4][4];        /* report log-conditionals over the variant alleles */
    int acn[4], total_cn;
} ngo_pcall;

/* CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts (variants/CalledGenomicVariantImpl.java:228-282) */
static void pool_update_cn(ngo_pcall* c, int total) {
    c->total_cn = total;
    for (int i = 0; i < 4; i++) c->acn[i] = 0;
    if (c->n_called == 0) return;
    if (c->n_called == 1 && c->called[0] == 0) { c->acn[0] = total; return; }
    int nc = c->n_called;
    if (total <= nc) { for (int i = 0; i < nc; i++) c->acn[c->called[i]] = 1; return; }
    if (!c->report) {
        int def = total / nc;
        for (int i = 0; i < nc; i++) c->acn[c->called[i]] = def;
        c->acn[c->called[0]] += total - def * nc;
        return;
    }
    int rc[2], tr = 0;
    for (int i = 0; i < nc; i++) { rc[i] = c->counts[c->called[i]]; if (rc[i] == 0) rc[i] = 1; tr += rc[i]; }
    int tc = 0;
    for (int i = 0; i < nc; i++) {
        int64_t r = ngo_java_round((double)total * rc[i] / tr);
        c->acn[c->called[i]] = (int)(r > 1 ? r : 1);
        tc += c->acn[c->called[i]];
    }
    if (tc < total) c->acn[c->called[0]] += total - tc;
    else {
        int ex = tc - total;
        for (int i = nc - 1; ex > 0 && i >= 0; i--) {
            int j = c->called[i];
            int rm = ex < c->acn[j] - 1 ? ex : c->acn[j] - 1;
            c->acn[j] -= rm; ex -= rm;
        }
    }
}

/* CountsHelper.calculateCountsGTSNV(alleles, calls, maxBaseQS, freq) (CountsHelper.java:86-95) */
static void pool_helper(ngo_counts* h, const int* dna, int n, const ngo_acalls* calls, double freq, int max_base_qs) {
    ngo_counts_init(h, n, freq, max_base_qs);
    for (int k = 0; k < calls->n; k++) {
        int idx = -1;                                    /* alleles.indexOf(allele) */
        for (int i = 0; i < n; i++) if (calls->c[k].base >= 0 && dna[i] == calls->c[k].base) { idx = i; break; }
        ngo_counts_update(h, idx, calls->c[k].q, calls->c[k].neg);
    }
}

/* genotypeVariantPool (SingleSampleVariantPileupListener.java:402-503) for the variant with alleles dna[0..n) */
static void genotype_pool(const int* dna, int n, int haplotypes, const ngo_acalls* calls, double h, int max_base_qs,
                          ngo_pcall* out) {
    memset(out, 0, sizeof(*out));
    double step = 1.0 / (double)haplotypes;
    int nf = 0;
    for (double freq = step; freq < 0.51; freq += step) nf++;
    double* freqs = malloc(sizeof(double) * (nf ? nf : 1));
    ngo_counts* hs = malloc(sizeof(ngo_counts) * (nf ? nf : 1));
    nf = 0;
    for (double freq = step; freq < 0.51; freq += step) {
        freqs[nf] = freq;
        pool_helper(&hs[nf], dna, n, calls, freq, max_base_qs);
        nf++;
    }
    const ngo_counts* helper = &hs[0];
    const int* counts = helper->counts;
    int major = 0;                                       /* NumberArrays.getIndexMaximum: first maximum */
    for (int i = 1; i < n; i++) if (counts[major] < counts[i]) major = i;
    if (counts[major] < haplotypes) {                    /* undecided, no report (:436-440) */
        pool_update_cn(out, haplotypes);
        free(freqs); free(hs);
        return;
    }
    double logPriorHetero = log10(h), logPriorHomo = log10(1 - h);
    double* terms = malloc(sizeof(double) * (nf + 1));
    double termHomozygous = helper->logc[major][major] + logPriorHomo;
    double maxHetPosterior = 0, minHomoPosterior = 1, maxFreq = 0;
    int maxFreqIdx = 0, maxAlt = -1;
    for (int i = 0; i < n; i++) {
        if (i == major) continue;
        terms[0] = termHomozygous;
        for (int j = 0; j < nf; j++) terms[j + 1] = hs[j].logc[major][i] + logPriorHetero;
        calc_posteriors(terms, nf + 1);
        int idxMax = 0;
        for (int j = 1; j <= nf; j++) if (terms[idxMax] < terms[j]) idxMax = j;
        if (idxMax == 0) {
            if (terms[0] < minHomoPosterior) minHomoPosterior = terms[0];
        } else if (maxAlt == -1 || maxHetPosterior < terms[idxMax]) {
            maxHetPosterior = terms[idxMax];
            maxFreqIdx = idxMax - 1;
            maxFreq = freqs[maxFreqIdx];
            maxAlt = i;
        }
    }
    free(terms);
    if (maxAlt == -1) { out->n_called = 1; out->called[0] = major; }
    else {
        out->n_called = 2;
        out->called[0] = major < maxAlt ? major : maxAlt;
        out->called[1] = major < maxAlt ? maxAlt : major;
    }
    out->dp = helper->total_count;
    if (maxAlt == -1) {
        out->gq = ngo_phred(1 - minHomoPosterior);
        out->acn[major] = haplotypes;
    } else {
        helper = &hs[maxFreqIdx];
        /* CountsHelper.getPosteriorProbabilities(hetRate, majorAlleleIdx) (CountsHelper.java:451-467) */
        double ev[4];
        double lph = log10(h / (n - 1)), lpo = log10(1 - h);
        for (int j = 0; j < n; j++) ev[j] = helper->logc[major][j] + (j == major ? lpo : lph);
        calc_posteriors(ev, n);
        out->gq = ngo_phred(1 - ev[maxAlt]);
        int altCN = (int)(int16_t)ngo_java_round(maxFreq * haplotypes);
        if (altCN == 0) altCN++;
        else if (altCN == haplotypes) altCN--;
        out->acn[maxAlt] = altCN;
        out->acn[major] = haplotypes - altCN;
    }
    out->total_cn = haplotypes;                          /* setAllelesCopyNumber */
    out->report = 1;
    for (int i = 0; i < n; i++) {
        out->counts[i] = counts[i];
        for (int j = 0; j < n; j++) out->logc[i][j] = helper->logc[i][j];
    }
    free(freqs); free(hs);
}

static void pool_to_call(const ngo_pcall* pc, const int* dna, int n, ngo_call* out) {
    out->pool = 1;
    out->pool_n = n;
    for (int i = 0; i < 4; i++) out->pool_dna[i] = i < n ? dna[i] : -1;
    out->pool_ncalled = pc->n_called;
    out->pool_called[0] = pc->called[0]; out->pool_called[1] = pc->called[1];
    out->pool_report = pc->report;
    for (int i = 0; i < 4; i++) { out->pool_counts[i] = pc->counts[i]; out->pool_acn[i] = pc->acn[i]; }
    out->pool_total_cn = pc->total_cn;
    out->gq = pc->gq; out->dp = pc->dp;
    for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) out->logc[i][j] = pc->logc[i][j];
}

/* discoverSNV with ploidy >= 3 (SingleSampleVariantPileupListener.java:238-254) and the discoverVariant
 * filters (:221-227: undecided / hom-ref / GQ below -minQuality dropped, ACN from the counts); 1 = kept */
static int pool_discover(const ngo_counts* h4, const ngo_acalls* calls, int pos, char refBase, const ngo_params* p,
                         double hetRate, ngo_call* out) {
    /* createSNVVariantPool(pileup, helperSNV, reference, 0.5/ploidy) (:297-332) */
    if (h4->total_count == 0) return 0;
    int refIdx = base_idx(refBase);
    if (refIdx < 0) return 0;
    int sum = h4->counts[0] + h4->counts[1] + h4->counts[2] + h4->counts[3];
    double minCount = (0.5 / (double)p->ploidy) * sum;
    if (minCount < 1) minCount = 1;
    int dna[4], n = 0;
    dna[n++] = refIdx;
    for (int i = 0; i < 4; i++) if (h4->counts[i] >= minCount && i != refIdx) dna[n++] = i;
    if (n < 2) return 0;
    int multi = n > 2;
    ngo_pcall pc;
    genotype_pool(dna, n, p->ploidy, calls, hetRate, p->max_base_qs, &pc);
    if (multi) {
        if (pc.n_called == 0 || (pc.n_called == 1 && pc.called[0] == 0)) return 0;
        if (!(pc.n_called == 2 && pc.called[0] != 0)) {
            /* makeNewVariant(variant, {ref} + called alleles) (:346-359): a biallelic SNV */
            int nd[4], nn = 0;
            nd[nn++] = refIdx;
            for (int i = 0; i < pc.n_called; i++) if (dna[pc.called[i]] != refIdx) nd[nn++] = dna[pc.called[i]];
            for (int i = 0; i < nn; i++) dna[i] = nd[i];
            n = nn;
            multi = 0;
            genotype_pool(dna, n, p->ploidy, calls, hetRate, p->max_base_qs, &pc);
        }
    }
    if (pc.n_called == 0 || (pc.n_called == 1 && pc.called[0] == 0) || (int16_t)p->min_quality > pc.gq) return 0;
    pool_update_cn(&pc, p->ploidy);                      /* discoverVariant / intersectVariantsCNVs */
    memset(out, 0, sizeof(*out));
    out->pos = pos; out->ref = refBase; out->strand_bias = -1; out->ploidy = p->ploidy;
    out->qual = 0;                                       /* the variant's QS is never set on this path */
    memcpy(out->counts, h4->counts, sizeof(out->counts));
    pool_to_call(&pc, dna, n, out);
    out->pool_multi = multi;
    out->n_alleles = n;
    return 1;
}

/* -knownVariants with ploidy >= 3: genotypeVariantSample (:361-391) -> genotypeVariantPool, setAllCounts,
 * makeUndecided below -minQuality */
static void pool_known(const ngo_counts* h4, const ngo_acalls* calls, const ngo_known* kv, const ngo_params* p,
                       double hetRate, ngo_call* out) {
    int dna[2] = {base_idx(kv->ref), base_idx(kv->alt)};
    ngo_pcall pc;
    genotype_pool(dna, 2, p->ploidy, calls, hetRate, p->max_base_qs, &pc);
    /* makeUndecided below -minQuality; otherwise the ACN genotypeVariantPool set stays (intersectVariantsCNVs recomputes
     * it from the counts for the first record of the sequence only: on_sequence_end) */
    if ((int16_t)p->min_quality > pc.gq) { pc.n_called = 0; pc.gq = 0; pool_update_cn(&pc, pc.total_cn); }
    memset(out, 0, sizeof(*out));
    out->pos = kv->pos; out->ref = kv->ref; out->known = 1; out->id = kv->id; out->qual = kv->qs; out->known_type = kv->type;
    out->strand_bias = -1; out->ploidy = p->ploidy;
    memcpy(out->counts, h4->counts, sizeof(out->counts));
    pool_to_call(&pc, dna, 2, out);
    out->n_alleles = 2;
}

/* One sample's call: CalledSNV (biallelic SNV) or CalledGenomicVariantImpl (multi-allelic SNV or
 * the no-data undecided call), as far as the VCF line and DiversityStatistics read them. */
typedef struct {
    int kind;                 /* 0 CalledSNV, 1 CalledGenomicVariantImpl */
    int n_called, called[2];  /* indexes into the variant alleles (CalledSNV: 0 ref, 1 alt) */
    int gq, dp;
    int counts[4];            /* getAllCounts: A,C,G,T */
    int has_logs;             /* report log-conditionals present */
    double logs[4][4];        /* over the variant alleles (CalledSNV: float values) */
    int total_cn;             /* getCopyNumber */
    int acn[4];               /* getAllelesCopyNumber over the variant alleles */
} ngo_scall;

/* GenomicVariant as the MVD path builds it: reference first, then alternatives in A,C,G,T order */
typedef struct { int n; int idx[4]; int multisnv_type; int known_type; } ngo_pvar;   /* known_type: an input record's TYPE */

/* CalledSNV.updateAllelesCopyNumberFromCounts (variants/CalledSNV.java:134-158); genotype -1..2 */
static void csnv_update_cn(int genotype, const int* counts, const ngo_pvar* v, int total, int* tot_out, int* ref_out) {
    int ref = 0;
    if (genotype == -1) { *tot_out = total; *ref_out = 0; return; }
    if (genotype == 0) ref = total;
    else if (genotype == 2) ref = 0;
    else if (total <= 2) { total = 2; ref = 1; }
    else {
        double cr = counts[v->idx[0]], sum = cr + counts[v->idx[1]];
        double prop = sum > 0 ? cr / sum : 0.5;
        if (prop > 1) prop = 1;
        ref = (int16_t)ngo_java_round(prop * total);
        if (ref == 0) ref = 1;
        else if (ref >= total) ref = total - 1;
    }
    *tot_out = total; *ref_out = ref;
}

/* CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts (variants/CalledGenomicVariantImpl.java:228-282) */
static void cgv_update_cn(ngo_scall* c, int n_alleles, int total, const int* report_counts /* NULL: absent */) {
    c->total_cn = total;
    for (int i = 0; i < 4; i++) c->acn[i] = 0;
    if (c->n_called == 0) return;
    if (c->n_called == 1 && c->called[0] == 0) { c->acn[0] = total; return; }
    int nc = c->n_called;
    if (total <= nc) { for (int i = 0; i < nc; i++) c->acn[c->called[i]] = 1; return; }
    if (!report_counts) {
        int def = total / nc;
        for (int i = 0; i < nc; i++) c->acn[c->called[i]] = def;
        c->acn[c->called[0]] += total - def * nc;
        return;
    }
    int rc[2], tr = 0;
    for (int i = 0; i < nc; i++) { rc[i] = report_counts[c->called[i]]; if (rc[i] == 0) rc[i] = 1; tr += rc[i]; }
    int tc = 0;
    for (int i = 0; i < nc; i++) {
        int64_t r = ngo_java_round((double)total * rc[i] / tr);
        c->acn[c->called[i]] = (int)(r > 1 ? r : 1);
        tc += c->acn[c->called[i]];
    }
    if (tc < total) c->acn[c->called[0]] += total - tc;
    else {
        int ex = tc - total;
        for (int i = nc - 1; ex > 0 && i >= 0; i--) {
            int j = c->called[i];
            int rm = ex < c->acn[j] - 1 ? ex : c->acn[j] - 1;
            c->acn[j] -= rm; ex -= rm;
        }
    }
    (void)n_alleles;
}

/* SingleSampleVariantPileupListener.genotypeVariantSample (:361-391) with a fresh listener
 * (minQuality = DEF_MIN_QUALITY 40) and VariantDiscoverySNVQAlgorithm.genotypeSNV (:21-97) */
static void genotype_sample(const ngo_counts* h, const ngo_acalls* calls, const ngo_pvar* v, double het, int ploidy,
                            ngo_scall* c) {
    memset(c, 0, sizeof(*c));
    memcpy(c->counts, h->counts, sizeof(c->counts));
    if (ploidy >= 3) {
        /* genotypeVariantPool + setAllCounts (:368-371), makeUndecided below the fresh listener's minQuality */
        ngo_pcall pc;
        genotype_pool(v->idx, v->n, ploidy, calls, het, h->max_base_qs, &pc);
        c->kind = 1;
        c->n_called = pc.n_called; c->called[0] = pc.called[0]; c->called[1] = pc.called[1];
        c->gq = pc.gq; c->dp = pc.dp;
        c->has_logs = pc.report;
        for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) c->logs[i][j] = pc.logc[i][j];
        if (40 > pc.gq) { pc.n_called = 0; pc.gq = 0; pool_update_cn(&pc, pc.total_cn); c->n_called = 0; c->gq = 0; }
        c->total_cn = pc.total_cn;
        for (int i = 0; i < 4; i++) c->acn[i] = pc.acn[i];
        return;
    }
    if (h->total_count == 0) {
        /* undecided CalledGenomicVariantImpl(variant, new byte[0]) with the counts, no report */
        c->kind = 1;
        cgv_update_cn(c, v->n, ploidy, NULL);
        return;
    }
    double post[16];
    ngo_counts_posteriors(h, het, post);
    c->dp = h->total_count;
    if (v->n == 2) {
        int r = v->idx[0], a = v->idx[1];
        double pHomoRef = post[r * 4 + r], pMax = pHomoRef;
        int genotype = 0;
        double pHomoAlt = post[a * 4 + a];
        if (pHomoAlt > pMax + 0.01) { pMax = pHomoAlt; genotype = 2; }
        double pHetero = post[r * 4 + a] + post[a * 4 + r];
        if (pHetero > pMax + 0.01) { pMax = pHetero; genotype = 1; }
        int gq = ngo_phred(1 - pMax);
        if (gq == 0) genotype = -1;
        c->kind = 0;
        c->gq = gq;
        float hr = (float)h->logc[r][r], ha = (float)h->logc[a][a], ra = (float)h->logc[r][a], ar = (float)h->logc[a][r];
        c->has_logs = (hr + ra + ar + ha) != 0;      /* float sum, CalledSNV.java:422 */
        c->logs[0][0] = hr; c->logs[0][1] = ra; c->logs[1][0] = ar; c->logs[1][1] = ha;
        /* constructor: setGenotype with copy number 0, then updateAllelesCopyNumberFromCounts(ploidy) */
        int tot = 0, ref = 0;
        if (genotype != -1) csnv_update_cn(genotype, h->counts, v, 0, &tot, &ref);
        csnv_update_cn(genotype, h->counts, v, ploidy, &tot, &ref);
        if (40 > gq) { genotype = -1; c->gq = 0; ref = 0; }          /* makeUndecided, CalledSNV.java:279-285 */
        c->total_cn = tot;
        if (genotype == -1) c->n_called = 0;
        else if (genotype == 0) { c->n_called = 1; c->called[0] = 0; }
        else if (genotype == 2) { c->n_called = 1; c->called[0] = 1; }
        else { c->n_called = 2; c->called[0] = 0; c->called[1] = 1; }
        c->acn[0] = genotype == -1 ? 0 : ref;
        c->acn[1] = genotype == -1 ? 0 : tot - ref;
        return;
    }
    /* multi-allelic: report submatrices over the variant alleles (:59-96) */
    int n = v->n;
    int rcounts[4] = {0, 0, 0, 0};
    double rpost[4][4] = {{0}};
    for (int i = 0; i < n; i++) {
        rcounts[i] = h->counts[v->idx[i]];
        for (int j = 0; j < n; j++) { c->logs[i][j] = h->logc[v->idx[i]][v->idx[j]]; rpost[i][j] = post[v->idx[i] * 4 + v->idx[j]]; }
    }
    c->has_logs = 1;
    int bi = 0, bj = 0;                                   /* getIndexesMaxGenotype(report, 0), :223-243 */
    double probMax = rpost[0][0];
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            double gp = rpost[i][j];
            if (i != j) gp += rpost[j][i];
            if (gp > probMax + 0.01) { probMax = gp; bi = i; bj = j; }
        }
    double maxP = rpost[bi][bj];
    if (bi != bj) { maxP += rpost[bj][bi]; c->n_called = 2; c->called[0] = bi; c->called[1] = bj; }
    else { c->n_called = 1; c->called[0] = bi; }
    c->gq = ngo_phred(1 - maxP);
    c->kind = 1;
    cgv_update_cn(c, n, ploidy, rcounts);                 /* genotypeVariantSample: updateAllelesCopyNumberFromCounts(ploidy) */
    if (40 > c->gq) { c->n_called = 0; c->gq = 0; cgv_update_cn(c, n, c->total_cn, rcounts); }   /* makeUndecided, :320-325 */
}

typedef struct ngo_mvd {
    int n_samples;
    char** ids;                   /* sorted sample ids (TreeMap order, MultisampleVariantsDetector.java:499-523) */
    int* rg_sample;               /* read group -> sample (-1: none) */
    int* rg_rank;                 /* rank of the read group in its sample's HashSet order */
    int* n_rank;                  /* read groups per sample */
    double min_adf;
    int ploidy;
    ngo_counts* h;                /* per-sample helpers */
    ngo_acalls* sc;               /* ploidy >= 3: per-sample allele calls in getAlleleCalls order */
    ngo_scall* calls;
} ngo_mvd;

/* DecimalFormat("##0.0#") (main/io/ParseUtils.java:29), HALF_EVEN on the exact binary value */
int ngo_java_fmt2(double x, char* buf, int cap) {
    double p = x * 100.0, err = fma(x, 100.0, -p);
    double k = floor(p), fr = p - k;
    long long n = (long long)k;
    if (fr > 0.5 || (fr == 0.5 && (err > 0 || (err == 0 && (n & 1))))) n++;
    if (n % 10 == 0) return snprintf(buf, cap, "%lld.%lld", n / 100, (n % 100) / 10);
    return snprintf(buf, cap, "%lld.%02lld", n / 100, n % 100);
}

/* VCFRecord.updateDiversityStatistics (vcf/VCFRecord.java:288-301) with
 * DiversityStatistics.calculateDiversityStatistics(calls, false) (variants/DiversityStatistics.java:123-218):
 * "NS=..;AN=..;AFS=..;OH=..[;MAF=..]" for calls given as (n_called, called[2], acn[4]) */
int ngo_population_info(int n_calls, const int* n_called, const int* called, const int* acn, int n_alleles,
                        char* buf, int cap) {
    int counts[4] = {0, 0, 0, 0}, sum = 0, ng = 0, nhet = 0;
    for (int s = 0; s < n_calls; s++) {
        if (n_called[s] == 0) continue;
        ng++;
        if (n_called[s] > 1) nhet++;
        for (int i = 0; i < n_called[s]; i++) { int j = called[2 * s + i]; counts[j] += acn[4 * s + j]; sum += acn[4 * s + j]; }
    }
    int ncalled = 0, minAC = 0;
    for (int i = 0; i < n_alleles; i++)
        if (counts[i] > 0) { ncalled++; if (minAC == 0 || minAC > counts[i]) minAC = counts[i]; }
    int k = snprintf(buf, cap, "NS=%d;AN=%d;AFS=", ng, ncalled);
    for (int i = 0; i < n_alleles; i++) k += snprintf(buf + k, cap - k, "%s%d", i ? "," : "", counts[i]);
    k += snprintf(buf + k, cap - k, ";OH=");
    k += ngo_java_fmt2(ng > 0 ? (double)nhet / ng : 0.0, buf + k, cap - k);
    if (n_alleles == 2) {
        k += snprintf(buf + k, cap - k, ";MAF=");
        k += ngo_java_fmt2(ncalled < 2 ? 0.0 : (double)minAC / sum, buf + k, cap - k);
    }
    return k;
}

static void mvd_genotype_all(ngo_mvd* M, const ngo_pvar* v, double het, int* qs) {
    int q = 0;
    for (int s = 0; s < M->n_samples; s++) {
        genotype_sample(&M->h[s], &M->sc[s], v, het, M->ploidy, &M->calls[s]);
        const ngo_scall* c = &M->calls[s];
        int homref = c->n_called == 1 && c->called[0] == 0;
        if (c->n_called > 0 && !homref && c->gq > q) q = c->gq;   /* MultisampleVariantsDetector.java:683-685 */
    }
    *qs = q;
}

static void mvd_print(FILE* out, const char* seqName, int pos, const char* id, const ngo_pvar* v, int qs, const ngo_mvd* M) {
    fprintf(out, "%s\t%d\t%s\t%c\t", seqName, pos, id ? id : ".", BASES[v->idx[0]]);
    for (int i = 1; i < v->n; i++) fprintf(out, "%s%c", i > 1 ? "," : "", BASES[v->idx[i]]);
    fprintf(out, "\t%d\t.\t", qs);
    {
        int S = M->n_samples;
        int* nc = malloc(sizeof(int) * (S ? S : 1));
        int* cl = malloc(sizeof(int) * 2 * (S ? S : 1));
        int* acn = malloc(sizeof(int) * 4 * (S ? S : 1));
        for (int s = 0; s < S; s++) {
            nc[s] = M->calls[s].n_called;
            cl[2 * s] = M->calls[s].called[0]; cl[2 * s + 1] = M->calls[s].called[1];
            for (int j = 0; j < 4; j++) acn[4 * s + j] = M->calls[s].acn[j];
        }
        char info[256];
        ngo_population_info(S, nc, cl, acn, v->n, info, sizeof info);
        fputs(info, out);
        free(nc); free(cl); free(acn);
    }
    if (v->multisnv_type == 2) fprintf(out, ";TYPE=EMBEDDED");   /* TYPE_EMBEDDED_SNV (MultisampleVariantsDetector.java:581) */
    else if (v->multisnv_type) fprintf(out, ";TYPE=MULTISNV");   /* VCFFileWriter.java:47-49 */
    else if (type_name(v->known_type)) fprintf(out, ";TYPE=%s", type_name(v->known_type));
    fprintf(out, "\tGT:PL:GQ:DP:BSDP:ACN");
    for (int s = 0; s < M->n_samples; s++) {
        const ngo_scall* c = &M->calls[s];
        fprintf(out, "\t");
        /* VCFFileWriter.printGenotypeInfo (:159-308) */
        if (c->n_called == 0) fprintf(out, M->ploidy > 1 ? "./." : ".");
        else if (c->n_called == 1) { fprintf(out, "%d", c->called[0]); if (M->ploidy > 1) fprintf(out, "/%d", c->called[0]); }
        else fprintf(out, "%d/%d", c->called[0], c->called[1]);
        fprintf(out, ":");
        for (int j = 0; j < v->n; j++)
            for (int i = 0; i <= j; i++) {
                if (i > 0 || j > 0) fprintf(out, ",");
                fprintf(out, "%d", c->has_logs ? (int)ngo_java_round(-10 * c->logs[i][j]) : 0);
            }
        fprintf(out, ":%d:%d:%d,%d,%d,%d:", c->gq, c->dp, c->counts[0], c->counts[1], c->counts[2], c->counts[3]);
        if (c->total_cn == 0) fprintf(out, ".");
        else {
            int nal = c->kind == 0 ? 2 : v->n;
            for (int j = 0; j < nal; j++) {
                int val = c->acn[j];
                if (c->n_called == 0 && j == 0) val = c->total_cn;
                fprintf(out, "%s%d", j ? "," : "", val);
            }
        }
    }
    fprintf(out, "\n");
}

/* the position's per-sample span-1 counts (getAlleleCalls(1, sample.getReadGroups()): the sample's read groups in
 * HashSet order, pending order inside each, PileupRecord.getAlleleCalls :104-152) and the pooled counts of every
 * alignment (getAlleleCalls(1, null)); `alns` is the pileup (its membership fixed before the realigner's edits:
 * aligned_read_pos drops an alignment an edit moved off the position) */
static void mvd_snv_counts(ngo_gen* G, int pos, ngo_aln** alns, int n, ngo_counts* pooled) {
    ngo_mvd* M = G->mvd;
    const ngo_params* p = G->p;
    ngo_counts_init(pooled, 4, 0.5, p->max_base_qs);
    for (int s = 0; s < M->n_samples; s++) { ngo_counts_init(&M->h[s], 4, 0.5, p->max_base_qs); M->sc[s].n = 0; }
    int maxrank = 0;
    for (int s = 0; s < M->n_samples; s++) if (M->n_rank[s] > maxrank) maxrank = M->n_rank[s];
    for (int rank = -1; rank < maxrank; rank++) {
        for (int k = 0; k < n; k++) {
            ngo_aln* a = alns[k];
            if (a->first > pos || a->last < pos) continue;
            int sm = a->rg >= 0 ? M->rg_sample[a->rg] : -1;
            if (rank >= 0 && (sm < 0 || M->rg_rank[a->rg] != rank)) continue;
            if (!a->chars) continue;
            int rp = aligned_read_pos(a, pos);
            if (rp < 0) continue;
            int len = a->acl[rp];
            if (len != 1) continue;
            int qc = a->quals ? a->quals[rp] : '+';
            int q = qc - 33; if (q > 30) q = 30;
            ngo_counts* h = rank < 0 ? pooled : &M->h[sm];
            ngo_counts_update(h, base_idx(a->chars[rp]), (int8_t)q, (a->flags & FLAG_REVERSE) != 0);
            if (rank >= 0 && M->ploidy >= 3) acalls_push(&M->sc[sm], base_idx(a->chars[rp]), (int8_t)q, (a->flags & FLAG_REVERSE) != 0);
        }
    }
}

/* discoverPopulationSNV (:585-597): createSNVVariantPool (SingleSampleVariantPileupListener.java:297-332) over the
 * pooled counts, then the multi-allelic loop (makeNewVariant :642-656); 1 with the variant in *v */
static int mvd_snv_variant(ngo_gen* G, char R, const ngo_counts* pooled, ngo_pvar* out) {
    ngo_mvd* M = G->mvd;
    if (pooled->total_count == 0) return 0;
    int refIdx = base_idx(R);
    if (refIdx < 0) return 0;
    int sum = pooled->counts[0] + pooled->counts[1] + pooled->counts[2] + pooled->counts[3];
    double minCount = M->min_adf * sum;
    if (minCount < 1) minCount = 1;
    ngo_pvar v = {0, {0}, 0, 0};
    v.idx[v.n++] = refIdx;
    for (int i = 0; i < 4; i++)
        if (pooled->counts[i] >= minCount && i != refIdx) v.idx[v.n++] = i;
    if (v.n < 2) return 0;
    v.multisnv_type = v.n > 2;
    int qs = 0;
    while (v.n > 2) {
        mvd_genotype_all(M, &v, G->het_rate, &qs);
        /* makeNewVariant (MultisampleVariantsDetector.java:642-656, SingleSampleVariantPileupListener.java:346-359) */
        int called[4] = {0, 0, 0, 0};
        called[v.idx[0]] = 1;
        for (int s = 0; s < M->n_samples; s++)
            for (int i = 0; i < M->calls[s].n_called; i++) called[v.idx[M->calls[s].called[i]]] = 1;
        int nset = called[0] + called[1] + called[2] + called[3];
        if (nset == v.n) break;
        ngo_pvar nv = {0, {0}, 0, 0};
        nv.idx[nv.n++] = v.idx[0];
        for (int i = 0; i < 4; i++) if (called[i] && i != v.idx[0]) nv.idx[nv.n++] = i;
        v = nv;   /* SNV (BIALLELIC type) or GenomicVariantImpl (UNDETERMINED type): no TYPE annotation */
    }
    if (v.n < 2) return 0;   /* only the reference allele is left: not an SNV, no decided non-reference call */
    *out = v;
    return 1;
}

static void mvd_on_pileup_known(ngo_gen* G, int pos);
/* MultisampleVariantsDetector.onPileup (:522-558) without the indel realigner (indel pass-through) */
static void mvd_on_pileup(ngo_gen* G, int pos) {
    ngo_mvd* M = G->mvd;
    const ngo_params* p = G->p;
    const ngo_seq* sq = &G->g->s[G->cur_seq];
    if (pos < 1 || pos > sq->len) return;
    char r = sq->seq[pos - 1];
    if (!G->known) {
        /* calculateReferenceAlleleDiscovery (SingleSampleVariantPileupListener.java:191-206) */
        if (p->ignore_lowercase_ref && islower((unsigned char)r)) return;
    }
    if (G->known) { mvd_on_pileup_known(G, pos); return; }
    char R = (char)toupper((unsigned char)r);
    ngo_counts pooled;
    mvd_snv_counts(G, pos, G->pending.a, G->pending.n, &pooled);
    ngo_pvar v;
    if (!mvd_snv_variant(G, R, &pooled, &v)) return;
    int qs = 0;
    mvd_genotype_all(M, &v, G->het_rate, &qs);
    if (qs == 0 || qs < p->min_quality) return;           /* MultisampleVariantsDetector.java:534 */
    mvd_print(G->out, sq->name, pos, NULL, &v, qs, M);
    G->st->variants_called++;
}

#include "ngsep_oracle_indel.inc"

/* ---- realigner trace (test infrastructure: NGO_REALIGN_TRACE=path; tests/test_oracle_realigner_kat.py compares it with
 * the independent Python restatement tests/realigner_restatement.py).  Per pileup the realigner ran on:
 * "P pos span str newSTR embedded"; when the span is > 1 the pileup's getAlleleCalls(span, null) as "C allele quals";
 * per alignment leaving the pending list (or left at the end): "A id first last CIGAR ignoreStart ignoreEnd". */
static FILE* g_rtrace = NULL;
static void rtrace_pileup(ngo_aln** alns, int n, int pos, int span, int is_str, int is_new_str, int embedded) {
    if (!g_rtrace) return;
    fprintf(g_rtrace, "P\t%d\t%d\t%d\t%d\t%d\n", pos, span, is_str, is_new_str, embedded);
    if (span <= 1) return;
    ngo_icalls calls = {0};
    pileup_calls(alns, n, pos, span, &calls);
    for (int i = 0; i < calls.n; i++) fprintf(g_rtrace, "C\t%s\t%s\n", calls.c[i].allele, calls.c[i].qual);
    icalls_free(&calls);
}
static void rtrace_aln(const ngo_aln* a) {
    if (!g_rtrace) return;
    static const char kOps[] = "HDIMPNSX";
    fprintf(g_rtrace, "A\t%d\t%d\t%d\t", a->id, a->first, a->last);
    for (int i = 0; i < a->n_ops; i++) fprintf(g_rtrace, "%d%c", a->ops[i] / 8, kOps[a->ops[i] & 7]);
    fprintf(g_rtrace, "\t%d\t%d\n", a->ignore_start, a->ignore_end);
}
struct ngo_indel_call_s { ngo_indel_call c; int ploidy; };
static void free_indel_call(struct ngo_indel_call_s* c) { for (int i = 0; i < c->c.n; i++) free(c->c.alleles[i]); free(c); }
static void print_indel_call_any(FILE* out, const char* seqName, const ngo_call* c) { print_indel_call(out, seqName, &c->indel->c, c->indel->ploidy); }

/* ==== MultisampleVariantsDetector with IndelRealignerPileupListener first in the listener chain
 * (MultisampleVariantsDetector.java:449-450): onPileup's span rules (:522-538), the span branch
 * discoverPopulationVariantWithSpan / discoverPopulationIndel (:599-634) and every sample's indel genotype
 * (SingleSampleVariantPileupListener.genotypeVariantSample :361-391 -> VariantDiscoverySNVQAlgorithm.callIndel
 * :265-361 with the variant given) ==== */

/* one sample's call of an indel variant of n alleles (a CalledGenomicVariantImpl) */
typedef struct {
    int n_called, called[2], gq, dp, has_report, total_cn;
    int* counts;               /* n: the report's counts (CountsHelper.getCounts) */
    double* logc;              /* n x n: the report's log-conditionals */
    int* acn;                  /* n: allelesCopyNumber */
} ngo_iscall;

static void iscall_free(ngo_iscall* c) { free(c->counts); free(c->logc); free(c->acn); c->counts = NULL; c->logc = NULL; c->acn = NULL; }

/* CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts (variants/CalledGenomicVariantImpl.java:228-282) */
static void iscall_update_cn(ngo_iscall* c, int n, int total) {
    c->total_cn = total;
    for (int i = 0; i < n; i++) c->acn[i] = 0;
    if (c->n_called == 0) return;
    if (c->n_called == 1 && c->called[0] == 0) { c->acn[0] = total; return; }
    const int nc = c->n_called;
    if (total <= nc) { for (int i = 0; i < nc; i++) c->acn[c->called[i]] = 1; return; }
    if (!c->has_report) {
        const int def = total / nc;
        for (int i = 0; i < nc; i++) c->acn[c->called[i]] = def;
        c->acn[c->called[0]] += total - def * nc;
        return;
    }
    int rc[2], tr = 0;
    for (int i = 0; i < nc; i++) { rc[i] = c->counts[c->called[i]]; if (rc[i] == 0) rc[i] = 1; tr += rc[i]; }
    int tc = 0;
    for (int i = 0; i < nc; i++) {
        const int64_t r = ngo_java_round((double)total * rc[i] / tr);
        c->acn[c->called[i]] = (int)(r > 1 ? (int16_t)r : 1);
        tc += c->acn[c->called[i]];
    }
    if (tc < total) c->acn[c->called[0]] += total - tc;
    else {
        int ex = tc - total;
        for (int i = nc - 1; ex > 0 && i >= 0; i--) {
            const int j = c->called[i];
            const int rm = ex < c->acn[j] - 1 ? ex : c->acn[j] - 1;
            c->acn[j] -= rm;
            ex -= rm;
        }
    }
}

/* genotypeVariantPool (SingleSampleVariantPileupListener.java:402-503) over an indel variant: one CountsHelper
 * .calculateCountsIndel per heterozygosity hypothesis (freq = k / haplotypes < 0.51, :410-414), the major allele by
 * the first helper's counts (undecided with no report and no depth below `haplotypes` calls, :428-432), every other
 * allele's homozygous-vs-heterozygous posteriors (:447-470), GQ and setAllelesCopyNumber (:482-498), the report from
 * the chosen helper (:499-500) */
static void genotype_pool_indel(const ngo_sv* alleles, const ngo_icalls* calls, int haplotypes, double h, int max_base_qs,
                                ngo_iscall* out) {
    const int n = alleles->n;
    memset(out, 0, sizeof(*out));
    out->counts = calloc((size_t)n, sizeof(int));
    out->logc = calloc((size_t)n * n, sizeof(double));
    out->acn = calloc((size_t)n, sizeof(int));
    const double step = 1.0 / (double)haplotypes;
    int nf = 0;
    for (double freq = step; freq < 0.51; freq += step) nf++;
    double* freqs = malloc(sizeof(double) * (nf ? nf : 1));
    ngo_icounts* hs = malloc(sizeof(ngo_icounts) * (nf ? nf : 1));
    nf = 0;
    for (double freq = step; freq < 0.51; freq += step) {
        freqs[nf] = freq;
        icounts_run(&hs[nf], alleles, calls, max_base_qs, freq);
        nf++;
    }
    const ngo_icounts* helper = &hs[0];
    int major = 0;                                            /* NumberArrays.getIndexMaximum: first maximum */
    for (int i = 1; i < n; i++) if (helper->counts[major] < helper->counts[i]) major = i;
    if (helper->counts[major] < haplotypes) {
        iscall_update_cn(out, n, haplotypes);                 /* undecided.updateAllelesCopyNumberFromCounts */
    } else {
        const double logPriorHetero = log10(h), logPriorHomo = log10(1 - h);
        double* terms = malloc(sizeof(double) * (size_t)(nf + 1));
        const double termHomozygous = helper->logc[major * n + major] + logPriorHomo;
        double maxHetPosterior = 0, minHomoPosterior = 1, maxFreq = 0;
        int maxFreqIdx = 0, maxAlt = -1;
        for (int i = 0; i < n; i++) {
            if (i == major) continue;
            terms[0] = termHomozygous;
            for (int j = 0; j < nf; j++) terms[j + 1] = hs[j].logc[major * n + i] + logPriorHetero;
            calc_posteriors(terms, nf + 1);
            int idxMax = 0;
            for (int j = 1; j <= nf; j++) if (terms[idxMax] < terms[j]) idxMax = j;
            if (idxMax == 0) {
                if (terms[0] < minHomoPosterior) minHomoPosterior = terms[0];
            } else if (maxAlt == -1 || maxHetPosterior < terms[idxMax]) {
                maxHetPosterior = terms[idxMax];
                maxFreqIdx = idxMax - 1;
                maxFreq = freqs[maxFreqIdx];
                maxAlt = i;
            }
        }
        free(terms);
        if (maxAlt == -1) { out->n_called = 1; out->called[0] = major; }
        else { out->n_called = 2; out->called[0] = major < maxAlt ? major : maxAlt; out->called[1] = major < maxAlt ? maxAlt : major; }
        out->dp = helper->total_count;
        if (maxAlt == -1) {
            out->gq = ngo_phred(1 - minHomoPosterior);
            out->acn[major] = haplotypes;
        } else {
            helper = &hs[maxFreqIdx];
            /* CountsHelper.getPosteriorProbabilities(hetRate, majorAlleleIdx) (CountsHelper.java:451-467) */
            double* ev = malloc(sizeof(double) * (size_t)n);
            const double lph = log10(h / (n - 1)), lpo = log10(1 - h);
            for (int j = 0; j < n; j++) ev[j] = helper->logc[major * n + j] + (j == major ? lpo : lph);
            calc_posteriors(ev, n);
            out->gq = ngo_phred(1 - ev[maxAlt]);
            free(ev);
            int altCN = (int)(int16_t)ngo_java_round(maxFreq * haplotypes);
            if (altCN == 0) altCN++;
            else if (altCN == haplotypes) altCN--;
            out->acn[maxAlt] = altCN;
            out->acn[major] = haplotypes - altCN;
        }
        out->total_cn = haplotypes;                           /* setAllelesCopyNumber */
        out->has_report = 1;
        memcpy(out->counts, hs[0].counts, sizeof(int) * (size_t)n);
        memcpy(out->logc, helper->logc, sizeof(double) * (size_t)n * n);
    }
    for (int j = 0; j < nf; j++) { free(hs[j].counts); free(hs[j].logc); }
    free(freqs); free(hs);
}

/* genotypeVariantSample for an indel variant at ploidy < 3 (SingleSampleVariantPileupListener.java:377-390) with a
 * fresh listener (minQuality = DEF_MIN_QUALITY 40): calculateCountsIndel over the variant's alleles, callIndel with
 * the variant (indexes of the maximum genotype taken as they are, :335-345), updateAllelesCopyNumberFromCounts(ploidy),
 * makeUndecided below 40 (:320-325) */
static void genotype_indel_sample(const ngo_sv* alleles, const ngo_icalls* calls, double het, int ploidy, int max_base_qs,
                                  int min_quality, ngo_iscall* c) {
    const int n = alleles->n;
    if (ploidy >= 3) {
        /* ploidy >= DEF_MIN_PLOIDY_POOL_ALGORITHM: genotypeVariantPool (:378-379), then makeUndecided below min_quality */
        genotype_pool_indel(alleles, calls, ploidy, het, max_base_qs, c);
        if ((int16_t)min_quality > c->gq) { c->n_called = 0; c->gq = 0; iscall_update_cn(c, n, c->total_cn); }
        return;
    }
    memset(c, 0, sizeof(*c));
    c->counts = calloc((size_t)n, sizeof(int));
    c->logc = calloc((size_t)n * n, sizeof(double));
    c->acn = calloc((size_t)n, sizeof(int));
    ngo_icounts ih;
    icounts_run(&ih, alleles, calls, max_base_qs, 0.5);
    if (ih.total_count == 0) {
        /* new CalledGenomicVariantImpl(variant, new byte[0]) (:274-277), then the copy number of the ploidy */
        free(ih.counts); free(ih.logc);
        iscall_update_cn(c, n, ploidy);
        return;
    }
    const int heteroGenotypes = n * (n - 1);                  /* getPosteriorProbabilities (CountsHelper.java:410-443) */
    const double logPriorHetero = log10(het / heteroGenotypes), logPriorHomo = log10((1 - het) / n);
    double* ev = malloc(sizeof(double) * (size_t)n * n);
    double* post = calloc((size_t)n * n, sizeof(double));
    int k = 0;
    for (int i = 0; i < n; i++) {
        ev[k++] = ih.logc[i * n + i] + logPriorHomo;
        for (int j = 0; j < n; j++) if (i != j) ev[k++] = ih.logc[i * n + j] + logPriorHetero;
    }
    calc_posteriors(ev, n * n);
    k = 0;
    for (int i = 0; i < n; i++) {
        post[i * n + i] = ev[k++];
        for (int j = 0; j < n; j++) if (i != j) post[i * n + j] = ev[k++];
    }
    free(ev);
    int im0 = 0, im1 = 0;                                     /* getIndexesMaxGenotype(post, 0) (:223-243) */
    double probMax = post[0];
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            double gp = post[i * n + j];
            if (i != j) gp += post[j * n + i];
            if (gp > probMax + 0.01) { probMax = gp; im0 = i; im1 = j; }
        }
    if (im0 > 100 || im1 > 100) c->n_called = 0;              /* GenomicVariant.MAX_NUM_ALLELES */
    else if (im1 != im0) { c->n_called = 2; c->called[0] = im0; c->called[1] = im1; }
    else { c->n_called = 1; c->called[0] = im0; }
    double maxP = post[im0 * n + im1];
    if (im0 != im1) maxP += post[im1 * n + im0];
    free(post);
    c->gq = ngo_phred(1 - maxP);
    c->dp = ih.total_count;
    c->has_report = 1;                                        /* setCallReport when totalDepth > 0 */
    memcpy(c->counts, ih.counts, sizeof(int) * (size_t)n);
    memcpy(c->logc, ih.logc, sizeof(double) * (size_t)n * n);
    free(ih.counts); free(ih.logc);
    iscall_update_cn(c, n, ploidy);
    if ((int16_t)min_quality > c->gq) { c->n_called = 0; c->gq = 0; iscall_update_cn(c, n, c->total_cn); }
}

/* the sample's span calls, PileupRecord.getAlleleCalls(span, sample.getReadGroups()) (:104-111): read groups in
 * HashSet order, the pileup's order inside each */
static void sample_span_calls(ngo_gen* G, int s, int pos, int span, ngo_alist* tmp, ngo_icalls* out) {
    ngo_mvd* M = G->mvd;
    tmp->n = 0;
    for (int rank = 0; rank < M->n_rank[s]; rank++)
        for (int k = 0; k < G->pileup.n; k++) {
            ngo_aln* a = G->pileup.a[k];
            if (a->rg < 0 || M->rg_sample[a->rg] != s || M->rg_rank[a->rg] != rank) continue;
            alist_push(tmp, a);
        }
    pileup_calls(tmp->a, tmp->n, pos, span, out);
}

/* MultisampleVariantsDetector.genotypeVariant (:674-693) over an indel variant: every sample's call, the variant QS */
static int mvd_genotype_indel_all(ngo_gen* G, int pos, const ngo_sv* alleles, ngo_iscall* calls) {
    ngo_mvd* M = G->mvd;
    ngo_alist tmp = {0};
    ngo_icalls ic = {0};
    int qs = 0;
    const int span = (int)strlen(alleles->s[0]);
    for (int s = 0; s < M->n_samples; s++) {
        sample_span_calls(G, s, pos, span, &tmp, &ic);
        genotype_indel_sample(alleles, &ic, G->het_rate, M->ploidy, G->p->max_base_qs, 40, &calls[s]);
        for (int i = 0; i < ic.n; i++) { free(ic.c[i].allele); free(ic.c[i].qual); }
        ic.n = 0;
        const ngo_iscall* c = &calls[s];
        const int homref = c->n_called == 1 && c->called[0] == 0;
        if (c->n_called > 0 && !homref && c->gq > qs) qs = c->gq;
    }
    icalls_free(&ic);
    free(tmp.a);
    return qs;
}

static int same_lengths(const ngo_sv* v) {                 /* SingleSampleVariantPileupListener.allelesSameLength, :339-345 */
    for (int i = 1; i < v->n; i++) if (strlen(v->s[i]) != strlen(v->s[0])) return 0;
    return 1;
}

/* discoverPopulationVariantWithSpan (:599-604) + discoverPopulationIndel (:616-634): 1 with the variant's alleles
 * in *v (reference first), 0 for null */
static int mvd_discover_indel(ngo_gen* G, int pos, const char* ref, int input_str, ngo_sv* v) {
    ngo_mvd* M = G->mvd;
    const int lref = (int)strlen(ref);
    ngo_icalls calls = {0};
    pileup_calls(G->pileup.a, G->pileup.n, pos, lref, &calls);
    ngo_sv alleles = {0};
    cluster_allele_calls(&calls, ref, G->p->max_base_qs, &alleles);
    ngo_icounts ih;
    icounts_run(&ih, &alleles, &calls, G->p->max_base_qs, 0.5);
    /* createIndelVariantPool (SingleSampleVariantPileupListener.java:333-338) */
    const int ok = alleles.n > 1 && ih.total_count > 0;
    free(ih.counts); free(ih.logc);
    icalls_free(&calls);
    if (!ok) { sv_free(&alleles); return 0; }
    ngo_iscall* sc = calloc((size_t)(M->n_samples ? M->n_samples : 1), sizeof(ngo_iscall));
    while (alleles.n > 2) {
        if (!input_str && same_lengths(&alleles)) { sv_free(&alleles); free(sc); return 0; }
        const int qs = mvd_genotype_indel_all(G, pos, &alleles, sc);
        int drop = qs < G->p->min_quality;
        /* makeNewVariant (:642-656): a TreeSet of the reference and every sample's called alleles */
        ngo_sv set = {0};
        sv_push(&set, alleles.s[0], (int)strlen(alleles.s[0]));
        for (int s = 0; s < M->n_samples; s++)
            for (int i = 0; i < sc[s].n_called; i++) sv_push(&set, alleles.s[sc[s].called[i]], (int)strlen(alleles.s[sc[s].called[i]]));
        for (int s = 0; s < M->n_samples; s++) iscall_free(&sc[s]);
        if (drop) { sv_free(&set); sv_free(&alleles); free(sc); return 0; }
        sv_sort_unique(&set);
        if (set.n == alleles.n) { sv_free(&set); break; }
        ngo_sv nv = {0};                                       /* SingleSampleVariantPileupListener.makeNewVariant, :346-359 */
        sv_push(&nv, alleles.s[0], lref);
        for (int i = 0; i < set.n; i++) if (strcmp(set.s[i], alleles.s[0]) != 0) sv_push(&nv, set.s[i], (int)strlen(set.s[i]));
        sv_free(&set);
        sv_free(&alleles);
        alleles = nv;
    }
    free(sc);
    *v = alleles;
    return 1;
}

/* VCFRecord.createDefaultPopulationVCFRecord (vcf/VCFRecord.java:277-282, FORMAT DEF_FORMAT_ARRAY_NGSEP_NOSNV) +
 * VCFFileWriter.printVCFRecord / printGenotypeInfo (:44-68,159-256) for an indel / STR variant */
static void mvd_print_indel(ngo_gen* G, const char* seqName, int pos, const char* id, const ngo_sv* v, const char* type, int qs,
                            const ngo_iscall* calls) {
    ngo_mvd* M = G->mvd;
    FILE* out = G->out;
    const int n = v->n, S = M->n_samples;
    fprintf(out, "%s\t%d\t%s\t%s\t", seqName, pos, id ? id : ".", v->s[0]);
    if (n == 1) fprintf(out, ".");
    for (int i = 1; i < n; i++) fprintf(out, "%s%s", i > 1 ? "," : "", v->s[i]);
    fprintf(out, "\t%d\t.\t", qs);
    /* DiversityStatistics.calculateDiversityStatistics(calls, false) (variants/DiversityStatistics.java:123-218) */
    int* counts = calloc((size_t)n, sizeof(int));
    int sum = 0, ng = 0, nhet = 0;
    for (int s = 0; s < S; s++) {
        const ngo_iscall* c = &calls[s];
        if (c->n_called == 0) continue;
        ng++;
        if (c->n_called > 1) nhet++;
        for (int i = 0; i < c->n_called; i++) { counts[c->called[i]] += c->acn[c->called[i]]; sum += c->acn[c->called[i]]; }
    }
    int ncalled = 0, minAC = 0;
    for (int i = 0; i < n; i++) if (counts[i] > 0) { ncalled++; if (minAC == 0 || minAC > counts[i]) minAC = counts[i]; }
    char buf[64];
    fprintf(out, "NS=%d;AN=%d;AFS=", ng, ncalled);
    for (int i = 0; i < n; i++) fprintf(out, "%s%d", i ? "," : "", counts[i]);
    ngo_java_fmt2(ng > 0 ? (double)nhet / ng : 0.0, buf, sizeof buf);
    fprintf(out, ";OH=%s", buf);
    if (n == 2) { ngo_java_fmt2(ncalled < 2 ? 0.0 : (double)minAC / sum, buf, sizeof buf); fprintf(out, ";MAF=%s", buf); }
    free(counts);
    if (type) fprintf(out, ";TYPE=%s", type);
    fprintf(out, "\tGT:PL:GQ:DP:ADP:ACN");
    for (int s = 0; s < S; s++) {
        const ngo_iscall* c = &calls[s];
        fprintf(out, "\t");
        if (c->n_called == 0) fprintf(out, M->ploidy > 1 ? "./." : ".");
        else if (c->n_called == 1) { fprintf(out, "%d", c->called[0]); if (M->ploidy > 1) fprintf(out, "/%d", c->called[0]); }
        else fprintf(out, "%d/%d", c->called[0], c->called[1]);
        fprintf(out, ":");
        for (int j = 0; j < n; j++)
            for (int i = 0; i <= j; i++)
                fprintf(out, "%s%d", (i > 0 || j > 0) ? "," : "", c->has_report ? (int)ngo_java_round(-10 * c->logc[i * n + j]) : 0);
        fprintf(out, ":%d:%d:", c->gq, c->dp);
        for (int i = 0; i < n; i++) fprintf(out, "%s%d", i ? "," : "", c->has_report ? c->counts[i] : 0);
        fprintf(out, ":");
        if (c->total_cn == 0) fprintf(out, ".");
        else for (int j = 0; j < n; j++) fprintf(out, "%s%d", j ? "," : "", (c->n_called == 0 && j == 0) ? c->total_cn : c->acn[j]);
    }
    fprintf(out, "\n");
}

/* ==== test entry points (tests/test_oracle_indel_kat.py): the indel functions above on given inputs, checked there
 * against an independent pure-Python restatement of the Java (tests/indel_restatement.py) ==== */
static void t_calls(int m, const char* const* calls, const char* const* quals, ngo_icalls* out) {
    out->n = 0;
    for (int i = 0; i < m; i++) {
        if (out->n == out->cap) { out->cap = out->cap ? 2 * out->cap : 16; out->c = realloc(out->c, sizeof(ngo_icall) * out->cap); }
        ngo_icall* c = &out->c[out->n++];
        c->allele = strdup(calls[i]);
        c->qual = strdup(quals[i]);
        c->len = (int)strlen(calls[i]);
        c->neg = 0;
    }
}
static void t_alleles(int n, const char* const* alleles, ngo_sv* v) { for (int i = 0; i < n; i++) sv_push(v, alleles[i], (int)strlen(alleles[i])); }

/* CountsHelper.calculateCountsIndel: counts[n] and the n x n log-conditionals; returns totalCount */
int ngo_t_indel_counts(int n, const char* const* alleles, int m, const char* const* calls, const char* const* quals,
                       int max_base_qs, int* counts, double* logc) {
    ngo_sv al = {0};
    ngo_icalls ic = {0};
    t_alleles(n, alleles, &al);
    t_calls(m, calls, quals, &ic);
    ngo_icounts h;
    icounts_run(&h, &al, &ic, max_base_qs, 0.5);
    memcpy(counts, h.counts, sizeof(int) * (size_t)n);
    memcpy(logc, h.logc, sizeof(double) * (size_t)n * n);
    const int t = h.total_count;
    free(h.counts); free(h.logc);
    sv_free(&al); icalls_free(&ic);
    return t;
}

/* AlleleCallClustersBuilder.clusterAlleleCalls: the alleles joined by ',' (reference first); returns their number */
int ngo_t_cluster(const char* ref, int m, const char* const* calls, const char* const* quals, int max_base_qs, char* out, int cap) {
    ngo_icalls ic = {0};
    t_calls(m, calls, quals, &ic);
    ngo_sv al = {0};
    cluster_allele_calls(&ic, ref, max_base_qs, &al);
    int k = 0;
    out[0] = 0;
    for (int i = 0; i < al.n; i++) k += snprintf(out + k, (size_t)(cap > k ? cap - k : 0), "%s%s", i ? "," : "", al.s[i]);
    const int n = al.n;
    sv_free(&al); icalls_free(&ic);
    return n;
}

/* callIndel with variant == null + the single-sample listener's filters: the record's fields
 * "REF\tALT\tQS\tTYPE\tGT:PL:GQ:DP:ADP:ACN" in `out`; returns 1 when a call is kept */
int ngo_t_call_indel(int n, const char* const* alleles, int m, const char* const* calls, const char* const* quals,
                     int max_base_qs, double het, int is_str, int is_input_str, int min_quality, int ploidy, char* out, int cap) {
    ngo_sv al = {0};
    ngo_icalls ic = {0};
    t_alleles(n, alleles, &al);
    t_calls(m, calls, quals, &ic);
    ngo_icounts h;
    icounts_run(&h, &al, &ic, max_base_qs, 0.5);
    ngo_indel_call c;
    const int ok = call_indel(&h, &al, 1, is_str, is_input_str, het, min_quality, ploidy, &c);
    out[0] = 0;
    if (ok) {
        char* buf = NULL; size_t len = 0;
        FILE* f = open_memstream(&buf, &len);
        print_indel_call(f, "s", &c, ploidy);
        fclose(f);
        snprintf(out, (size_t)cap, "%s", buf);
        free(buf);
        for (int i = 0; i < c.n; i++) free(c.alleles[i]);
    }
    free(h.counts); free(h.logc);
    sv_free(&al); icalls_free(&ic);
    return ok;
}

/* genotypeVariantSample over an indel variant (the population path): "GT:PL:GQ:DP:ADP:ACN" of the call */
void ngo_t_genotype_indel_sample(int n, const char* const* alleles, int m, const char* const* calls, const char* const* quals,
                                 int max_base_qs, double het, int ploidy, char* out, int cap) {
    ngo_sv al = {0};
    ngo_icalls ic = {0};
    t_alleles(n, alleles, &al);
    t_calls(m, calls, quals, &ic);
    ngo_iscall c;
    genotype_indel_sample(&al, &ic, het, ploidy, max_base_qs, 40, &c);
    int k = 0;
    if (c.n_called == 0) k += snprintf(out + k, (size_t)(cap - k), ploidy > 1 ? "./." : ".");
    else if (c.n_called == 1) k += snprintf(out + k, (size_t)(cap - k), ploidy > 1 ? "%d/%d" : "%d", c.called[0], c.called[0]);
    else k += snprintf(out + k, (size_t)(cap - k), "%d/%d", c.called[0], c.called[1]);
    k += snprintf(out + k, (size_t)(cap - k), ":");
    for (int j = 0; j < n; j++)
        for (int i = 0; i <= j; i++)
            k += snprintf(out + k, (size_t)(cap - k), "%s%d", (i > 0 || j > 0) ? "," : "", c.has_report ? (int)ngo_java_round(-10 * c.logc[i * n + j]) : 0);
    k += snprintf(out + k, (size_t)(cap - k), ":%d:%d:", c.gq, c.dp);
    for (int i = 0; i < n; i++) k += snprintf(out + k, (size_t)(cap - k), "%s%d", i ? "," : "", c.has_report ? c.counts[i] : 0);
    k += snprintf(out + k, (size_t)(cap - k), ":");
    if (c.total_cn == 0) k += snprintf(out + k, (size_t)(cap - k), ".");
    else for (int j = 0; j < n; j++) k += snprintf(out + k, (size_t)(cap - k), "%s%d", j ? "," : "", (c.n_called == 0 && j == 0) ? c.total_cn : c.acn[j]);
    iscall_free(&c);
    sv_free(&al); icalls_free(&ic);
}

/* genotypeVariantSample over an indel variant at any ploidy (the pool algorithm from 3) with the given minQuality:
 * "GT:PL:GQ:DP:ADP:ACN" of the call */
void ngo_t_genotype_indel_sample_q(int n, const char* const* alleles, int m, const char* const* calls, const char* const* quals,
                                   int max_base_qs, double het, int ploidy, int min_quality, char* out, int cap) {
    ngo_sv al = {0};
    ngo_icalls ic = {0};
    t_alleles(n, alleles, &al);
    t_calls(m, calls, quals, &ic);
    ngo_iscall c;
    genotype_indel_sample(&al, &ic, het, ploidy, max_base_qs, min_quality, &c);
    int k = 0;
    if (c.n_called == 0) k += snprintf(out + k, (size_t)(cap - k), ploidy > 1 ? "./." : ".");
    else if (c.n_called == 1) k += snprintf(out + k, (size_t)(cap - k), ploidy > 1 ? "%d/%d" : "%d", c.called[0], c.called[0]);
    else k += snprintf(out + k, (size_t)(cap - k), "%d/%d", c.called[0], c.called[1]);
    k += snprintf(out + k, (size_t)(cap - k), ":");
    for (int j = 0; j < n; j++)
        for (int i = 0; i <= j; i++)
            k += snprintf(out + k, (size_t)(cap - k), "%s%d", (i > 0 || j > 0) ? "," : "", c.has_report ? (int)ngo_java_round(-10 * c.logc[i * n + j]) : 0);
    k += snprintf(out + k, (size_t)(cap - k), ":%d:%d:", c.gq, c.dp);
    for (int i = 0; i < n; i++) k += snprintf(out + k, (size_t)(cap - k), "%s%d", i ? "," : "", c.has_report ? c.counts[i] : 0);
    k += snprintf(out + k, (size_t)(cap - k), ":");
    if (c.total_cn == 0) k += snprintf(out + k, (size_t)(cap - k), ".");
    else for (int j = 0; j < n; j++) k += snprintf(out + k, (size_t)(cap - k), "%s%d", j ? "," : "", (c.n_called == 0 && j == 0) ? c.total_cn : c.acn[j]);
    iscall_free(&c);
    sv_free(&al); icalls_free(&ic);
}

/* ReadAlignment edits on an alignment given by its first position and CIGAR (NGSEP codes via parse_cigar):
 * op 0 moveIndelStart(a1, a2), 1 realignStart(a1, a2, a3, a4), 2 realignEnd(a1, a2, a3, a4).  The new CIGAR (the
 * alignment's codes written as SAM text, not collapsed), first and last go to out / *first / *last; returns
 * moveIndelStart's result (1 for the others) */
int ngo_t_edit(int op, const char* cigar, int first, int a1, int a2, int a3, int a4, char* out, int cap, int* first_out, int* last_out) {
    ngo_aln a;
    memset(&a, 0, sizeof a);
    if (parse_cigar(cigar, &a.ops, &a.n_ops) != 0) return -1;
    a.first = first;
    int span = 0;
    for (int i = 0; i < a.n_ops; i++) { if (a.ops[i] & 1) span += a.ops[i] / 8; if (a.ops[i] & 2) a.read_length += a.ops[i] / 8; }
    a.last = first + span - 1;
    update_allele_calls(&a);
    int r = 1;
    if (op == 0) r = aln_move_indel_start(&a, a1, a2);
    else if (op == 1) aln_realign_start(&a, a1, a2, a3, a4);
    else aln_realign_end(&a, a1, a2, a3, a4);
    static const char kOps[] = "HDIMPNSX";
    int k = 0;
    out[0] = 0;
    for (int i = 0; i < a.n_ops; i++) k += snprintf(out + k, (size_t)(cap > k ? cap - k : 0), "%d%c", a.ops[i] / 8, kOps[a.ops[i] & 7]);
    *first_out = a.first;
    *last_out = a.last;
    free(a.ops); free(a.acl); free(a.indel);
    return r;
}

/* MultisampleVariantsDetector.onPileup (:522-538) after the realigner set the pileup's span / STR / embedded flags */
static void mvd_on_pileup_realign(ngo_gen* G, int pos, int span, int is_str, int is_new_str, int r_embedded) {
    ngo_mvd* M = G->mvd;
    const ngo_params* p = G->p;
    const ngo_seq* sq = &G->g->s[G->cur_seq];
    const int input_str = is_str && !is_new_str;
    int embedded = r_embedded;
    if (input_str) G->last_indel_end = pos + span - 1;        /* (no ">= lastIndelEnd" test here, unlike the single-sample listener) */
    else if (pos <= G->last_indel_end) embedded = 1;
    /* calculateReferenceAlleleDiscovery (SingleSampleVariantPileupListener.java:191-206) */
    if (!p->call_embedded && embedded) return;
    const int last = pos + span - 1;
    if (pos < 1 || last > sq->len) return;
    if (p->ignore_lowercase_ref && islower((unsigned char)sq->seq[pos - 1])) return;
    const int lref = embedded ? 1 : span;
    if (embedded) { is_str = 0; }
    const char R = (char)toupper((unsigned char)sq->seq[pos - 1]);
    ngo_counts pooled;
    mvd_snv_counts(G, pos, G->pileup.a, G->pileup.n, &pooled);
    /* discoverPopulationVariant (:573-584) */
    if (lref > 1) {
        int lr = 0;
        char* ref = ref_upper(sq, pos, last, &lr);
        ngo_sv v = {0};
        const int got = mvd_discover_indel(G, pos, ref, input_str, &v);
        free(ref);
        if (got) {
            ngo_iscall* sc = calloc((size_t)(M->n_samples ? M->n_samples : 1), sizeof(ngo_iscall));
            const int qs = mvd_genotype_indel_all(G, pos, &v, sc);
            if (!(qs == 0 || qs < p->min_quality)) {
                mvd_print_indel(G, sq->name, pos, NULL, &v, is_str ? "STR" : "INDEL", qs, sc);
                G->st->variants_called++;
                G->last_indel_end = pos + (int)strlen(v.s[0]) - 1;   /* !variant.isSNV(): lastIndelEnd = variant.getLast() */
            }
            for (int s = 0; s < M->n_samples; s++) iscall_free(&sc[s]);
            free(sc);
            sv_free(&v);
            return;
        }
        if (input_str) return;                                   /* no SNV fallback for an input STR (:605) */
        /* (isNewSTR: setSTR(false), setNewSTR(false) -- the SNV fallback does not read them) */
    }
    ngo_pvar v;
    if (!mvd_snv_variant(G, R, &pooled, &v)) return;
    if (embedded) v.multisnv_type = 2;                         /* TYPE_EMBEDDED_SNV (:581) */
    int qs = 0;
    mvd_genotype_all(M, &v, G->het_rate, &qs);
    if (qs == 0 || qs < p->min_quality) return;
    mvd_print(G->out, sq->name, pos, NULL, &v, qs, M);
    G->st->variants_called++;
}

/* the position's alignments as PileupRecord.getAlignments (built by the realigner's step; here when it is off) */
static void ensure_pileup(ngo_gen* G, int pos) {
    if (G->realign) return;
    G->pileup.n = 0;
    for (int k = 0; k < G->pending.n; k++) {
        ngo_aln* a = G->pending.a[k];
        if (a->first <= pos && a->last >= pos) alist_push(&G->pileup, a);
    }
}
static void known_alleles(const ngo_known* kv, ngo_sv* v) {
    for (int i = 0; i < kv->n_alleles; i++) sv_push(v, kv->alleles[i], (int)strlen(kv->alleles[i]));
}

/* MultisampleVariantsDetector.onPileup with input variants (:539-551): every input variant at this position
 * (nextSIVIndex), genotypeVariant (:664-693) over its own alleles -- an SNV through the per-sample SNV counts, an
 * indel / MNP through every sample's getAlleleCalls(|REF|, readGroups) and callIndel with the variant (fresh
 * listener: minQuality 40) -- and the record always written (QUAL = the variant QS genotypeVariant sets, ID and
 * TYPE the input's) */
static void mvd_on_pileup_known(ngo_gen* G, int pos) {
    ngo_mvd* M = G->mvd;
    const ngo_seq* sq = &G->g->s[G->cur_seq];
    int counted = 0;
    ngo_counts pooled;
    while (G->known_next < G->n_known && G->known[G->known_next].seq == G->cur_seq && G->known[G->known_next].pos <= pos) {
        const ngo_known* kv = &G->known[G->known_next++];
        if (kv->pos != pos) continue;
        if (kv->snv) {
            if (!counted) {
                if (G->realign) mvd_snv_counts(G, pos, G->pileup.a, G->pileup.n, &pooled);
                else mvd_snv_counts(G, pos, G->pending.a, G->pending.n, &pooled);
                counted = 1;
            }
            ngo_pvar kvv = {0, {0}, 0, kv->type};
            kvv.idx[kvv.n++] = base_idx(kv->ref);
            kvv.idx[kvv.n++] = base_idx(kv->alt);
            int kqs = 0;
            mvd_genotype_all(M, &kvv, G->het_rate, &kqs);
            mvd_print(G->out, sq->name, pos, kv->id, &kvv, kqs, M);
        } else {
            ensure_pileup(G, pos);
            ngo_sv v = {0};
            known_alleles(kv, &v);
            ngo_iscall* sc = calloc((size_t)(M->n_samples ? M->n_samples : 1), sizeof(ngo_iscall));
            const int qs = mvd_genotype_indel_all(G, pos, &v, sc);
            mvd_print_indel(G, sq->name, pos, kv->id, &v, type_name(kv->type), qs, sc);
            for (int s = 0; s < M->n_samples; s++) iscall_free(&sc[s]);
            free(sc);
            sv_free(&v);
        }
        G->st->variants_called++;
    }
}

/* a genotyped -knownVariants indel / MNP of the single-sample listener, or an indel of the pool algorithm (ploidy >= 3)
 * -- a CalledGenomicVariantImpl over a GenomicVariantImpl, FORMAT DEF_FORMAT_ARRAY_NGSEP_NOSNV */
struct ngo_kindel {
    ngo_iscall c;
    int pos, n, qs, type, ploidy;
    char** alleles;            /* reference first */
    int own;                   /* alleles owned (a discovered variant) or the input record's */
    const char* id;
    int pool_known;            /* ploidy >= 3 input record: ACN from genotypeVariantPool unless first of its sequence */
};

/* SingleSampleVariantPileupListener.genotypeVariantSample (:361-391), non-SNV branch at ploidy < 3: getAlleleCalls(
 * |REF|, null), calculateCountsIndel over the variant's alleles, callIndel with the variant (VariantDiscoverySNVQ
 * Algorithm.java:265-361), updateAllelesCopyNumberFromCounts(ploidy), makeUndecided below -minQuality */
static void genotype_known_indel(ngo_gen* G, const ngo_known* kv, int pos, ngo_call* out) {
    const ngo_params* p = G->p;
    ensure_pileup(G, pos);
    ngo_sv v = {0};
    known_alleles(kv, &v);
    ngo_icalls calls = {0};
    pileup_calls(G->pileup.a, G->pileup.n, pos, (int)strlen(kv->alleles[0]), &calls);
    struct ngo_kindel* k = calloc(1, sizeof(*k));
    genotype_indel_sample(&v, &calls, G->het_rate, p->ploidy, p->max_base_qs, p->min_quality, &k->c);
    k->pos = kv->pos; k->n = kv->n_alleles; k->alleles = kv->alleles; k->own = 0;
    k->id = kv->id; k->qs = kv->qs; k->type = kv->type;
    k->ploidy = p->ploidy;
    k->pool_known = p->ploidy >= 3;
    icalls_free(&calls);
    sv_free(&v);
    memset(out, 0, sizeof(*out));
    out->pos = pos;
    out->known = 1;
    out->kindel = k;
}

/* VCFFileWriter.printVCFRecord of the call: the input's ID, alleles, QS and TYPE, FORMAT DEF_FORMAT_ARRAY_NGSEP_NOSNV */
static void print_kindel(FILE* out, const char* seqName, const struct ngo_kindel* k) {
    const ngo_iscall* c = &k->c;
    const int n = k->n;
    fprintf(out, "%s\t%d\t%s\t%s\t", seqName, k->pos, k->id ? k->id : ".", k->alleles[0]);
    for (int i = 1; i < n; i++) fprintf(out, "%s%s", i > 1 ? "," : "", k->alleles[i]);
    fprintf(out, "\t%d\t.\t", k->qs);
    if (type_name(k->type)) fprintf(out, "TYPE=%s", type_name(k->type));
    else fprintf(out, ".");
    fprintf(out, "\tGT:PL:GQ:DP:ADP:ACN\t");
    if (c->n_called == 0) fprintf(out, k->ploidy > 1 ? "./." : ".");
    else if (c->n_called == 1) { fprintf(out, "%d", c->called[0]); if (k->ploidy > 1) fprintf(out, "/%d", c->called[0]); }
    else fprintf(out, "%d/%d", c->called[0], c->called[1]);
    fprintf(out, ":");
    for (int j = 0; j < n; j++)
        for (int i = 0; i <= j; i++)
            fprintf(out, "%s%d", (i > 0 || j > 0) ? "," : "", c->has_report ? (int)ngo_java_round(-10 * c->logc[i * n + j]) : 0);
    fprintf(out, ":%d:%d:", c->gq, c->dp);
    for (int i = 0; i < n; i++) fprintf(out, "%s%d", i ? "," : "", c->has_report ? c->counts[i] : 0);
    fprintf(out, ":");
    if (c->total_cn == 0) fprintf(out, ".");
    else for (int j = 0; j < n; j++) fprintf(out, "%s%d", j ? "," : "", (c->n_called == 0 && j == 0) ? c->total_cn : c->acn[j]);
    fprintf(out, "\n");
}
static void free_kindel(struct ngo_kindel* k) {
    iscall_free(&k->c);
    if (k->own) { for (int i = 0; i < k->n; i++) free(k->alleles[i]); free(k->alleles); }
    free(k);
}

static void push_call(ngo_gen* G, const ngo_call* c);
static int same_lengths(const ngo_sv* v);
static void pool_known_first_cn(ngo_call* c, int ploidy) {
    if (c->kindel && c->kindel->pool_known) iscall_update_cn(&c->kindel->c, c->kindel->n, ploidy);
    if (c->pool && c->known) {
        ngo_pcall pc;
        memset(&pc, 0, sizeof(pc));
        pc.n_called = c->pool_ncalled; pc.called[0] = c->pool_called[0]; pc.called[1] = c->pool_called[1];
        pc.report = c->pool_report;
        for (int i = 0; i < 4; i++) pc.counts[i] = c->pool_counts[i];
        pool_update_cn(&pc, ploidy);
        for (int i = 0; i < 4; i++) c->pool_acn[i] = pc.acn[i];
        c->pool_total_cn = pc.total_cn;
    }
}
static void ngo_call_kindel(ngo_gen* G, int pos, const ngo_sv* alleles, ngo_iscall* c) {
    struct ngo_kindel* k = calloc(1, sizeof(*k));
    k->c = *c;
    k->pos = pos; k->n = alleles->n; k->own = 1;
    k->alleles = malloc(sizeof(char*) * (size_t)alleles->n);
    for (int i = 0; i < alleles->n; i++) k->alleles[i] = strdup(alleles->s[i]);
    k->ploidy = G->p->ploidy;
    ngo_call call;
    memset(&call, 0, sizeof(call));
    call.pos = pos;
    call.kindel = k;
    push_call(G, &call);
}

/* ploidy >= 3, a span > 1 (discoverVariantWithSpan :257-273 -> discoverIndel :275-296): the clustered alleles' pool
 * variant (createIndelVariantPool :333-338: none for one allele, no calls or alleles of one length), genotypeVariantPool;
 * a multi-allelic variant keeps its alleles when two non-reference alleles are called, else becomes the reference and
 * the called allele (makeNewVariant :346-359) and is genotyped again; an undecided, homozygous-reference or low-GQ
 * call is dropped (:263, :223); a kept call's ACN from its counts (:226) and lastIndelEnd = its last (:157-160).
 * The variant's type stays TYPE_UNDETERMINED (no INFO TYPE) and its QS 0.  1 when a call is kept. */
static int pool_discover_indel(ngo_gen* G, int pos, int last, int is_input_str) {
    const ngo_params* p = G->p;
    const ngo_seq* s = &G->g->s[G->cur_seq];
    int lr = 0;
    char* ref = ref_upper(s, pos, last, &lr);
    ngo_icalls calls = {0};
    pileup_calls(G->pileup.a, G->pileup.n, pos, lr, &calls);
    ngo_sv alleles = {0};
    cluster_allele_calls(&calls, ref, p->max_base_qs, &alleles);
    ngo_icounts ih;
    icounts_run(&ih, &alleles, &calls, p->max_base_qs, 0.5);
    const int total = ih.total_count;
    free(ih.counts); free(ih.logc);
    int kept = 0;
    (void)is_input_str;
    if (alleles.n > 1 && total > 0 && !same_lengths(&alleles)) {
        ngo_iscall c;
        genotype_pool_indel(&alleles, &calls, p->ploidy, G->het_rate, p->max_base_qs, &c);
        int ok = 1;
        if (alleles.n > 2) {
            const int homref = c.n_called == 1 && c.called[0] == 0;
            if (c.n_called == 0 || homref) ok = 0;
            else if (!(c.n_called == 2 && c.called[0] != 0)) {
                ngo_sv nv = {0};                               /* {reference} + the called alleles, in that order */
                sv_push(&nv, alleles.s[0], (int)strlen(alleles.s[0]));
                for (int i = 0; i < c.n_called; i++)
                    if (strcmp(alleles.s[c.called[i]], alleles.s[0]) != 0) sv_push(&nv, alleles.s[c.called[i]], (int)strlen(alleles.s[c.called[i]]));
                iscall_free(&c);
                if (same_lengths(&nv)) { ok = 0; sv_free(&nv); }
                else {
                    sv_free(&alleles);
                    alleles = nv;
                    genotype_pool_indel(&alleles, &calls, p->ploidy, G->het_rate, p->max_base_qs, &c);
                }
            }
        }
        if (ok) {
            const int homref = c.n_called == 1 && c.called[0] == 0;
            if (c.n_called == 0 || homref || (int16_t)p->min_quality > c.gq) ok = 0;
        }
        if (ok) {
            iscall_update_cn(&c, alleles.n, p->ploidy);         /* discoverVariant: updateAllelesCopyNumberFromCounts */
            ngo_call_kindel(G, pos, &alleles, &c);
            G->last_indel_end = pos + (int)strlen(alleles.s[0]) - 1;
            kept = 1;
        } else if (c.counts) {
            iscall_free(&c);
        }
    }
    sv_free(&alleles);
    icalls_free(&calls);
    free(ref);
    return kept;
}

static void push_call(ngo_gen* G, const ngo_call* c) {
    if (G->calls.n == G->calls.cap) { G->calls.cap = G->calls.cap ? 2 * G->calls.cap : 1024; G->calls.c = realloc(G->calls.c, sizeof(ngo_call) * G->calls.cap); }
    G->calls.c[G->calls.n++] = *c;
}

/* SingleSampleVariantPileupListener.onPileup (no input variants, :146-161) -> calculateReferenceAlleleDiscovery
 * (:191-206) -> discoverVariant (:213-232) with the pileup's reference span from the indel realigner: span 1 is
 * discoverSNV over `h`, a longer span discoverVariantWithSpan (:257-273) */
static void discover_with_span(ngo_gen* G, int pos, int span, int is_str, int is_new_str, int r_embedded, const ngo_counts* h) {
    const ngo_params* p = G->p;
    const ngo_seq* s = &G->g->s[G->cur_seq];
    const int is_input_str = is_str && !is_new_str;
    int embedded = r_embedded;                                   /* inside an input STR (the realigner's flag) */
    if (is_input_str && pos >= G->last_indel_end) G->last_indel_end = pos + span - 1;
    else if (pos <= G->last_indel_end) embedded = 1;
    if (!p->call_embedded && embedded) return;
    const int last = pos + span - 1;
    if (pos < 1 || last > s->len) return;                       /* getReference -> null */
    if (p->ignore_lowercase_ref && islower((unsigned char)s->seq[pos - 1])) return;
    int eff = embedded ? 1 : span;
    ngo_call c;
    const int pool = p->ploidy >= 3;
    if (eff > 1 && pool) {
        if (pool_discover_indel(G, pos, last, is_input_str)) return;
        if (is_input_str) return;
    } else if (eff > 1) {
        int lr = 0;
        char* ref = ref_upper(s, pos, last, &lr);
        ngo_icalls calls = {0};
        pileup_calls(G->pileup.a, G->pileup.n, pos, eff, &calls);
        ngo_sv alleles = {0};
        cluster_allele_calls(&calls, ref, p->max_base_qs, &alleles);
        ngo_icounts ih;
        icounts_run(&ih, &alleles, &calls, p->max_base_qs, 0.5);
        struct ngo_indel_call_s* ic = calloc(1, sizeof(*ic));
        const int ok = call_indel(&ih, &alleles, pos, is_str, is_input_str, G->het_rate, p->min_quality, p->ploidy, &ic->c);
        free(ih.counts); free(ih.logc);
        sv_free(&alleles);
        icalls_free(&calls);
        free(ref);
        if (ok) {
            memset(&c, 0, sizeof(c));
            c.pos = pos;
            ic->ploidy = p->ploidy;
            c.indel = ic;
            push_call(G, &c);
            G->last_indel_end = ic->c.last;                     /* a decided non-SNV call, :157-160 */
            return;
        }
        free(ic);
        if (is_input_str) return;
    }
    /* discoverSNV (also the fallback of a span whose indel alleles made no call, :264-271) */
    char R = (char)toupper((unsigned char)s->seq[pos - 1]);
    if (pool ? pool_discover(h, &G->acalls, pos, R, p, G->het_rate, &c) : discover_snv(h, pos, R, p, G->het_rate, &c)) {
        c.embedded = embedded;
        c.indel = NULL;
        push_call(G, &c);
    }
}

/* processCurrentPosition + listeners for one position, AlignmentsPileupGenerator.java:475-498 */
static int process_current_position(ngo_gen* G) {
    if (G->pending.n == 0) { G->cur_pos++; return 0; }
    const ngo_params* p = G->p;
    if (p->query_seq && (G->cur_pos < p->query_first || G->cur_pos > p->query_last)) { G->cur_pos++; return 0; }
    int pos = G->cur_pos;
    if (G->cov) {
        /* CoverageStatisticsCalculator.onPileup -> processPileup (CoverageStatisticsCalculator.java:124-131,
         * 177-190): PileupRecord.getNumAlignments / getNumUniqueAlns (PileupRecord.java:154-177; unique =
         * !FLAG_MULTIPLE_ALN, ReadAlignment.isUnique) binned at [0, maxCoverage), the rest in "More" */
        ngo_coverage* cv = G->cov;
        int numAlignments = 0, numUnique = 0;
        for (int k = 0; k < G->pending.n; k++) {
            const ngo_aln* a = G->pending.a[k];
            if (a->first > pos || a->last < pos) continue;
            numAlignments++;
            if (!(a->flags & FLAG_MULTIPLE)) numUnique++;
        }
        if (numAlignments < cv->max_coverage) cv->counts[numAlignments]++; else cv->high++;
        if (numUnique < cv->max_coverage) cv->counts_unique[numUnique]++; else cv->high_unique++;
        if (numAlignments > 0) G->st->positions_genotyped++;
        G->cur_pos++;
        return numAlignments > 0;
    }
    if (G->rac) {
        int numAlignments = 0;
        for (int k = 0; k < G->pending.n; k++)
            if (G->pending.a[k]->first <= pos && G->pending.a[k]->last >= pos) numAlignments++;
        if (numAlignments > 0) {
            G->st->positions_genotyped++;
            rac_on_pileup(G, pos);
        }
        G->cur_pos++;
        return numAlignments > 0;
    }
    if (G->mvd) {
        int numAlignments = 0;
        for (int k = 0; k < G->pending.n; k++)
            if (G->pending.a[k]->first <= pos && G->pending.a[k]->last >= pos) numAlignments++;
        if (numAlignments > 0) {
            G->st->positions_genotyped++;
            if (G->realign) {
                /* IndelRealignerPileupListener.onPileup first (MultisampleVariantsDetector.java:449-450) */
                G->pileup.n = 0;
                for (int k = 0; k < G->pending.n; k++) {
                    ngo_aln* a = G->pending.a[k];
                    if (a->first <= pos && a->last >= pos) alist_push(&G->pileup, a);
                }
                int var_first, var_last, var_str, is_str = 0, is_new_str = 0, r_embedded = 0;
                realigner_input_at(G, pos, &var_first, &var_last, &var_str);
                const int span = realigner_on_pileup(&G->g->s[G->cur_seq], G->pileup.a, G->pileup.n, pos, var_first, var_last,
                                                     var_str, &is_str, &is_new_str, &r_embedded);
                rtrace_pileup(G->pileup.a, G->pileup.n, pos, span, is_str, is_new_str, r_embedded);
                if (G->known) mvd_on_pileup_known(G, pos);
                else mvd_on_pileup_realign(G, pos, span, is_str, is_new_str, r_embedded);
            } else {
                mvd_on_pileup(G, pos);
            }
        }
        G->cur_pos++;
        return numAlignments > 0;
    }
    int numAlignments = 0;
    int span = 1, is_str = 0, is_new_str = 0, r_embedded = 0;
    if (G->realign) {
        /* IndelRealignerPileupListener.onPileup runs first and may edit the alignments (:85-126) */
        G->pileup.n = 0;
        for (int k = 0; k < G->pending.n; k++) {
            ngo_aln* a = G->pending.a[k];
            if (a->first <= pos && a->last >= pos) alist_push(&G->pileup, a);
        }
        if (G->pileup.n > 0) {
            int var_first, var_last, var_str;
            realigner_input_at(G, pos, &var_first, &var_last, &var_str);
            span = realigner_on_pileup(&G->g->s[G->cur_seq], G->pileup.a, G->pileup.n, pos, var_first, var_last, var_str, &is_str,
                                       &is_new_str, &r_embedded);
            rtrace_pileup(G->pileup.a, G->pileup.n, pos, span, is_str, is_new_str, r_embedded);
        }
    }
    ngo_counts h;
    ngo_counts_init(&h, 4, 0.5, p->max_base_qs);     /* CountsHelper.calculateCountsSNV(calls, maxBaseQS, 0.5) */
    const int pool = p->ploidy >= 3;                 /* SingleSampleVariantPileupListener.DEF_MIN_PLOIDY_POOL_ALGORITHM */
    G->acalls.n = 0;
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
        if (pool) acalls_push(&G->acalls, base_idx(a->chars[rp]), (int8_t)q, (a->flags & FLAG_REVERSE) != 0);
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
        if (G->known) {
            /* onPileup with input variants: every input variant at this position, in input order */
            while (G->known_next < G->n_known && G->known[G->known_next].seq == G->cur_seq && G->known[G->known_next].pos <= pos) {
                const ngo_known* kv = &G->known[G->known_next++];
                if (kv->pos != pos) continue;
                ngo_call c;
                if (!kv->snv) genotype_known_indel(G, kv, pos, &c);
                else if (pool) pool_known(&h, &G->acalls, kv, p, G->het_rate, &c);
                else genotype_known(&h, kv, p, G->het_rate, &c);
                if (G->calls.n == G->calls.cap) { G->calls.cap = G->calls.cap ? 2 * G->calls.cap : 1024; G->calls.c = realloc(G->calls.c, sizeof(ngo_call) * G->calls.cap); }
                G->calls.c[G->calls.n++] = c;
            }
        } else if (G->realign) {
            discover_with_span(G, pos, span, is_str, is_new_str, r_embedded, &h);
        } else if (!(p->ignore_lowercase_ref && islower((unsigned char)r))) {
            char R = (char)toupper((unsigned char)r);
            ngo_call c;
            if (pool ? pool_discover(&h, &G->acalls, pos, R, p, G->het_rate, &c)
                     : discover_snv(&h, pos, R, p, G->het_rate, &c)) {
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
        else { rtrace_aln(a); alist_push(&G->retired, a); }
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
        if (G->rac) rac_on_sequence_start(G, a->seq);
        G->last_indel_end = 0;                                 /* SingleSampleVariantPileupListener.onSequenceStart, :186 */
        G->str_next = 0;                                       /* IndelRealignerPileupListener.onSequenceStart, :128-133 */
        while (G->str_next < G->n_strs && G->strs[G->str_next].seq != a->seq) G->str_next++;
        if (G->known) {          /* onSequenceStart: this sequence's input variants, nextSIVIndex = 0 */
            G->known_next = 0;
            while (G->known_next < G->n_known && G->known[G->known_next].seq != a->seq) G->known_next++;
            G->rk_next = G->known_next;                        /* and the realigner's idxNextVariant */
        }
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

/* VCFFileReader.loadVariants(file, true, true) (vcf/VCFFileReader.java:585-600) sorted as a
 * GenomicRegionSortedCollection over the genome's sequences (GenomicRegionPositionComparator: first, then last;
 * stable).  loadGenomicVariant (:192-255): a biallelic SNV object for one-base ACGT REF and ALT, else a
 * GenomicVariantImpl over REF and the ALT alleles (indels, MNPs, alleles with N); a multi-allelic SNV (every allele
 * one ACGT base) is refused (NGO_UNSUPPORTED).  ALT '.' records are skipped (filterReferenceSitesGVCF), so are
 * structural types (filterSVs) and records on sequences outside the genome. */
static void known_free(ngo_known* v, int n) {
    for (int i = 0; i < n; i++) {
        free(v[i].id);
        for (int j = 0; j < v[i].n_alleles; j++) free(v[i].alleles[j]);
        free(v[i].alleles);
    }
    free(v);
}
static int known_cmp(const void* a, const void* b) {
    const ngo_known *x = a, *y = b;
    if (x->seq != y->seq) return x->seq < y->seq ? -1 : 1;
    if (x->pos != y->pos) return x->pos < y->pos ? -1 : 1;
    if (x->last != y->last) return x->last < y->last ? -1 : 1;
    return 0;
}
static int load_known(const char* path, const ngo_genome* g, ngo_known** out, int* n_out) {
    FILE* f = fopen(path, "r");
    if (!f) return NGO_ERR_IO;
    char* line = NULL; size_t cap = 0; ssize_t l;
    ngo_known* v = NULL; int n = 0, vc = 0, rc = NGO_OK;
    while ((l = getline(&line, &cap, f)) >= 0) {
        while (l > 0 && (line[l - 1] == '\n' || line[l - 1] == '\r')) line[--l] = 0;
        if (l == 0 || line[0] == '#') continue;
        char* fld[8]; int k = 0; char* s2 = line;
        while (k < 8) { fld[k++] = s2; char* t = strchr(s2, '\t'); if (!t) break; *t = 0; s2 = t + 1; }
        if (k < 6) { rc = NGO_ERR_ARG; break; }
        if (fld[4][0] == '.') continue;                        /* loadVariants: reference sites (< 2 alleles) */
        const int seq = genome_find(g, fld[0]);
        if (seq < 0) continue;
        /* loadInfoField (:261-305), attribute by attribute: TYPE sets a type id in (0, TYPE_INVERSION], SVTYPE one >= 10
         * (GenomicVariantImpl.getVariantTypeId names, GenomicVariant.java:32-56), END the last position of a
         * GenomicVariantImpl */
        int type = 0, end = 0;
        if (k >= 8 && strcmp(fld[7], ".") != 0) {
            static const char* kNames[] = {"SNV", "MULTISNV", "EMBEDDED", "INDEL", "STR", "CNV", "REPEAT", "DEL", "INS", "INV", "DUP",
                                           "Deletion", "Insertion"};
            static const int kIds[] = {1, 2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 12, 13};
            for (char* t = fld[7]; t && *t;) {
                char* e = strchr(t, ';');
                if (e) *e = 0;
                int is_type = strncmp(t, "TYPE=", 5) == 0, is_sv = strncmp(t, "SVTYPE=", 7) == 0;
                if (is_type || is_sv) {
                    const char* name = t + (is_type ? 5 : 7);
                    int id = 0;
                    for (int q = 0; q < 13; q++) if (strcmp(name, kNames[q]) == 0) id = kIds[q];
                    if (is_type && id > 0 && id <= 14) type = id;
                    if (is_sv && id >= 10) type = id;
                }
                if (strncmp(t, "END=", 4) == 0) end = atoi(t + 4);
                t = e ? e + 1 : NULL;
            }
        }
        if (type >= 10) continue;                              /* loadVariants: filterSVs (isStructural) */
        /* the alleles: REF, then ALT split at commas */
        int na = 1;
        for (const char* t = fld[4]; *t; t++) na += *t == ',';
        na += 1;
        int snv = na == 2 && strlen(fld[3]) == 1 && strlen(fld[4]) == 1 && strchr("ACGT", fld[3][0]) && strchr("ACGT", fld[4][0]);
        int allsnv = 1;                                        /* GenomicVariantImpl.isSNV: every allele one base */
        if (!snv) {
            if (strlen(fld[3]) != 1 || !strchr("ACGT", fld[3][0])) allsnv = 0;
            for (char* t = fld[4]; allsnv && *t;) {
                char* e = strchr(t, ',');
                const size_t len = e ? (size_t)(e - t) : strlen(t);
                if (len != 1 || !strchr("ACGT", t[0])) allsnv = 0;
                t = e ? e + 1 : t + len;
            }
            if (allsnv) { rc = NGO_UNSUPPORTED; break; }       /* multi-allelic SNV inputs: not supported here */
        }
        int qs = 0;
        if (fld[5][0] && fld[5][0] != '.') { double q = atof(fld[5]); if (q > 32767) q = 255; qs = (int)ngo_java_round(q); }
        if (n == vc) { vc = vc ? 2 * vc : 256; v = realloc(v, sizeof(ngo_known) * vc); }
        ngo_known* kv = &v[n];
        memset(kv, 0, sizeof(*kv));
        kv->seq = seq; kv->pos = atoi(fld[1]); kv->qs = qs; kv->snv = snv; kv->type = type;
        kv->id = strcmp(fld[2], ".") == 0 ? NULL : strdup(fld[2]);
        kv->last = kv->pos + (int)strlen(fld[3]) - 1;
        if (!snv && end > 0) kv->last = end;                   /* the END attribute of a GenomicVariantImpl (:282-289) */
        if (snv) { kv->ref = fld[3][0]; kv->alt = fld[4][0]; }
        else {
            kv->n_alleles = na;
            kv->alleles = malloc(sizeof(char*) * (size_t)na);
            kv->alleles[0] = strdup(fld[3]);
            int j = 1;
            for (char* t = fld[4]; *t && j < na;) {
                char* e = strchr(t, ',');
                const size_t len = e ? (size_t)(e - t) : strlen(t);
                kv->alleles[j] = strndup(t, len);
                for (char* c = kv->alleles[j]; *c; c++) *c = (char)toupper((unsigned char)*c);
                j++;
                t = e ? e + 1 : t + len;
            }
            for (char* c = kv->alleles[0]; *c; c++) *c = (char)toupper((unsigned char)*c);
            kv->n_alleles = j;
            int dup = 0;                                       /* a repeated allele: refused (not restated) */
            for (int x = 0; x < j; x++) for (int y = 0; y < x; y++) dup |= strcmp(kv->alleles[x], kv->alleles[y]) == 0;
            if (dup || j > 100) { n++; rc = NGO_UNSUPPORTED; break; }
        }
        n++;
    }
    free(line); fclose(f);
    if (rc != NGO_OK) { known_free(v, n); return rc; }
    /* GenomicRegionSortedCollection: GenomicRegionPositionComparator (first, then last), stable */
    int* ord = malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) ord[i] = i;
    for (int i = 1; i < n; i++) {          /* insertion sort keeps equal keys in order; input is nearly sorted */
        int x = ord[i], j = i - 1;
        while (j >= 0 && known_cmp(&v[ord[j]], &v[x]) > 0) { ord[j + 1] = ord[j]; j--; }
        ord[j + 1] = x;
    }
    ngo_known* w = malloc(sizeof(ngo_known) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) w[i] = v[ord[i]];
    free(v); free(ord);
    *out = w; *n_out = n;
    return NGO_OK;
}

/* ---- -knownSTRs ---- */

/* Integer.parseInt: an optional sign and decimal digits, within the int range */
static int java_parse_int(const char* t, int* out) {
    const char* c = t;
    int neg = 0;
    if (*c == '-' || *c == '+') { neg = *c == '-'; c++; }
    if (!*c) return 0;
    long long v = 0;
    for (; *c; c++) {
        if (*c < '0' || *c > '9') return 0;
        v = v * 10 + (*c - '0');
        if (v > 2147483648LL) return 0;
    }
    if (neg) v = -v;
    if (v > 2147483647LL || v < -2147483648LL) return 0;
    *out = (int)v;
    return 1;
}

/* genome.getReference(seq, first, last) upper-cased (ReferenceGenome.java:217-237: null outside [1, length]) */
static char* ref_sub_upper(const ngo_seq* s, int first, int last) {
    if (first < 1 || last > s->len || last < first - 1) return NULL;
    const int n = last - first + 1;
    char* r = malloc((size_t)n + 1);
    for (int i = 0; i < n; i++) r[i] = (char)toupper((unsigned char)s->seq[first - 1 + i]);
    r[n] = 0;
    return r;
}

/* AbstractLimitedSequence.getOverlapLength (sequences/AbstractLimitedSequence.java:376-390): the longest suffix of a
 * that is a prefix of b (a suffix longer than b never matches) */
static int overlap_length(const char* a, const char* b) {
    const int la = (int)strlen(a), lb = (int)strlen(b);
    for (int i = 0; i < la; i++) {
        if (la - i > lb) continue;
        if (memcmp(a + i, b, (size_t)(la - i)) == 0) return la - i;
    }
    return 0;
}

/* SingleSampleVariantsDetector.mergeSTRs (:873-881) */
static int merge_strs(const ngo_seq* s, int first, int last, int rfirst, int rlast) {
    if (rfirst - last > 5) return 0;
    if (rfirst - last <= 2) return 1;
    char* r1 = ref_sub_upper(s, first > last - 10 ? first : last - 10, last);
    char* r2 = ref_sub_upper(s, rfirst, rlast);
    int ans = 0;
    if (r1 && r2) ans = overlap_length(r1, r2) > 5;
    free(r1); free(r2);
    return ans;
}

static int strv_cmp(const void* a, const void* b) {
    const ngo_strv* x = a; const ngo_strv* y = b;
    if (x->seq != y->seq) return x->seq - y->seq;
    if (x->first != y->first) return x->first < y->first ? -1 : 1;
    return x->last < y->last ? -1 : x->last > y->last;
}

/* SimpleGenomicRegionFileHandler.loadRegions (genome/io/SimpleGenomicRegionFileHandler.java:57-80: fields split at
 * every space or tab, lines whose name / first / last do not parse are skipped) + makeNonRedundantSTRs / mergeSTRs /
 * makeSTRVariant (SingleSampleVariantsDetector.java:843-894).  Regions on sequences the genome does not hold are
 * never emitted (makeNonRedundantSTRs walks the genome's sequences); a region with last < first - 1 (Java's
 * subSequence would throw) is skipped. */
static int load_known_strs(const char* path, const ngo_genome* g, ngo_strv** out, int* n_out) {
    FILE* f = fopen(path, "r");
    if (!f) return NGO_ERR_IO;
    char* line = NULL; size_t cap = 0; ssize_t l;
    ngo_strv* v = NULL; int n = 0, vc = 0;
    while ((l = getline(&line, &cap, f)) >= 0) {
        while (l > 0 && (line[l - 1] == '\n' || line[l - 1] == '\r')) line[--l] = 0;
        char* fld[3]; int k = 0; char* s2 = line;
        while (k < 3) {
            fld[k++] = s2;
            char* t = s2;
            while (*t && *t != ' ' && *t != '\t') t++;
            if (!*t) break;
            *t = 0; s2 = t + 1;
        }
        if (k < 3) continue;
        int a, b;
        if (!java_parse_int(fld[1], &a) || !java_parse_int(fld[2], &b)) continue;
        const int seq = genome_find(g, fld[0]);
        if (seq < 0 || b < a - 1) continue;
        if (n == vc) { vc = vc ? 2 * vc : 256; v = realloc(v, sizeof(ngo_strv) * vc); }
        v[n].seq = seq; v[n].first = a; v[n].last = b;
        n++;
    }
    free(line); fclose(f);
    /* GenomicRegionSortedCollection: per sequence, GenomicRegionPositionComparator (first, then last), stable */
    int* ord = malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) ord[i] = i;
    for (int i = 1; i < n; i++) {
        int x = ord[i], j = i - 1;
        while (j >= 0 && strv_cmp(&v[ord[j]], &v[x]) > 0) { ord[j + 1] = ord[j]; j--; }
        ord[j + 1] = x;
    }
    ngo_strv* w = malloc(sizeof(ngo_strv) * (n > 0 ? n : 1));
    int m = 0;
    for (int i = 0; i < n;) {
        const int seq = v[ord[i]].seq;
        const ngo_seq* s = &g->s[seq];
        int first = 0, last = 0;
        for (; i < n && v[ord[i]].seq == seq; i++) {
            const ngo_strv* r = &v[ord[i]];
            if (last == 0 || !merge_strs(s, first, last, r->first, r->last)) {
                if (last > 0) {
                    const int vf = first - 1 > 1 ? first - 1 : 1, vl = last + 1 < s->len ? last + 1 : (int)s->len;
                    if (vf >= 1 && vl <= s->len && vl >= vf - 1) { w[m].seq = seq; w[m].first = vf; w[m].last = vl; m++; }
                }
                first = r->first;
            }
            last = r->last;
        }
        if (last > 0) {
            const int vf = first - 1 > 1 ? first - 1 : 1, vl = last + 1 < s->len ? last + 1 : (int)s->len;
            if (vf >= 1 && vl <= s->len && vl >= vf - 1) { w[m].seq = seq; w[m].first = vf; w[m].last = vl; m++; }
        }
    }
    free(v); free(ord);
    /* the variants' collection is sorted again (same comparator) */
    qsort(w, (size_t)m, sizeof(ngo_strv), strv_cmp);
    *out = w; *n_out = m;
    return NGO_OK;
}

static int run_detector(const char* fasta, const char* sam, const char* out_vcf,
                        const char* dump_path, const ngo_params* p, ngo_stats* stats, double min_adf, int multisample,
                        ngo_coverage* cov, ngo_rac* rac) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    ngo_stats st_local; ngo_stats* st = stats ? stats : &st_local;
    memset(st, 0, sizeof(*st));
    ngo_genome g;
    if (load_fasta(fasta, &g) != NGO_OK) return NGO_ERR_IO;
    FILE* in = fopen(sam, "r");
    if (!in) return NGO_ERR_IO;
    FILE* out = strcmp(out_vcf, "-") == 0 ? stdout : fopen(out_vcf, "w");
    if (!out) { fclose(in); return NGO_ERR_IO; }
    FILE* dump = dump_path ? fopen(dump_path, "w") : NULL;
    {
        const char* tp = getenv("NGO_REALIGN_TRACE");
        g_rtrace = tp && tp[0] ? fopen(tp, "w") : NULL;
    }

    ngo_gen G; memset(&G, 0, sizeof(G));
    G.p = p; G.g = &g; G.out = out; G.dump = dump; G.cur_seq = -1; G.st = st;
    /* SingleSampleVariantsDetector.run, :591-593 (MultisampleVariantsDetector keeps -h as given) */
    G.het_rate = p->het_rate;
    if (!multisample && !p->het_rate_set && p->ploidy == 1) G.het_rate = 1e-6;
    G.cov = cov;
    G.rac = rac;
    /* the indel realigner: first in both detectors' listener chains (SingleSampleVariantsDetector.java:919-925,
     * MultisampleVariantsDetector.java:449-450), at every ploidy; with -knownVariants its input variants are the known
     * records (fixed events), else the -knownSTRs */
    G.realign = !cov && !rac && !p->indel_passthrough;
    if (p->known_vcf && p->known_vcf[0]) {
        int lrc = load_known(p->known_vcf, &g, &G.known, &G.n_known);
        if (lrc != NGO_OK) {
            if (G.known) known_free(G.known, G.n_known);
            fclose(in); if (out != stdout) fclose(out); if (dump) fclose(dump);
            return lrc == NGO_ERR_IO ? NGO_ERR_IO : NGO_UNSUPPORTED;
        }
        /* inputVariants.size() == 0: the listeners discover (SingleSampleVariantPileupListener.java:148, Multisample
         * VariantsDetector.java:523); the -knownSTRs stay unread (else-if, :906) */
        if (G.n_known == 0) { known_free(G.known, 0); G.known = NULL; }
    }
    if (G.realign && !(p->known_vcf && p->known_vcf[0]) && p->known_strs && p->known_strs[0]) {
        if (load_known_strs(p->known_strs, &g, &G.strs, &G.n_strs) != NGO_OK) {
            fclose(in); if (out != stdout) fclose(out); if (dump) fclose(dump);
            return NGO_ERR_IO;
        }
    }
    if (!multisample && !cov && !rac) print_header(out, p);
    ngo_mvd M; memset(&M, 0, sizeof(M));
    ngo_strlist rg_sm = {0};       /* SM of each @RG (parallel to rgs) */
    int header_done = !multisample;

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
                char* sm = strstr(line, "\tSM:");
                char smv[256] = "";
                if (sm) { sm += 4; size_t k = 0; while (sm[k] && sm[k] != '\t' && k < sizeof(smv) - 1) { smv[k] = sm[k]; k++; } smv[k] = 0; }
                if (id) {
                    id += 4; char* e = strchr(id, '\t'); char save = 0; if (e) { save = *e; *e = 0; }
                    int before = rgs.n;
                    int ri = strlist_get(&rgs, id, 1);
                    if (rgs.n > before) {
                        if (rg_sm.n == rg_sm.cap) { rg_sm.cap = rg_sm.cap ? 2 * rg_sm.cap : 8; rg_sm.ids = realloc(rg_sm.ids, sizeof(char*) * rg_sm.cap); }
                        rg_sm.ids[rg_sm.n++] = strdup(sm ? smv : "");
                    }
                    (void)ri;
                    if (e) *e = save;
                }
            }
            continue;
        }
        if (!header_done) {
            /* MultisampleVariantsDetector.loadSamplesFromAlignmentHeaders (:499-523): samples by id
             * (TreeMap), each with its read groups (HashSet, Sample.java:36) */
            header_done = 1;
            ngo_strlist smids = {0};
            for (int i = 0; i < rg_sm.n; i++) if (rg_sm.ids[i][0]) strlist_get(&smids, rg_sm.ids[i], 1);
            M.n_samples = smids.n;
            M.ids = malloc(sizeof(char*) * (smids.n ? smids.n : 1));
            for (int i = 0; i < smids.n; i++) M.ids[i] = smids.ids[i];
            for (int i = 1; i < M.n_samples; i++) {
                char* v = M.ids[i]; int j = i - 1;
                while (j >= 0 && strcmp(M.ids[j], v) > 0) { M.ids[j + 1] = M.ids[j]; j--; }
                M.ids[j + 1] = v;
            }
            free(smids.ids);
            M.rg_sample = malloc(sizeof(int) * (rgs.n ? rgs.n : 1));
            M.rg_rank = malloc(sizeof(int) * (rgs.n ? rgs.n : 1));
            M.n_rank = calloc(M.n_samples ? M.n_samples : 1, sizeof(int));
            int* tmp = malloc(sizeof(int) * (rgs.n ? rgs.n : 1));
            for (int i = 0; i < rgs.n; i++) { M.rg_sample[i] = -1; M.rg_rank[i] = 0; }
            for (int s2 = 0; s2 < M.n_samples; s2++) {
                int n = 0;
                for (int i = 0; i < rgs.n; i++) if (rg_sm.ids[i][0] && strcmp(rg_sm.ids[i], M.ids[s2]) == 0) tmp[n++] = i;
                java_hashset_order(rgs.ids, tmp, n);
                for (int k = 0; k < n; k++) { M.rg_sample[tmp[k]] = s2; M.rg_rank[tmp[k]] = k; }
                M.n_rank[s2] = n;
            }
            free(tmp);
            M.min_adf = min_adf;
            M.ploidy = p->ploidy;
            M.h = calloc(M.n_samples ? M.n_samples : 1, sizeof(ngo_counts));
            M.calls = calloc(M.n_samples ? M.n_samples : 1, sizeof(ngo_scall));
            M.sc = calloc(M.n_samples ? M.n_samples : 1, sizeof(ngo_acalls));
            G.mvd = &M;
            print_header_samples(out, p, (const char* const*)M.ids, M.n_samples);
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
        a->id = (int)st->alignments_read - 1;
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
        /* reads with I/D: the indel realigner + indel discovery run for single-sample discovery at ploidy < 3; the
         * other listener chains with indels are outside this restatement (or pass-through on request) */
        if (a->has_indel && !cov && !rac && !p->indel_passthrough && !G.realign) { G.unsupported = 1; aln_free(a); rc = NGO_UNSUPPORTED; break; }
        process_alignment(&G, a);
    }
    if (multisample && !header_done) { header_done = 1; print_header_samples(out, p, NULL, 0); }
    if (rc == NGO_OK) notify_end(&G);
    if (rc == NGO_OK && cov) {
        /* CoverageStatisticsCalculator.printCoverageStats (:209-215) */
        for (int i = 1; i < cov->max_coverage; i++)
            fprintf(out, "%d\t%lld\t%lld\n", i, (long long)cov->counts[i], (long long)cov->counts_unique[i]);
        fprintf(out, "More\t%lld\t%lld\n", (long long)cov->high, (long long)cov->high_unique);
    }
    if (rc == NGO_OK && rac) rac_print(out, rac);
    free(line); free(last_qname); fclose(in);
    if (out != stdout) fclose(out); else fflush(out);
    if (dump) fclose(dump);
    for (int i = 0; i < G.pending.n; i++) { rtrace_aln(G.pending.a[i]); aln_free(G.pending.a[i]); }
    if (g_rtrace) { fclose(g_rtrace); g_rtrace = NULL; }
    for (int i = 0; i < G.ss_primary.n; i++) aln_free(G.ss_primary.a[i]);
    for (int i = 0; i < G.ss_secondary.n; i++) aln_free(G.ss_secondary.a[i]);
    for (int i = 0; i < G.calls.n; i++) {
        if (G.calls.c[i].indel) free_indel_call(G.calls.c[i].indel);
        if (G.calls.c[i].kindel) free_kindel(G.calls.c[i].kindel);
    }
    free(G.pending.a); free(G.ss_primary.a); free(G.ss_secondary.a); free(G.retired.a); free(G.calls.c); free(G.acalls.c); free(G.pileup.a);
    free(G.strs);
    if (G.known) known_free(G.known, G.n_known);
    for (int i = 0; i < g.n; i++) { free(g.s[i].name); free(g.s[i].seq); }
    free(g.s);
    for (int i = 0; i < rgs.n; i++) free(rgs.ids[i]);
    free(rgs.ids);
    for (int i = 0; i < rg_sm.n; i++) free(rg_sm.ids[i]);
    free(rg_sm.ids);
    if (multisample) {
        for (int i = 0; i < M.n_samples; i++) free(M.ids[i]);
        free(M.ids); free(M.rg_sample); free(M.rg_rank); free(M.n_rank); free(M.h); free(M.calls);
        for (int i = 0; i < M.n_samples; i++) free(M.sc[i].c);
        free(M.sc);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    st->seconds = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    return rc;
}

int ngo_run_ssvd(const char* fasta, const char* sam, const char* out_vcf,
                 const char* dump_path, const ngo_params* p, ngo_stats* stats) {
    return run_detector(fasta, sam, out_vcf, dump_path, p, stats, 0.0, 0, NULL, NULL);
}

/* MultisampleVariantsDetector.run (discovery/MultisampleVariantsDetector.java:421-459) on one SAM
 * holding every sample's read groups (the generator's merge of per-sample files). */
int ngo_run_mvd(const char* fasta, const char* sam, const char* out_vcf, const ngo_params* p,
                double min_allele_depth_freq, ngo_stats* stats) {
    return run_detector(fasta, sam, out_vcf, NULL, p, stats, min_allele_depth_freq, 1, NULL, NULL);
}

/* CoverageStatisticsCalculator.processFile (discovery/CoverageStatisticsCalculator.java:108-122): the
 * generator with processSecondaryAlignments=true (reader filters only unmapped records), maxAlnsPerStartPos
 * 100 and -minMQ (which decides isUnique); reads with indels are admitted (the coverage listener reads no
 * allele calls).  counts/counts_unique: max_coverage entries, caller-owned. */
int ngo_run_coverage(const char* fasta, const char* sam, const char* out_txt, int min_mq, int max_coverage,
                     int64_t* counts, int64_t* counts_unique, int64_t* high, int64_t* high_unique, ngo_stats* stats) {
    if (max_coverage < 1) return NGO_ERR_ARG;
    ngo_params p;
    ngo_params_default(&p);
    p.min_mq = min_mq;
    p.process_secondary = 1;
    p.max_alns_per_start = 100;
    ngo_coverage cv;
    memset(&cv, 0, sizeof(cv));
    cv.max_coverage = max_coverage;
    cv.counts = calloc(max_coverage, sizeof(int64_t));
    cv.counts_unique = calloc(max_coverage, sizeof(int64_t));
    int rc = run_detector(fasta, sam, out_txt, NULL, &p, stats, 0.0, 0, &cv, NULL);
    if (counts) memcpy(counts, cv.counts, sizeof(int64_t) * max_coverage);
    if (counts_unique) memcpy(counts_unique, cv.counts_unique, sizeof(int64_t) * max_coverage);
    if (high) *high = cv.high;
    if (high_unique) *high_unique = cv.high_unique;
    free(cv.counts); free(cv.counts_unique);
    return rc;
}

/* RelativeAlleleCountsCalculator.runProcess + printResults (discovery/RelativeAlleleCountsCalculator.java:183-244):
 * the generator with maxAlnsPerStartPos = maxRD and processSecondaryAlignments = secondaryAlns, default
 * minMQ; reads with indels are admitted (no realigner in this listener chain). */
int ngo_run_rac(const char* fasta, const char* sam, const char* out_txt, int min_rd, int max_rd, int min_bq,
                int secondary, ngo_stats* stats) {
    ngo_params p;
    ngo_params_default(&p);
    p.max_alns_per_start = max_rd;
    p.process_secondary = secondary;
    ngo_rac R;
    memset(&R, 0, sizeof(R));
    R.min_rd = min_rd;
    R.min_bq = min_bq;
    int rc = run_detector(fasta, sam, out_txt, NULL, &p, stats, 0.0, 0, NULL, &R);
    free(R.seq_names);
    free(R.seq_dist);
    return rc;
}
