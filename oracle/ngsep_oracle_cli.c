/*
 * ngsep_oracle_cli.c -- command-line front end of the CPU restatement (TEST INFRASTRUCTURE ONLY).
 * Mirrors `java -jar NGSEPcore.jar SingleSampleVariantsDetector` option names
 * (src/ngsep/main/CommandsDescriptor.xml:565-703) for the options the oracle restates.
 * Input alignments are SAM text (the oracle does not decode BAM).
 */
#include "ngsep_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv) {
    ngo_params p; ngo_params_default(&p);
    const char *ref = NULL, *in = NULL, *outp = NULL, *dump = NULL;
    int i = 1, mvd = 0;
    double min_adf = 0;
    if (i < argc && strcmp(argv[i], "SingleSampleVariantsDetector") == 0) i++;
    else if (i < argc && strcmp(argv[i], "MultisampleVariantsDetector") == 0) { i++; mvd = 1; }
    for (; i < argc; i++) {
        const char* a = argv[i];
        const char* v = (i + 1 < argc) ? argv[i + 1] : NULL;
#define OPT(name) (strcmp(a, name) == 0 && v && (i++, 1))
        if (OPT("-r")) ref = v;
        else if (OPT("-i")) in = v;
        else if (OPT("-o")) outp = v;
        else if (OPT("-dump")) dump = v;
        else if (OPT("-minAlleleDepthFrequency")) min_adf = atof(v);
        else if (mvd && a[0] != '-' && !in) in = a;    /* MultisampleVariantsDetector: positional alignments file */
        else if (OPT("-sampleId")) p.sample_id = v;
        else if (OPT("-ploidy")) p.ploidy = atoi(v);
        else if (OPT("-minMQ")) p.min_mq = atoi(v);
        else if (OPT("-maxAlnsPerStartPos")) p.max_alns_per_start = atoi(v);
        else if (OPT("-ignore5")) p.ignore5 = atoi(v);
        else if (OPT("-ignore3")) p.ignore3 = atoi(v);
        else if (OPT("-maxBaseQS")) p.max_base_qs = atoi(v);
        else if (OPT("-minQuality")) p.min_quality = atoi(v);
        else if (OPT("-h")) { p.het_rate = atof(v); p.het_rate_set = 1; }
        else if (OPT("-querySeq")) p.query_seq = v;
        else if (OPT("-first")) p.query_first = atoi(v);
        else if (OPT("-last")) p.query_last = atoi(v);
        else if (OPT("-knownVariants")) p.known_vcf = v;
        else if (OPT("-knownSTRs")) p.known_strs = v;
        else if (strcmp(a, "-p") == 0) p.process_nonunique = 1;
        else if (strcmp(a, "-s") == 0) p.process_secondary = 1;
        else if (strcmp(a, "-ignoreLowerCaseRef") == 0) p.ignore_lowercase_ref = 1;
        else if (strcmp(a, "-embeddedSNVs") == 0) p.call_embedded = 1;
        else if (strcmp(a, "-csb") == 0) p.calc_strand_bias = 1;
        else if (strcmp(a, "-psp") == 0) p.print_sample_ploidy = 1;
        else { fprintf(stderr, "unknown or incomplete option %s\n", a); return 2; }
#undef OPT
    }
    if (!ref || !in || !outp) { fprintf(stderr, "usage: %s [SingleSampleVariantsDetector] -r ref.fa -i in.sam -o prefix [options]\n", argv[0]); return 2; }
    char* vcf = malloc(strlen(outp) + 8);
    sprintf(vcf, "%s.vcf", outp);
    ngo_stats st;
    int rc = mvd ? ngo_run_mvd(ref, in, outp, &p, min_adf, &st)     /* MVD: -o is the VCF path (MultisampleVariantsDetector.java:64) */
                 : ngo_run_ssvd(ref, in, strcmp(outp, "-") == 0 ? "-" : vcf, dump, &p, &st);
    fprintf(stderr, "oracle rc=%d alignments=%lld admitted=%lld positions=%lld variants=%lld seconds=%.3f\n", rc,
            (long long)st.alignments_read, (long long)st.alignments_admitted, (long long)st.positions_genotyped,
            (long long)st.variants_called, st.seconds);
    free(vcf);
    return rc;
}
