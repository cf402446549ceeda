// synth_cli.cpp -- writes a synthetic dataset to disk (test/bench data infrastructure).
// usage: ngsep_synth OUTPREFIX [genome yeast|human|custom:LEN] [depth] [seed] [n_contigs] [contig_first] [extras]
#include "ngsep_synth.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: %s OUTPREFIX [yeast|human|custom:LEN] [depth] [seed] [n_contigs] [contig_first] [variety]\n", argv[0]); return 2; }
    ngs_synth_params p; ngs_synth_default(&p);
    if (argc > 2) {
        if (!std::strcmp(argv[2], "human")) p.genome = NGS_GENOME_HUMAN;
        else if (!std::strncmp(argv[2], "custom:", 7)) { p.genome = NGS_GENOME_CUSTOM; p.custom_len = std::atoll(argv[2] + 7); }
    }
    if (argc > 3) p.depth = std::atof(argv[3]);
    if (argc > 4) p.seed = std::strtoull(argv[4], nullptr, 10);
    if (argc > 5) p.n_contigs = std::atoi(argv[5]);
    if (argc > 6) p.contig_first = std::atoi(argv[6]);
    if (argc > 7 && std::atoi(argv[7])) {  // exercise reader / admission edge cases
        p.secondary_rate = 0.01; p.lowmq_rate = 0.01; p.noqual_rate = 0.005; p.softclip_rate = 0.05; p.dup_rate = 0.02; p.lower_frac = 0.01;
    }
    ngs_synth* s = ngs_synth_create(&p);
    std::string o = argv[1];
    int rc = ngs_synth_write_fasta(s, (o + ".fa").c_str()) | ngs_synth_write_sam(s, (o + ".sam").c_str()) |
             ngs_synth_write_bam(s, (o + ".bam").c_str()) | ngs_synth_write_truth(s, (o + "_truth.vcf").c_str());
    std::fprintf(stderr, "contigs=%d reads=%lld bases=%lld rc=%d\n", ngs_synth_n_contigs(s), (long long)ngs_synth_n_reads(s), (long long)ngs_synth_n_bases(s), rc);
    ngs_synth_free(s);
    return rc;
}
