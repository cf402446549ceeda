"""Host staging profile (no GPU needed): the chr20 30x end-to-end BAM of bench.py, then
  (1) BAM decode alone (ngsep_bam_next_batch),
  (2) decode + admission + projection (ngsep_stage_alignments, NGSEP_HOST_TIMING breakdown),
  (3) the layout of ngsep_stage_finish up to the device (fails there without a GPU).
usage: python tools/host_profile.py [--keep DIR] [--depth 30]"""
import argparse
import ctypes
import os
import sys
import tempfile
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "synth")]
import pysynth  # noqa: E402
from ngsepcore_amd import GpuPileupSession, _lib, default_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=None)
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--contig", type=int, default=19)
    ap.add_argument("--e2e-only", action="store_true", help="only the BAM -> VCF run (needs a GPU)")
    ap.add_argument("--decode-only", action="store_true", help="only the BAM decode (ngsep_bam_next_batch)")
    a = ap.parse_args()
    d = a.dir or tempfile.mkdtemp(prefix="ngsep_hp_")
    os.makedirs(d, exist_ok=True)
    fa, bam = os.path.join(d, "c.fa"), os.path.join(d, "c.bam")
    if not os.path.exists(bam):
        t = time.time()
        syn = pysynth.Synth(genome=pysynth.HUMAN, depth=a.depth, seed=4, contig_first=a.contig, n_contigs=1, rng_per_contig=1)
        pysynth.lib().ngs_synth_write_fasta(syn.h, fa.encode())
        pysynth.lib().ngs_synth_write_bam(syn.h, bam.encode())
        syn.close()
        print(f"wrote {bam} ({os.path.getsize(bam) / 1e9:.2f} GB) in {time.time() - t:.1f}s", flush=True)
    lib = _lib.load()
    if a.e2e_only:
        import resource
        with GpuPileupSession(default_params()) as s:
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            t = time.time()
            s.load_fasta(fa)
            try:
                s.processFile(bam, os.path.join(d, "out.vcf"))
            except Exception as e:  # no device here: the time up to the device step
                print("processFile:", str(e)[:80])
            wall = time.time() - t
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            print(f"end-to-end: {wall:.2f}s, {s.stats().positions_genotyped} positions; cpu user {ru1.ru_utime - ru0.ru_utime:.2f}s "
                  f"sys {ru1.ru_stime - ru0.ru_stime:.2f}s, minor faults {ru1.ru_minflt - ru0.ru_minflt}", flush=True)
        return
    s = GpuPileupSession(default_params())
    s.load_fasta(fa)
    # (1) decode only
    b = ctypes.c_void_p()
    batch = _lib.NgsepReadBatch()
    t = time.time()
    assert lib.ngsep_bam_open(s._ctx, bam.encode(), ctypes.byref(b)) == 0
    n = 0
    while True:
        assert lib.ngsep_bam_next_batch(b, 1 << 20, ctypes.byref(batch)) == 0
        if batch.n_reads == 0:
            break
        n += batch.n_reads
    lib.ngsep_bam_close(b)
    t_dec = time.time() - t
    print(f"decode: {n} reads in {t_dec:.2f}s", flush=True)
    if a.decode_only:
        return
    # (2) decode + staging
    t = time.time()
    assert lib.ngsep_bam_open(s._ctx, bam.encode(), ctypes.byref(b)) == 0
    while True:
        assert lib.ngsep_bam_next_batch(b, 1 << 20, ctypes.byref(batch)) == 0
        if batch.n_reads == 0:
            break
        s.stage(batch)
    lib.ngsep_bam_close(b)
    t_stage = time.time() - t
    print(f"decode + admission + projection: {t_stage:.2f}s", flush=True)
    t = time.time()
    try:
        s.stage_finish()
    except Exception as e:  # no device here
        print("stage_finish:", str(e)[:80])
    print(f"layout (+ device attempt): {time.time() - t:.2f}s", flush=True)
    print(f"data kept in {d}")


if __name__ == "__main__":
    main()
