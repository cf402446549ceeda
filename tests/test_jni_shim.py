"""The JNI binding (jni/ngsep_gpu_jni.c: the natives of ngsep.discovery.gpu.GpuPileupEngine)
compiled and RUN: the image has no JDK, so tests/jni_harness supplies a JNIEnv of its own (Java strings, int[] / long[] /
String[] arrays, exceptions) and a C API that calls the natives as the JVM would.  CPU: the option array reaches
ngsep_params, the reference loads, errors surface as status codes and IOExceptions (no device: NGSEP_E_DEVICE, never a
CPU fallback).  GPU: findSNVS, the multi-device run and MultisampleVariantsDetector through the natives write the same
VCFs as the library's own entry points."""
import ctypes
import os

import pytest

import pysynth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "jni", "build", "libngsep_jni_harness.so")
I64, I32, CP = ctypes.c_int64, ctypes.c_int32, ctypes.c_char_p


def harness():
    l = ctypes.CDLL(SO)
    l.h_open.restype = I64
    l.h_open.argtypes = [ctypes.c_int, ctypes.POINTER(I32), ctypes.c_int, ctypes.c_double, CP, CP]
    l.h_close.argtypes = [I64]
    l.h_last_error.argtypes = [I64, ctypes.c_char_p, ctypes.c_int]
    l.h_exception.restype = CP
    for f in ("h_load_fasta", "h_set_known_variants", "h_set_known_strs"):
        getattr(l, f).argtypes = [I64, CP]
    l.h_call_bam.argtypes = [I64, CP, CP]
    l.h_call_region_bam.argtypes = [I64, CP, CP, I64, I64, CP]
    l.h_call_population_bams.argtypes = [I64, ctypes.POINTER(CP), ctypes.c_int, CP]
    l.h_call_bam_multi.argtypes = [ctypes.POINTER(I64), ctypes.c_int, CP, CP, I64]
    l.h_call_population_bams_multi.argtypes = [ctypes.POINTER(I64), ctypes.c_int, ctypes.POINTER(CP), ctypes.c_int, CP, I64]
    l.h_carved_regions.restype = I64
    l.h_carved_regions.argtypes = [I64, ctypes.POINTER(I64), I64]
    P = ctypes.POINTER
    l.h_process_alignments.argtypes = [I64, ctypes.c_int, P(I32), P(I32), P(I32), P(I32), P(I64), P(I32), P(I32),
                                       ctypes.c_int, P(I64), P(I32), ctypes.c_void_p, ctypes.c_void_p, I64,
                                       P(ctypes.c_uint8)]
    l.h_notify_end.argtypes = [I64]
    l.h_fetch_sites.restype = I64
    l.h_fetch_sites.argtypes = [I64, ctypes.c_void_p, I64, P(ctypes.c_int)]
    return l


def shim_path_a(l, ctx, batch):
    """processAlignments (the batch copied into Java arrays) + notifyEnd + fetchSites through the natives: the sites'
    bytes and whether the buffer's order was set to LITTLE_ENDIAN"""
    import numpy as np
    n = batch.n_reads
    def arr(ptr, k, t):
        return np.ctypeslib.as_array(ptr, shape=(k,)).astype(t)
    cig_off = arr(batch.cigar_off, n, np.int64)
    cig_n = arr(batch.cigar_n, n, np.int32)
    n_cig = int((cig_off + cig_n).max()) if n else 0
    seq_off = arr(batch.seq_off, n, np.int64)
    seq_len = arr(batch.seq_len, n, np.int32)
    n_bases = int((seq_off + seq_len).max()) if n else 0
    keep = []

    def P32(a):
        a = np.ascontiguousarray(a, dtype=np.int32)
        keep.append(a)
        return a.ctypes.data_as(ctypes.POINTER(I32))
    bases_p = ctypes.c_void_p.from_buffer(batch, type(batch).bases.offset).value
    quals_p = ctypes.c_void_p.from_buffer(batch, type(batch).quals.offset).value
    hq = np.ascontiguousarray(arr(batch.has_quals, n, np.uint8))
    rc = l.h_process_alignments(ctx, n, P32(arr(batch.seq_id, n, np.int32)), P32(arr(batch.first, n, np.int32)),
                                P32(arr(batch.flags, n, np.int32)), P32(arr(batch.read_group, n, np.int32)),
                                cig_off.ctypes.data_as(ctypes.POINTER(I64)), P32(cig_n),
                                P32(np.ctypeslib.as_array(batch.cigar, shape=(n_cig,))), n_cig,
                                seq_off.ctypes.data_as(ctypes.POINTER(I64)), P32(seq_len), bases_p, quals_p, n_bases,
                                hq.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    if rc != 0:
        return rc, None, 0
    rc = l.h_notify_end(ctx)
    if rc != 0:
        return rc, None, 0
    # (fetchSites hands the records over once and clears them: one call with room for them all)
    cap = 152 * (1 << 16)
    buf = ctypes.create_string_buffer(cap)
    le = ctypes.c_int(0)
    m = l.h_fetch_sites(ctx, buf, cap, ctypes.byref(le))
    assert m <= cap
    return 0, buf.raw[:max(0, m)], le.value


def options(**kw):
    """GpuPileupEngine.optionArray(): ngsep_params fields in the shim's order"""
    order = ["min_mq", "max_alns_per_start", "ignore5", "ignore3", "max_base_qs", "min_quality", "ploidy", "process_nonunique",
             "process_secondary", "ignore_lowercase_ref", "call_embedded", "calc_strand_bias", "print_sample_ploidy",
             "het_rate_set", "query_first", "query_last", "multisample", "coverage_stats", "max_coverage",
             "relative_allele_counts", "rac_min_rd", "rac_min_bq", "indel_passthrough"]
    from ngsepcore_amd import default_params
    p = default_params()
    vals = [int(kw.get(k, getattr(p, k))) for k in order]
    return (I32 * len(vals))(*vals), len(vals)


def err(l, ctx):
    b = ctypes.create_string_buffer(1024)
    l.h_last_error(ctx, b, 1024)
    return b.value.decode()


def test_shim_cpu_paths(tmp_path):
    l = harness()
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=20000, seed=91, depth=6)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "j"))
    syn.close()
    o, n = options(min_quality=30, ploidy=1)
    ctx = l.h_open(0, o, n, 0.001, None, b"S1")
    assert ctx != 0 and l.h_exception() == b""
    assert l.h_load_fasta(ctx, fa.encode()) == 0
    assert l.h_load_fasta(ctx, b"/nonexistent.fa") == -2 and "nonexistent" in err(l, ctx)
    assert l.h_load_fasta(ctx, fa.encode()) == 0
    out = os.path.join(str(tmp_path), "j.vcf").encode()
    if not __import__("torch").cuda.is_available():
        assert l.h_call_bam(ctx, bam.encode(), out) == -4            # NGSEP_E_DEVICE: no CPU fallback
        assert err(l, ctx)
    cr = (I64 * 3)()
    assert l.h_carved_regions(ctx, cr, 1) == 0
    # fetchSites on a context without calls: an empty buffer, its order set to LITTLE_ENDIAN, no exception
    le = ctypes.c_int(0)
    assert l.h_fetch_sites(ctx, None, 0, ctypes.byref(le)) == 0 and le.value == 1 and l.h_exception() == b""
    l.h_close(ctx)
    # processAlignments' marshalling (the twelve arrays through Get<Type>ArrayElements): without a device the batch is
    # refused with NGSEP_E_DEVICE or buffered, never an OutOfMemoryError
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=20000, seed=91, depth=6)
    o, n = options()
    ctx = l.h_open(0, o, n, 0.001, None, None)
    assert l.h_load_fasta(ctx, fa.encode()) == 0
    rc, _, _ = shim_path_a(l, ctx, syn.batch())
    syn.close()
    assert rc in (0, -4) and b"OutOfMemoryError" not in l.h_exception()
    l.h_close(ctx)
    # an option the library refuses: ngsep_open throws IOException through the shim and returns 0
    o, n = options(ploidy=500)
    assert l.h_open(0, o, n, 0.001, None, None) == 0
    assert l.h_exception().startswith(b"java/io/IOException")


@pytest.mark.gpu
def test_shim_gpu_runs_equal_library(tmp_path):
    from ngsepcore_amd import GpuPileupSession, MultisampleVariantsDetector
    l = harness()
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=120000, seed=92, depth=15, snv_rate=2e-3, indel_rate=4e-4,
                        n_samples=1)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "g"))
    syn.close()
    want = os.path.join(str(tmp_path), "lib.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        s.processFile(bam, want)
    o, n = options()
    ctx = l.h_open(0, o, n, 0.001, None, None)
    assert ctx and l.h_load_fasta(ctx, fa.encode()) == 0
    got = os.path.join(str(tmp_path), "jni.vcf")
    assert l.h_call_bam(ctx, bam.encode(), got.encode()) == 0, err(l, ctx)
    assert open(got).read() == open(want).read()
    ctx2 = l.h_open(0, o, n, 0.001, None, None)
    ctxs = (I64 * 2)(ctx, ctx2)
    multi = os.path.join(str(tmp_path), "multi.vcf")
    assert l.h_call_bam_multi(ctxs, 2, bam.encode(), multi.encode(), 30000) == 0, err(l, ctx)
    assert open(multi).read() == open(want).read()
    l.h_close(ctx)
    l.h_close(ctx2)
    # path A through the natives (processAlignments with Get<Type>ArrayElements, notifyEnd, fetchSites): the records,
    # read little endian from the returned buffer, are the library's own calls (the VCF's positions)
    import struct
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=60000, seed=94, depth=15, snv_rate=2e-3)
    fa2, sam2, bam2 = syn.write(os.path.join(str(tmp_path), "a"))
    want2 = os.path.join(str(tmp_path), "a_lib.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa2)
        s.processFile(bam2, want2)
    ctx = l.h_open(0, o, n, 0.001, None, None)
    assert l.h_load_fasta(ctx, fa2.encode()) == 0
    rc, raw, le = shim_path_a(l, ctx, syn.batch())
    assert rc == 0, err(l, ctx)
    assert le == 1
    recs = [struct.unpack_from("<ii", raw, k) for k in range(0, len(raw), 152)]
    vcf_pos = [int(x.split("\t")[1]) for x in open(want2) if not x.startswith("#")]
    assert [p for _, p in recs] == vcf_pos and len(vcf_pos) > 50
    l.h_close(ctx)
    syn.close()
    # MultisampleVariantsDetector through callPopulationBams
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=40000, seed=93, depth=8, snv_rate=3e-3, n_samples=6)
    fa, sam, _ = syn.write(os.path.join(str(tmp_path), "p"))
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    syn.close()
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    d.setOutFilename(os.path.join(str(tmp_path), "pop_lib.vcf"))
    d.run(bams).close()
    o, n = options(multisample=1)
    ctx = l.h_open(0, o, n, 0.001, None, None)
    assert l.h_load_fasta(ctx, fa.encode()) == 0
    arr = (CP * len(bams))(*[b.encode() for b in bams])
    got = os.path.join(str(tmp_path), "pop_jni.vcf")
    assert l.h_call_population_bams(ctx, arr, len(bams), got.encode()) == 0, err(l, ctx)
    assert open(got).read() == open(d.outFilename).read()
    l.h_close(ctx)
