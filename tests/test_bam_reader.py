"""The C++ BAM reader (libngsep_amd.so ngsep_bam_*; htsjdk's role in ReadAlignmentFileReader.java:171-354)
on the CPU: the threaded BGZF decoder and the parallel record decoder against the generator's own view of
the same records, and BAI region reads (ngsep_bam_set_region) against a filter of the whole stream."""
import ctypes
import os

import pytest

import pysynth
from ngsepcore_amd import _lib, default_params


def _ctx(contigs):
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    p = default_params()
    assert lib.ngsep_open(0, ctypes.byref(p), ctypes.byref(ctx)) == 0
    for name, seq in contigs:
        assert lib.ngsep_set_reference(ctx, name.encode(), seq, len(seq)) == 0
    return lib, ctx


def _records(batch):
    """(seq_id, first, flags, rg, cigar, bases, quals, has_quals) per read of a batch."""
    out = []
    # the raw pointers (reading a c_char_p field would copy up to the first NUL)
    bases = ctypes.c_void_p.from_buffer(batch, _lib.NgsepReadBatch.bases.offset).value
    quals = ctypes.c_void_p.from_buffer(batch, _lib.NgsepReadBatch.quals.offset).value
    for i in range(batch.n_reads):
        co, cn = batch.cigar_off[i], batch.cigar_n[i]
        so, sl = batch.seq_off[i], batch.seq_len[i]
        hq = batch.has_quals[i] if batch.has_quals else 1
        out.append((batch.seq_id[i], batch.first[i], batch.flags[i], batch.read_group[i],
                    tuple(batch.cigar[co + k] for k in range(cn)), ctypes.string_at(bases + so, sl),
                    ctypes.string_at(quals + so, sl) if hq else b"*", hq))
    return out


def _read_all(lib, ctx, bam, batch_reads=1 << 20, region=None):
    b = ctypes.c_void_p()
    assert lib.ngsep_bam_open(ctx, bam.encode(), ctypes.byref(b)) == 0, lib.ngsep_last_error(ctx)
    if region is not None:
        rc = lib.ngsep_bam_set_region(b, region[0].encode(), region[1], region[2])
        assert rc == 0, lib.ngsep_last_error(ctx)
    out = []
    batch = _lib.NgsepReadBatch()
    while True:
        assert lib.ngsep_bam_next_batch(b, batch_reads, ctypes.byref(batch)) == 0, lib.ngsep_last_error(ctx)
        if batch.n_reads == 0:
            break
        out += _records(batch)
    lib.ngsep_bam_close(b)
    return out


@pytest.mark.parametrize("kw,batch_reads", [
    (dict(genome=pysynth.YEAST, n_contigs=3, depth=12, seed=21), 1 << 20),
    (dict(genome=pysynth.YEAST, n_contigs=3, depth=12, seed=22, softclip_rate=0.05), 20000),   # parallel cuts stopped at max_reads
    (dict(genome=pysynth.YEAST, n_contigs=2, depth=15, seed=7, secondary_rate=0.02, lowmq_rate=0.02, noqual_rate=0.01,
          softclip_rate=0.05, dup_rate=0.03, quality_model=2), 777),
])
def test_reader_matches_generator(tmp_path, kw, batch_reads):
    """Every record the reader keeps (after isSameAlignment, isMultiple and the filter flags) equals the
    generator's filtered view, in order, whatever the batch size (records cut across decoded chunks; a whole
    decoded chunk cut on all threads, bam.cpp parallel_cut, at 1 << 20 and 20000 reads a batch)."""
    syn = pysynth.Synth(**kw)
    _, _, bam = syn.write(os.path.join(str(tmp_path), "r"))
    lib, ctx = _ctx(syn.contigs())
    got = _read_all(lib, ctx, bam, batch_reads)
    want = _records(syn.batch())
    lib.ngsep_close(ctx)
    syn.close()
    assert len(got) == len(want) > 1000
    assert got == want


@pytest.mark.parametrize("read_bytes", ["4096", "100000", "1000003"])
def test_reader_small_file_reads(tmp_path, monkeypatch, read_bytes):
    """The decoder's file reads cut BGZF blocks (the cut block carried to the front of the reused buffer): every record
    equal to the generator's whatever the read size (NGSEP_BGZF_READ, test hook; 32 MB otherwise)."""
    monkeypatch.setenv("NGSEP_BGZF_READ", read_bytes)
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=10, seed=31, softclip_rate=0.05)
    _, _, bam = syn.write(os.path.join(str(tmp_path), "r"))
    lib, ctx = _ctx(syn.contigs())
    got = _read_all(lib, ctx, bam, 50000)
    want = _records(syn.batch())
    lib.ngsep_close(ctx)
    syn.close()
    assert len(got) == len(want) > 1000
    assert got == want


def test_parallel_cut_merge_walks_missed_segments(tmp_path, monkeypatch):
    """A parallel-cut segment whose own walk never meets the true record chain is walked sequentially by the
    merge (NGSEP_PCUT_MISS: odd segments start off the chain): the records are the same."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=12, seed=23)
    _, _, bam = syn.write(os.path.join(str(tmp_path), "m"))
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = %r; import test_bam_reader as t, pysynth, hashlib; "
            "syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=12, seed=23); "
            "lib, ctx = t._ctx(syn.contigs()); print(hashlib.sha1(repr(t._read_all(lib, ctx, %r)).encode()).hexdigest())"
            % (sys.path[:6], bam))
    runs = []
    for miss in ("", "1"):
        env = dict(os.environ, NGSEP_HOST_TIMING="1")
        env.pop("NGSEP_PCUT_MISS", None)
        if miss:
            env["NGSEP_PCUT_MISS"] = miss
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
        runs.append(out.stdout.strip())
        if miss:
            assert "0 segments walked sequentially" not in out.stderr, out.stderr
    lib, ctx = _ctx(syn.contigs())
    want = _records(syn.batch())
    lib.ngsep_close(ctx)
    syn.close()
    import hashlib
    assert runs[0] == runs[1] == hashlib.sha1(repr(want).encode()).hexdigest()


def test_reader_zlib_and_libdeflate_agree(tmp_path, monkeypatch):
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=10, seed=3)
    _, _, bam = syn.write(os.path.join(str(tmp_path), "z"))
    lib, ctx = _ctx(syn.contigs())
    a = _read_all(lib, ctx, bam)
    lib.ngsep_close(ctx)
    syn.close()
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = %r; import test_bam_reader as t, pysynth; "
            "syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=10, seed=3); "
            "lib, ctx = t._ctx(syn.contigs()); print(len(t._read_all(lib, ctx, %r)))" % (sys.path[:6], bam))
    env = dict(os.environ, NGSEP_ZLIB="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert int(out.stdout.strip()) == len(a) > 1000


@pytest.mark.parametrize("region", [("chrII", 1, 5000), ("chrII", 200000, 400000), ("chrI", 100000, 100150),
                                    ("chrIII", 316000, 316620), ("chrI", 1, 230218)])
def test_region_reads(tmp_path, region):
    """ngsep_bam_set_region through the generator's BAI: the records returned are of the region's
    sequence, start at or before its last position, and include every record overlapping it."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=10, seed=5, softclip_rate=0.05)
    _, _, bam = syn.write(os.path.join(str(tmp_path), "g"))
    names = [n for n, _ in syn.contigs()]
    lib, ctx = _ctx(syn.contigs())
    allr = _read_all(lib, ctx, bam)
    got = _read_all(lib, ctx, bam, region=region)
    lib.ngsep_close(ctx)
    syn.close()
    sid = names.index(region[0])

    def last_of(r):
        return r[1] + sum(c // 8 for c in r[4] if c & 1) - 1
    want = [r for r in allr if r[0] == sid and r[1] <= region[2] and last_of(r) >= region[1]]
    assert all(r[0] == sid and r[1] <= region[2] for r in got)
    gs = set(got)
    assert all(r in gs for r in want) and len(want) > 0
    # the seek skipped the records before the region (not a whole-file scan)
    assert len(got) < len([r for r in allr if r[0] == sid]) or region[1] == 1


def test_region_without_index_is_io_error(tmp_path):
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=5, seed=5)
    _, _, bam = syn.write(os.path.join(str(tmp_path), "n"))
    os.remove(bam + ".bai")
    lib, ctx = _ctx(syn.contigs())
    b = ctypes.c_void_p()
    assert lib.ngsep_bam_open(ctx, bam.encode(), ctypes.byref(b)) == 0
    assert lib.ngsep_bam_set_region(b, b"chrI", 1, 100) == _lib.NGSEP_E_IO
    lib.ngsep_bam_close(b)
    lib.ngsep_close(ctx)
    syn.close()
