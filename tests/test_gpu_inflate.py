"""BGZF inflate on the device (inflate.hip, KZ) against zlib, and the BAM readers with it against the host inflate.

The reference reads BAMs through htsjdk's BlockCompressedInputStream (ReadAlignmentFileReader.java:171-183), which
inflates with java.util.zip.Inflater; zlib is the same DEFLATE (RFC 1951), so the decoded bytes must be identical.
The blocks below cover every DEFLATE block type and code path: stored blocks (level 0, incompressible data, the
empty blocks of a sync flush), fixed Huffman codes (Z_FIXED), dynamic codes with literals only (Z_HUFFMAN_ONLY), run
copies (Z_RLE, distance 1 overlapping copies), codes longer than the 9-bit fast table (skewed byte frequencies),
several deflate blocks in one BGZF block, the 65536-byte ISIZE bound and the empty EOF block.
"""
import ctypes
import gzip
import os
import struct
import zlib

import numpy as np
import pytest

from helpers import gpu_vcf_bam, make_data
import pysynth
from ngsepcore_amd import GpuPileupSession, _lib

pytestmark = pytest.mark.gpu


def bgzf_block(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, flush_every=0):
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    if flush_every:
        c = b"".join(co.compress(data[i:i + flush_every]) + co.flush(zlib.Z_SYNC_FLUSH)
                     for i in range(0, len(data), flush_every)) + co.flush()
    else:
        c = co.compress(data) + co.flush()
    assert len(c) + 25 < 65536
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(c) + 25)
    return hdr + c + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def gpu_inflate(s, comp, cap=None):
    lib = s._lib
    n = len(comp)
    cap = (64 << 10) * max(1, n // 18 + 1) if cap is None else cap
    inb = (ctypes.c_uint8 * max(n, 1)).from_buffer_copy(comp or b"\0")
    outb = (ctypes.c_uint8 * max(cap, 1))()
    out_n = ctypes.c_int64(0)
    rc = lib.ngsep_bgzf_inflate(s._ctx, inb, n, outb, cap, ctypes.byref(out_n))
    return rc, bytes(outb[:out_n.value]) if rc == _lib.NGSEP_OK else out_n.value


def _payloads():
    rng = np.random.default_rng(11)
    text = b"".join(b"read%07d\tchr1\t%d\t60\t150M\tACGTTGCA" % (i, 1000 + 7 * i) for i in range(3000))
    skew = np.minimum(rng.geometric(0.08, 60000), 255).astype(np.uint8).tobytes()   # long codes (> 10 bits)
    return [
        ("zeros_max_isize", bytes(65536), 6, zlib.Z_DEFAULT_STRATEGY, 0),
        ("random_stored", rng.integers(0, 256, 65000, dtype=np.uint8).tobytes(), 6, zlib.Z_DEFAULT_STRATEGY, 0),
        ("level0_text", text[:60000], 0, zlib.Z_DEFAULT_STRATEGY, 0),
        ("fixed_codes", text[:65000], 6, zlib.Z_FIXED, 0),
        ("huffman_only", text[:65000], 6, zlib.Z_HUFFMAN_ONLY, 0),
        ("rle", bytes(rng.integers(0, 3, 4000, dtype=np.uint8).repeat(16)), 6, zlib.Z_RLE, 0),
        ("skewed_long_codes", skew, 9, zlib.Z_HUFFMAN_ONLY, 0),
        ("skewed_dynamic", skew, 1, zlib.Z_DEFAULT_STRATEGY, 0),
        ("sync_flushes", text[:64000], 6, zlib.Z_DEFAULT_STRATEGY, 5000),
        ("level9_text", text[:65280], 9, zlib.Z_DEFAULT_STRATEGY, 0),
        ("tiny", b"A", 6, zlib.Z_DEFAULT_STRATEGY, 0),
    ]


@pytest.fixture(scope="module")
def session():
    with GpuPileupSession() as s:
        yield s


@pytest.mark.parametrize("case", [p[0] for p in _payloads()])
def test_block_kinds_equal_zlib(session, case):
    name, data, level, strategy, fe = next(p for p in _payloads() if p[0] == case)
    comp = bgzf_block(data, level, strategy, fe)
    rc, got = gpu_inflate(session, comp)
    assert rc == _lib.NGSEP_OK, session._lib.ngsep_last_error(session._ctx).decode()
    assert got == data


def test_many_blocks_and_offsets(session):
    """Blocks of every size class back to back (unaligned input and output offsets), plus the EOF block."""
    rng = np.random.default_rng(3)
    datas, comp = [], b""
    for k in range(300):
        n = int(rng.integers(0, 65281))
        kind = k % 4
        if kind == 0:
            d = rng.integers(0, 4, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 2:
            d = bytes(rng.integers(65, 70, max(1, n // 8), dtype=np.uint8).repeat(8))[:n]
        else:
            d = (b"ACGT" * (n // 4 + 1))[:n]
        datas.append(d)
        comp += bgzf_block(d, int(rng.integers(0, 10)))
    comp += EOF_BLOCK
    rc, got = gpu_inflate(session, comp)
    assert rc == _lib.NGSEP_OK, session._lib.ngsep_last_error(session._ctx).decode()
    assert got == b"".join(datas)


def test_real_bam_equals_gzip(session, tmp_path):
    _, _, _, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=1, depth=8, seed=21)
    comp = open(bam, "rb").read()
    rc, got = gpu_inflate(session, comp)
    assert rc == _lib.NGSEP_OK, session._lib.ngsep_last_error(session._ctx).decode()
    assert got == gzip.decompress(comp)


def test_errors(session):
    good = bgzf_block(b"ACGT" * 1000)
    # an ISIZE the data does not inflate to
    bad = good[:-4] + struct.pack("<I", 4001)
    rc, _ = gpu_inflate(session, bad)
    assert rc == _lib.NGSEP_E_FORMAT
    # a cut block
    rc, _ = gpu_inflate(session, good[:-3])
    assert rc == _lib.NGSEP_E_FORMAT
    # invalid block type 3 in the deflate stream
    hdr_len = 18
    corrupt = bytearray(good)
    corrupt[hdr_len] = (corrupt[hdr_len] & ~0x6) | 0x6
    rc, _ = gpu_inflate(session, bytes(corrupt))
    assert rc == _lib.NGSEP_E_FORMAT
    # output too small: E_INVALID with the size needed
    rc, need = gpu_inflate(session, good, cap=100)
    assert rc == _lib.NGSEP_E_INVALID and need == 4000
    # nothing to do
    rc, got = gpu_inflate(session, b"", cap=0)
    assert rc == _lib.NGSEP_OK and got == b""


@pytest.mark.parametrize("read_bytes", [None, "100000", "4096"])
def test_bam_reader_device_inflate_vcf_identical(tmp_path, monkeypatch, read_bytes):
    """ngsep_call_bam with the device inflate (NGSEP_GPU_INFLATE) == the host inflate, whole reads and 100 kB reads
    (blocks cut across reads, many batches in flight); a 4 KB read request is raised to one whole BGZF block (a
    smaller buffer could never hold a 64 KB block: the reader looped on empty chunks)."""
    _, fa, _, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=2, contig_first=0, depth=25, seed=7,
                              secondary_rate=0.01, lowmq_rate=0.01, noqual_rate=0.005, softclip_rate=0.05, dup_rate=0.02)
    monkeypatch.delenv("NGSEP_GPU_INFLATE", raising=False)
    host, _ = gpu_vcf_bam(tmp_path, fa, bam, name="host")
    monkeypatch.setenv("NGSEP_GPU_INFLATE", "1")
    if read_bytes:
        monkeypatch.setenv("NGSEP_BGZF_READ", read_bytes)
    dev, _ = gpu_vcf_bam(tmp_path, fa, bam, name="dev")
    assert open(host).read() == open(dev).read()


@pytest.mark.parametrize("read_bytes", ["65536", "300000"])
def test_bam_reader_small_reads_vcf_identical(tmp_path, monkeypatch, read_bytes):
    """ngsep_call_bam (host inflate) with small file reads: many decoded chunks, the packed batches read in place from
    them and the chunks recycled only once no batch can still read them -- the VCF of whole 32 MB reads."""
    _, fa, _, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=2, contig_first=0, depth=25, seed=11,
                              softclip_rate=0.05, dup_rate=0.02, noqual_rate=0.005)
    monkeypatch.delenv("NGSEP_GPU_INFLATE", raising=False)
    whole, _ = gpu_vcf_bam(tmp_path, fa, bam, name="whole")
    monkeypatch.setenv("NGSEP_BGZF_READ", read_bytes)
    small, _ = gpu_vcf_bam(tmp_path, fa, bam, name="small")
    assert open(whole).read() == open(small).read()


def test_bam_reader_device_inflate_region(tmp_path, monkeypatch):
    """A region read (BAI seek) through the device inflate == the host inflate's."""
    _, fa, _, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=2, contig_first=0, depth=20, seed=9)
    opts = {"query_seq": "chrII", "query_first": 20000, "query_last": 150000}
    monkeypatch.delenv("NGSEP_GPU_INFLATE", raising=False)
    host, _ = gpu_vcf_bam(tmp_path, fa, bam, name="host", **opts)
    monkeypatch.setenv("NGSEP_GPU_INFLATE", "1")
    monkeypatch.setenv("NGSEP_BGZF_READ", "65536")
    dev, _ = gpu_vcf_bam(tmp_path, fa, bam, name="dev", **opts)
    assert open(host).read() == open(dev).read()
