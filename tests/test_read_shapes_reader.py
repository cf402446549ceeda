"""The C++ BAM reader on the read shapes real BAMs carry (tests/read_shapes.py: paired-end flags, overlapping mates,
mixed lengths incl. 5-20 kb reads, hard clips, '=' / 'X' / 'N' / 'P' CIGAR ops, duplicate / QC-fail / supplementary /
secondary records, NH tags, SEQ '*', repeated records, unmapped mates) against a Python restatement of htsjdk +
ReadAlignmentFileReader.loadAlignment's view of the same SAM text (ReadAlignmentFileReader.java:219-354, filters of
AlignmentsPileupGenerator.createReader :363-373, ReadAlignment.setCigarString :1222-1266 with collapseEqualEvents).

Also a BAM record with an invalid CIGAR op code (9-15): htsjdk's CigarOperator.binaryToEnum throws for it, the
reader's loadAlignment catches the RuntimeException, logs a warning and skips the record (:340-347) -- the C++ reader
skips it the same way.  CPU only (no device call)."""
import gzip
import os
import struct
import zlib

import pytest

import pysynth
import read_shapes
from test_bam_reader import _ctx, _read_all

OPS = "HDIMPNSX"                                   # NGSEP op codes (ReadAlignment.java:60-69)


def _fasta(path):
    out, name, buf = [], None, []
    for l in open(path):
        l = l.rstrip("\n")
        if l.startswith(">"):
            if name:
                out.append((name, "".join(buf).encode()))
            name, buf = l[1:].split()[0], []
        else:
            buf.append(l)
    if name:
        out.append((name, "".join(buf).encode()))
    return out


def expected_view(sam, min_mq=20):
    """(seq_id, first, flags, rg, cigar codes, bases, quals, has_quals) of every record the reference's reader hands
    to the pileup generator, in file order"""
    seqs, rgs, out = [], [], []
    last = None
    for l in open(sam):
        l = l.rstrip("\n")
        if l.startswith("@SQ"):
            seqs.append(dict(kv.split(":", 1) for kv in l.split("\t")[1:])["SN"])
            continue
        if l.startswith("@RG"):
            rgs.append(dict(kv.split(":", 1) for kv in l.split("\t")[1:])["ID"])
            continue
        if l.startswith("@"):
            continue
        f = l.split("\t")
        name, flag, pos = f[0], int(f[1]), int(f[3])
        paired, fop = bool(flag & 1), bool(flag & 0x40)
        key = (name, pos, paired, fop if paired else None)
        if last is not None and key == last:       # isSameAlignment (:292-306): lastRecord kept
            continue
        last = key
        tags = dict((t[:2], t[5:]) for t in f[11:])
        nh = int(tags["NH"]) if "NH" in tags else None
        multiple = bool(flag & 0x100) or (nh is not None and nh > 1) or (nh is None and int(f[4]) < min_mq)
        flags = flag | (0x1000 if multiple else 0)
        if flags & (0x4 | 0x100 | 0x1000):           # unmapped, secondary, multiple
            continue
        if f[2] not in seqs or f[5] == "*":
            continue
        codes, n = [], 0
        for ch in f[5]:
            if ch.isdigit():
                n = n * 10 + int(ch)
                continue
            op = 3 if ch == "=" else OPS.index(ch)
            if codes and codes[-1] & 7 == op:
                codes[-1] += n * 8
            else:
                codes.append(n * 8 + op)
            n = 0
        read_len = sum(c // 8 for c in codes if c & 2)
        bases = b"" if f[9] == "*" else f[9].upper().encode()
        if bases and len(bases) != read_len:       # setReadCharacters throws
            continue
        hq = 0 if f[10] == "*" or not bases else 1
        quals = f[10].encode() if hq else b"*"
        out.append((seqs.index(f[2]), pos, flags, rgs.index(tags["RG"]) if tags.get("RG") in rgs else -1, tuple(codes),
                    bases, quals, hq))
    return out


@pytest.mark.parametrize("seed,n_samples,batch", [(1, 1, 1 << 20), (3, 3, 3000)])
def test_reader_on_real_read_shapes(tmp_path, seed, n_samples, batch):
    d = str(tmp_path)
    sam, fa = os.path.join(d, "s.sam"), os.path.join(d, "s.fa")
    read_shapes.make_sam(sam, fa, seed=seed, n_samples=n_samples, depth=8 if n_samples == 1 else 4,
                         lengths=(30000, 12000))
    st = read_shapes.shape_stats(sam)
    for k in ("paired", "overlap", "eqx", "hard", "skip", "pad", "long", "dup", "qcfail", "supp", "secondary",
              "mate_other", "mate_unmapped", "seq_star"):
        assert st[k] > 0, k
    bam = pysynth.sam_to_bam(sam, os.path.join(d, "s.bam"))
    want = expected_view(sam)
    lib, ctx = _ctx(_fasta(fa))
    got = _read_all(lib, ctx, bam, batch)
    lib.ngsep_close(ctx)
    got = [(r[0], r[1], r[2] & ~0x2000, r[3], r[4], r[5], r[6] if r[7] else b"*", r[7]) for r in got]
    assert len(got) == len(want) > 500
    for k, (a, b) in enumerate(zip(got, want)):
        assert a == b, (k, a[:5], b[:5])


# ---- a BAM with one record's CIGAR op code set to 9 (invalid) -------------------------------------------------------
def _bgzf(data: bytes) -> bytes:
    out = []
    for i in range(0, len(data), 65280):
        chunk = data[i:i + 65280]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        z = c.compress(chunk) + c.flush()
        out.append(b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", len(z) + 25) + z +
                   struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def _records_of(raw: bytes):
    """offsets of the records of an uncompressed BAM stream"""
    (lt,) = struct.unpack_from("<i", raw, 4)
    p = 8 + lt
    (nref,) = struct.unpack_from("<i", raw, p)
    p += 4
    for _ in range(nref):
        (ln,) = struct.unpack_from("<i", raw, p)
        p += 8 + ln
    offs = []
    while p < len(raw):
        (bs,) = struct.unpack_from("<i", raw, p)
        offs.append(p)
        p += 4 + bs
    return offs


def test_invalid_cigar_op_record_skipped(tmp_path):
    d = str(tmp_path)
    sam, fa = os.path.join(d, "s.sam"), os.path.join(d, "s.fa")
    read_shapes.make_sam(sam, fa, seed=5, depth=4, lengths=(20000,), long_frac=0.0)
    bam = pysynth.sam_to_bam(sam, os.path.join(d, "s.bam"))
    raw = bytearray(gzip.open(bam, "rb").read())
    offs = _records_of(bytes(raw))
    lib, ctx = _ctx(_fasta(fa))
    base = _read_all(lib, ctx, bam)
    # the 100th plain record: its first op code becomes 9 (BAM ops are 0-8, "MIDNSHP=X")
    def plain(i):                                   # a kept record: mapped, primary, MAPQ 60, not a repeat
        o = offs[i]
        n_cig, flag = struct.unpack_from("<HH", raw, o + 4 + 12)
        name = raw[o + 36:o + 36 + raw[o + 12] - 1]
        prev = offs[i - 1]
        return n_cig > 0 and not flag & 0x104 and raw[o + 13] == 60 and name != raw[prev + 36:prev + 36 + raw[prev + 12] - 1]
    k = offs[[i for i in range(1, len(offs)) if plain(i)][100]]
    l_name = raw[k + 4 + 8]
    c0 = k + 4 + 32 + l_name
    (v,) = struct.unpack_from("<I", raw, c0)
    struct.pack_into("<I", raw, c0, (v & ~15) | 9)
    bad = os.path.join(d, "bad.bam")
    open(bad, "wb").write(_bgzf(bytes(raw)))
    got = _read_all(lib, ctx, bad)
    lib.ngsep_close(ctx)
    assert len(got) == len(base) - 1
    # exactly that record is missing (its position and CIGAR identify it among the kept ones)
    pos = struct.unpack_from("<i", raw, k + 4 + 4)[0] + 1
    missing = [r for r in base if r not in got]
    assert len(missing) == 1 and missing[0][1] == pos
