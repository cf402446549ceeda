// inflate.hip -- BGZF block inflate on gfx950: the BAM reader's decompression (SAM spec 4.1, RFC 1951 DEFLATE)
// on the device, so the host threads keep the record decode, admission and projection (bam.cpp) to themselves.
//
// htsjdk's BlockCompressedInputStream plays this role in the reference (ReadAlignmentFileReader.java:171-183 opens
// the BAM through it); the reference inflates one 64 KB block at a time with java.util.zip.Inflater.  Here every
// BGZF block of a 32 MB read of the file is one workgroup of one wavefront (KZ, k_inflate):
//   - the block's last 16 KB of output live in an LDS ring, so most LZ77 copies never wait on memory (one from further
//     back, DEFLATE's distances reach 32 KB, reads the flushed bytes from HBM), and leave for HBM 8 KB at a time; ~20 KB
//     of LDS a wavefront -> 8 wavefronts a CU, 2048 blocks in flight on the chip;
//   - the bit stream is decoded as scalar code (the bit buffer, table entries and lengths in SGPRs: the decode is serial
//     by nature, and a vector decode costs 4 cycles an instruction for nothing), and the wavefront's 64 lanes split the
//     parallel parts: a Huffman table build (ballot ranks), an LZ77 copy (up to 64 bytes per instruction), a stored
//     block's copy and the 16-B flush of the finished block to HBM;
//   - the input arrives 16 B at a time, one group ahead (the decode never waits on a load it could have issued
//     earlier); Huffman codes of <= 9 bits (lit/len) / 7 bits (distance) take one LDS lookup, longer ones the
//     canonical walk from the 10th / 8th bit.
// The kernel is latency-bound (a dependent LDS lookup per symbol), not HBM-bound: its algorithmic traffic is the
// compressed bytes in plus the decoded bytes out, ~5.4 B per compressed byte on BAM data.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
#include "engine.hpp"

namespace ngsep {

constexpr int kZThreads = 64;
constexpr int kZLitBits = 9;                     // fast lit/len lookup bits
constexpr int kZDistBits = 7;                    // fast distance lookup bits (the code-length code's 7 bits too)
constexpr int kZOutMax = 65536;                  // BGZF ISIZE bound
constexpr size_t kZInSlack = 256;                // readable bytes past a batch's input (the one-group-ahead loads)

// one BGZF block: its raw deflate data in[in_off, in_off + in_len) -> out[out_off, out_off + isize)
struct ZBlock {
    uint64_t out_off;
    uint32_t in_off, in_len;
    uint32_t isize, pad;
};

// lit/len and distance table entries: bits 0-4 the code length (0: no fast entry), 5-6 the kind, 8-11 the extra
// bits, 16-31 the literal / length base / distance base
enum : uint32_t { kZLit = 0, kZLen = 1, kZEob = 2, kZBad = 3 };

__constant__ uint16_t kZLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59,
                                       67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kZLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kZDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                        1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kZDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kZClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ uint32_t z_lit_entry(uint32_t s, uint32_t len) {
    if (s < 256) return len | (kZLit << 5) | (s << 16);
    if (s == 256) return len | (kZEob << 5);
    if (s <= 285) return len | (kZLen << 5) | ((uint32_t)kZLenExtra[s - 257] << 8) | ((uint32_t)kZLenBase[s - 257] << 16);
    return len | (kZBad << 5);
}
__device__ __forceinline__ uint32_t z_dist_entry(uint32_t s, uint32_t len) {
    if (s < 30) return len | ((uint32_t)kZDistExtra[s] << 8) | ((uint32_t)kZDistBase[s] << 16);
    return len | (kZBad << 5);
}

// one Huffman code's canonical description in LDS (RFC 1951 3.2.2): per length its count, first code and first index
// into the symbols sorted by (length, symbol) -- the walk for codes longer than the fast table
template <int NSYM>
struct ZHuff {
    uint16_t count[16], first[16], offs[16];
    uint16_t sym[NSYM];
};

// the output window: the last 16 KB in an LDS ring, flushed to HBM 8 KB at a time; a copy from further back (DEFLATE
// allows 32 KB) reads the flushed bytes from HBM.  ~20 KB of LDS a wavefront: 8 resident a CU.
constexpr uint32_t kZRing = 16384;
constexpr uint32_t kZFlush = 8192;
static_assert(kZRing >= kZFlush + 2 * 258, "a copy never overwrites unflushed ring bytes");

struct ZLds {
    uint8_t ring[kZRing];                        // output byte x of the block at ring[(x + (out_off & 15)) % kZRing]
    uint32_t lit[1 << kZLitBits];
    uint32_t dist[1 << kZDistBits];              // (while a block's code lengths are read: the code-length code's table)
    ZHuff<288> hl;
    ZHuff<32> hd;                                // (the code-length code's 19 symbols first, then the distances')
    uint8_t lens[320];                           // code lengths being built (HLIT + HDIST <= 320)
};
static_assert(sizeof(ZLds) <= 20480, "8 wavefronts a CU");

// wavefront-uniform values live in scalar registers: every LDS / memory value the decode branches on is read into
// one (the decode is then scalar code; only the copies and the table builds use the lanes)
__device__ __forceinline__ uint32_t z_u(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t z_u64(uint64_t v) { return ((uint64_t)z_u((uint32_t)(v >> 32)) << 32) | z_u((uint32_t)v); }

// the wavefront's shared bit reader: 16-B groups of the block's input, one group ahead
struct ZBits {
    const uint4* ip;                             // the next group to load
    const uint4* ip_end;                         // no load at or past this group
    uint4 q, nq;                                 // current group, next group
    int k;                                       // next word of q
    int64_t wpos;                                // absolute index of the next word to take
    uint64_t buf;                                // unconsumed bits, LSB first
    int cnt;
};

__device__ __forceinline__ uint4 z_load(const ZBits& b, const uint4* p) {
    if (p >= b.ip_end) return make_uint4(0, 0, 0, 0);
    const uint4 v = *p;
    return make_uint4(z_u(v.x), z_u(v.y), z_u(v.z), z_u(v.w));
}
__device__ __forceinline__ uint32_t z_take(ZBits& b) {
    const uint32_t w = b.k == 0 ? b.q.x : b.k == 1 ? b.q.y : b.k == 2 ? b.q.z : b.q.w;
    b.wpos++;
    if (++b.k == 4) {
        b.q = b.nq;
        b.nq = z_load(b, b.ip);
        b.ip++;
        b.k = 0;
    }
    return w;
}
// positions the reader at byte `start` of in (in is 16-B aligned; loads stop at in + lim)
__device__ __forceinline__ void z_init(ZBits& b, const uint8_t* in, uint64_t start, uint64_t lim) {
    const uint4* g = (const uint4*)(in + (start & ~(uint64_t)15));
    b.ip_end = (const uint4*)(in + ((lim + 15) & ~(uint64_t)15));
    b.q = z_load(b, g);
    b.nq = z_load(b, g + 1);
    b.ip = g + 2;
    b.k = (int)((start & 15) >> 2);
    b.wpos = (int64_t)(start >> 2);
    const int sh = (int)(start & 3) * 8;
    b.buf = (uint64_t)(z_take(b) >> sh);
    b.cnt = 32 - sh;
}
__device__ __forceinline__ void z_refill(ZBits& b) {
    // (the reader's state restated as uniform: the compiler's divergence analysis loses it across the lane loops)
    b.buf = z_u64(b.buf);
    b.cnt = (int)z_u((uint32_t)b.cnt);
    b.k = (int)z_u((uint32_t)b.k);
    b.wpos = (int64_t)z_u64((uint64_t)b.wpos);
    b.ip = (const uint4*)z_u64((uint64_t)b.ip);
    if (b.cnt <= 32) {
        b.buf |= (uint64_t)z_take(b) << b.cnt;
        b.cnt += 32;
    }
}
__device__ __forceinline__ uint32_t z_bits(ZBits& b, int n) {      // n <= 32 bits, cnt >= n
    const uint32_t v = (uint32_t)b.buf & (uint32_t)(((uint64_t)1 << n) - 1);
    b.buf >>= n;
    b.cnt -= n;
    return v;
}
// the absolute byte offset of the next unconsumed bit's byte (cnt a multiple of 8)
__device__ __forceinline__ uint64_t z_byte_pos(const ZBits& b) { return (uint64_t)b.wpos * 4 - (uint64_t)(b.cnt >> 3); }

// builds a code's tables from lens[0, n) (lengths <= 15): the canonical (count, sym) arrays of h and the fast table
// tab[1 << fb] (codes of <= fb bits; longer codes leave their prefix's entry 0).  MODE: kZModeLit lit/len entries,
// kZModeDist distance entries, kZModeRaw the symbol itself (bits 16-31; the code-length code).  Returns false for an
// over-subscribed code.  Whole wavefront; the tables are read after its closing barrier.
enum { kZModeRaw = 0, kZModeLit = 1, kZModeDist = 2 };
template <int MODE, class H>
__device__ __attribute__((noinline)) bool z_build(const uint8_t* lens, int n, H& h, uint32_t* tab, int fb) {
    const int lane = (int)threadIdx.x;
    for (int i0 = 0; i0 < (1 << fb); i0 += kZThreads)
        if (i0 + lane < (1 << fb)) tab[i0 + lane] = 0;
    if (lane < 16) h.count[lane] = 0;
    __syncthreads();
    // counts per length (lane l of the wavefront holds length l's: ballots over 64-symbol chunks)
    uint32_t cntv = 0;
    for (int c = 0; c < n; c += kZThreads) {
        const int s = c + lane;
        const int v = s < n ? lens[s] : 0;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            const uint32_t k = (uint32_t)__popcll(__ballot(v == l));
            if (lane == l) cntv += k;
        }
    }
    if (lane > 0 && lane < 16) h.count[lane] = (uint16_t)cntv;
    __syncthreads();
    // the first code and the first sorted index of every length (lane l keeps length l's); over-subscription check
    int left = 1;
    uint32_t code = 0, off = 0, firstv = 0, offv = 0;
    bool ok = true;
    for (int l = 1; l < 16; l++) {
        const uint32_t c = h.count[l];
        left = left * 2 - (int)c;
        if (left < 0) ok = false;
        if (lane == l) { firstv = code; offv = off; }
        code = (code + c) << 1;
        off += c;
    }
    if (lane > 0 && lane < 16) { h.first[lane] = (uint16_t)firstv; h.offs[lane] = (uint16_t)offv; }
    // ranks within a length (symbol order), codes, sorted symbols and fast entries
    uint32_t runv = 0;                                   // lane l: length-l symbols in earlier chunks
    const uint64_t lt = (((uint64_t)1) << lane) - 1;
    for (int c = 0; c < n; c += kZThreads) {
        const int s = c + lane;
        const int v = s < n ? lens[s] : 0;
        const uint32_t base = (uint32_t)__shfl((int)runv, v);
        const uint32_t f = (uint32_t)__shfl((int)firstv, v), o = (uint32_t)__shfl((int)offv, v);
        uint32_t rank = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            const uint64_t m = __ballot(v == l);
            if (v == l) rank = base + (uint32_t)__popcll(m & lt);
            if (lane == l) runv += (uint32_t)__popcll(m);
        }
        if (v > 0) {
            h.sym[o + rank] = (uint16_t)s;
            if (v <= fb) {
                const uint32_t rev = __brev(f + rank) >> (32 - v);
                const uint32_t e = MODE == kZModeLit ? z_lit_entry((uint32_t)s, (uint32_t)v)
                                 : MODE == kZModeDist ? z_dist_entry((uint32_t)s, (uint32_t)v)
                                                      : ((uint32_t)v | ((uint32_t)s << 16));
                for (uint32_t i = rev; i < (1u << fb); i += (1u << v)) tab[i] = e;
            }
        }
    }
    __syncthreads();
    return ok;
}

// canonical walk for a code longer than the fast table's fb bits (no fast entry: its length is > fb): the code's bits
// MSB first, length by length from fb + 1 against (first, count); the symbol, or -1 for a bit string that is no code;
// consumes its bits
template <class H>
__device__ __forceinline__ int z_slow(ZBits& b, const H& h, int fb) {
    uint32_t code = __brev((uint32_t)b.buf & ((1u << fb) - 1u)) >> (32 - fb);
#pragma unroll 1
    for (int l = fb + 1; l < 16; l++) {
        code = (code << 1) | (uint32_t)((b.buf >> (l - 1)) & 1u);
        const uint32_t c = z_u(h.count[l]), f = z_u(h.first[l]);
        if (code - f < c) {
            b.buf >>= l;
            b.cnt -= l;
            return (int)z_u(h.sym[z_u(h.offs[l]) + code - f]);
        }
    }
    return -1;
}

// writes output bytes [a, e) of the block from the ring to HBM: whole 16-B groups as such, the partial groups at
// the ends byte by byte (their other bytes belong to the neighbouring blocks / flushes)
__device__ __forceinline__ void z_flush(const ZLds& L, uint8_t* __restrict__ out, uint64_t out_off, uint32_t ab, uint32_t a, uint32_t e) {
    if (a >= e) return;
    const int lane = (int)threadIdx.x;
    const uint64_t lo = out_off + a, hi = out_off + e;
    const uint64_t g0 = lo >> 4, g1 = (hi - 1) >> 4;
    for (uint64_t gb = g0; gb <= g1; gb += kZThreads) {
        const uint64_t g = gb + (uint64_t)lane;
        if (g > g1) continue;
        const uint64_t ga = g * 16;
        if (ga >= lo && ga + 16 <= hi) {
            const uint32_t r = (uint32_t)(ga - out_off + ab) & (kZRing - 1);
            *reinterpret_cast<uint4*>(out + ga) = *reinterpret_cast<const uint4*>(L.ring + r);
        } else {
            for (uint64_t x = ga < lo ? lo : ga; x < (ga + 16 < hi ? ga + 16 : hi); x++)
                out[x] = L.ring[(uint32_t)(x - out_off + ab) & (kZRing - 1)];
        }
    }
}

// KZ: one wavefront per BGZF block (grid = blocks).  err[0] counts the blocks that failed (corrupt data, a size
// other than ISIZE); err[1] the first of them + 1.
__global__ void __launch_bounds__(kZThreads)
k_inflate(const uint8_t* __restrict__ in, uint64_t in_n, const ZBlock* __restrict__ blocks, int64_t nb,
          uint8_t* __restrict__ out, unsigned long long* __restrict__ err) {
    extern __shared__ __align__(16) uint8_t z_smem[];
    ZLds& L = *reinterpret_cast<ZLds*>(z_smem);
    const int64_t bi = blockIdx.x;
    if (bi >= nb) return;
    const int lane = (int)threadIdx.x;
    const ZBlock blk = blocks[bi];
    const uint64_t out_off = ((uint64_t)z_u((uint32_t)(blk.out_off >> 32)) << 32) | z_u((uint32_t)blk.out_off);
    const uint32_t in_off = z_u(blk.in_off), in_len = z_u(blk.in_len), isize = z_u(blk.isize);
    const uint32_t ab = (uint32_t)(out_off & 15);
    constexpr uint32_t M = kZRing - 1;
    bool bad = isize > (uint32_t)kZOutMax;
    uint32_t pos = 0, flushed = 0;
    if (!bad && in_len > 0) {
        ZBits b;
        const uint64_t lim = (uint64_t)in_off + in_len + 64 < in_n + kZInSlack ? (uint64_t)in_off + in_len + 64 : in_n + kZInSlack;
        z_init(b, in, in_off, lim);
        const int64_t wlim = (int64_t)(((uint64_t)in_off + in_len + 16) >> 2);
        bool last = false;
        while (!last && !bad) {
            z_refill(b);
            if (b.wpos > wlim + 4) { bad = true; break; }
            last = z_bits(b, 1) != 0;
            const uint32_t type = z_bits(b, 2);
            if (type == 0) {                                   // stored
                z_bits(b, b.cnt & 7);
                z_refill(b);
                const uint32_t ln = z_bits(b, 16), nln = z_bits(b, 16);
                if ((ln ^ 0xFFFFu) != nln || pos + ln > isize) { bad = true; break; }
                const uint64_t src = z_byte_pos(b);
                if (src + ln > (uint64_t)in_off + in_len) { bad = true; break; }
                for (uint32_t c0 = 0; c0 < ln; c0 += kZFlush) {    // (pieces: the ring holds a flush's worth ahead)
                    const uint32_t c1 = c0 + kZFlush < ln ? c0 + kZFlush : ln;
                    for (uint32_t j0 = c0; j0 < c1; j0 += kZThreads) {
                        const uint32_t j = j0 + (uint32_t)lane;
                        if (j < c1) L.ring[(pos + j + ab) & M] = in[src + j];
                    }
                    __syncthreads();
                    while (pos + c1 - flushed >= kZFlush) {
                        z_flush(L, out, out_off, ab, flushed, flushed + kZFlush);
                        flushed += kZFlush;
                    }
                    __threadfence_block();
                }
                pos += ln;
                z_init(b, in, src + ln, lim);
                continue;
            }
            if (type == 3) { bad = true; break; }
            if (type == 1) {                                   // fixed codes
                for (int s0 = 0; s0 < 320; s0 += kZThreads) {
                    const int s = s0 + lane;
                    L.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
                }
                __syncthreads();
                z_build<kZModeLit>(L.lens, 288, L.hl, L.lit, kZLitBits);
                z_build<kZModeDist>(L.lens + 288, 30, L.hd, L.dist, kZDistBits);
            } else {                                           // dynamic codes
                z_refill(b);
                const int hlit = (int)z_bits(b, 5) + 257, hdist = (int)z_bits(b, 5) + 1, hclen = (int)z_bits(b, 4) + 4;
                if (hlit > 286 || hdist > 30) { bad = true; break; }
                // the code-length code's 19 lengths, 3 bits each, in kZClenOrder
                if (lane < 19) L.lens[lane] = 0;
                __syncthreads();
                uint32_t cl = 0;
                for (int i = 0; i < hclen; i++) {
                    z_refill(b);
                    const uint32_t v = z_bits(b, 3);
                    if (lane == i) cl = v;
                }
                if (lane < hclen) L.lens[kZClenOrder[lane]] = (uint8_t)cl;
                __syncthreads();
                if (!z_u((uint32_t)z_build<kZModeRaw>(L.lens, 19, L.hd, L.dist, 7))) { bad = true; break; }
                // the lit/len and distance lengths (run-length coded by the code-length code)
                const int total = hlit + hdist;
                int i = 0, prev = 0;
                while (i < total) {
                    z_refill(b);
                    const uint32_t e = z_u(L.dist[(uint32_t)b.buf & 127u]);
                    const int ln = (int)(e & 31);
                    if (ln == 0) { bad = true; break; }
                    b.buf >>= ln;
                    b.cnt -= ln;
                    const int sym = (int)(e >> 16);
                    int rep = 0, val = 0;
                    if (sym < 16) { val = sym; rep = 1; prev = sym; }
                    else if (sym == 16) { if (i == 0) { bad = true; break; } val = prev; rep = 3 + (int)z_bits(b, 2); }
                    else if (sym == 17) { val = 0; rep = 3 + (int)z_bits(b, 3); prev = 0; }
                    else { val = 0; rep = 11 + (int)z_bits(b, 7); prev = 0; }
                    if (i + rep > total) { bad = true; break; }
                    for (int j0 = 0; j0 < rep; j0 += kZThreads)
                        if (j0 + lane < rep) L.lens[i + j0 + lane] = (uint8_t)val;
                    i += rep;
                }
                if (bad) break;
                __syncthreads();
                if (z_u(L.lens[256]) == 0) { bad = true; break; }
                if (!z_u((uint32_t)z_build<kZModeDist>(L.lens + hlit, hdist, L.hd, L.dist, kZDistBits))) { bad = true; break; }
                if (!z_u((uint32_t)z_build<kZModeLit>(L.lens, hlit, L.hl, L.lit, kZLitBits))) { bad = true; break; }
            }
            // the block's symbols (scalar decode; a literal is one lane's LDS byte, a copy up to 64 lanes' bytes)
            while (true) {
                pos = z_u(pos);
                flushed = z_u(flushed);
                z_refill(b);
                uint32_t e = z_u(L.lit[(uint32_t)b.buf & ((1u << kZLitBits) - 1)]);
                if ((e & 31) == 0) {
                    const int s = z_slow(b, L.hl, kZLitBits);
                    if (s < 0) { bad = true; break; }
                    e = z_u(z_lit_entry((uint32_t)s, 0));
                } else {
                    b.buf >>= (e & 31);
                    b.cnt -= (int)(e & 31);
                }
                const uint32_t kind = (e >> 5) & 3;
                if (kind == kZLit) {
                    if (pos >= isize) { bad = true; break; }
                    if (lane == 0) L.ring[(pos + ab) & M] = (uint8_t)(e >> 16);
                    pos++;
                } else {
                    if (kind == kZEob) break;
                    if (kind == kZBad) { bad = true; break; }
                    const uint32_t len = (e >> 16) + z_bits(b, (int)((e >> 8) & 15));
                    z_refill(b);
                    uint32_t d = z_u(L.dist[(uint32_t)b.buf & ((1u << kZDistBits) - 1)]);
                    if ((d & 31) == 0) {
                        const int s = z_slow(b, L.hd, kZDistBits);
                        if (s < 0) { bad = true; break; }
                        d = z_u(z_dist_entry((uint32_t)s, 0));
                    } else {
                        b.buf >>= (d & 31);
                        b.cnt -= (int)(d & 31);
                    }
                    if ((d >> 5) & 3) { bad = true; break; }
                    const uint32_t dist = (d >> 16) + z_bits(b, (int)((d >> 8) & 15));
                    if (dist > pos || pos + len > isize) { bad = true; break; }
                    // (uniform trip counts, the lanes past len idle: a lane-bounded loop would make the decode state
                    // look divergent to the compiler)
                    if (dist > kZRing) {                 // further back than the ring: the flushed bytes in HBM
                        const uint8_t* src = out + out_off + pos - dist;
                        for (uint32_t j0 = 0; j0 < len; j0 += kZThreads) {
                            const uint32_t j = j0 + (uint32_t)lane;
                            if (j < len) L.ring[(pos + j + ab) & M] = src[j];
                        }
                    } else if (dist >= len) {
                        for (uint32_t j0 = 0; j0 < len; j0 += kZThreads) {
                            const uint32_t j = j0 + (uint32_t)lane;
                            if (j < len) L.ring[(pos + j + ab) & M] = L.ring[(pos - dist + j + ab) & M];
                        }
                    } else {
                        for (uint32_t j0 = 0; j0 < len; j0 += kZThreads) {
                            const uint32_t j = j0 + (uint32_t)lane;
                            if (j < len) L.ring[(pos + j + ab) & M] = L.ring[(pos - dist + j % dist + ab) & M];
                        }
                    }
                    pos += len;
                }
                if (pos - flushed >= kZFlush) {
                    __syncthreads();
                    z_flush(L, out, out_off, ab, flushed, flushed + kZFlush);
                    flushed += kZFlush;
                    __threadfence_block();               // (the flushed bytes visible to this wavefront's far copies)
                }
            }
            __syncthreads();
        }
    }
    if (!bad && pos != isize) bad = true;
    if (bad) {
        if (lane == 0) {
            atomicAdd(err, 1ull);
            atomicMin(err + 1, (unsigned long long)bi + 1);
        }
        return;
    }
    __syncthreads();
    z_flush(L, out, out_off, ab, flushed, isize);
}

// ---- host side ----

// two slots, each with its own stream and buffers: a batch's copies and kernel run while the caller reads the next
struct GzSlot {
    hipStream_t stream = nullptr;
    uint8_t* d_in = nullptr;
    size_t cap_in = 0;
    uint8_t* d_out = nullptr;
    size_t cap_out = 0;
    ZBlock* d_blk = nullptr;
    size_t cap_blk = 0;
    unsigned long long* d_err = nullptr;
    unsigned long long* h_err = nullptr;         // pinned
    std::vector<ZBlock> h_blk;
    bool busy = false;
};
struct GzDevice {
    int ordinal = 0;
    int wave_blocks = 2048;                      // KZ workgroups resident at once (CUs x workgroups a CU)
    GzSlot slot[2];
};

#define GZ_TRY(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);                   \
            return -1;                                                                 \
        }                                                                              \
    } while (0)

GzDevice* gz_create(int ordinal, std::string& err) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        err = "no HIP device available (libngsep_amd requires an MI355X / gfx950 GPU)";
        return nullptr;
    }
    if (ordinal < 0 || ordinal >= n) { err = "device ordinal out of range"; return nullptr; }
    if (hipSetDevice(ordinal) != hipSuccess) { err = "hipSetDevice failed"; return nullptr; }
    GzDevice* d = new GzDevice();
    d->ordinal = ordinal;
    for (GzSlot& s : d->slot)
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&s.d_err, 2 * sizeof(unsigned long long)) != hipSuccess ||
            hipHostMalloc(&s.h_err, 2 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
            err = "inflate device setup failed";
            gz_destroy(d);
            return nullptr;
        }
    // (> 64 KB of dynamic LDS: a launch the runtime refuses is reported by gz_wait)
    (void)hipFuncSetAttribute((const void*)k_inflate, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(ZLds));
    hipDeviceProp_t prop;
    int per_cu = 0;
    if (hipGetDeviceProperties(&prop, ordinal) == hipSuccess && prop.multiProcessorCount > 0 &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_inflate, kZThreads, sizeof(ZLds)) == hipSuccess && per_cu > 0)
        d->wave_blocks = prop.multiProcessorCount * per_cu;
    return d;
}

void gz_destroy(GzDevice* d) {
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    for (GzSlot& s : d->slot) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        (void)hipFree(s.d_in);
        (void)hipFree(s.d_out);
        (void)hipFree(s.d_blk);
        (void)hipFree(s.d_err);
        if (s.h_err) (void)hipHostFree(s.h_err);
        if (s.stream) (void)hipStreamDestroy(s.stream);
    }
    delete d;
}

// BGZF blocks one KZ launch runs at once: a batch of at most this many takes one block's latency (a few more would
// take two)
int gz_wave_blocks(const GzDevice* d) { return d ? d->wave_blocks : 2048; }

void* gz_host_alloc(size_t n) {
    void* p = nullptr;
    return hipHostMalloc(&p, n, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}
void gz_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// enqueues the inflate of nb BGZF blocks (raw deflate data at in[boff[k], + bclen[k]) -> out[dout[k], + bisize[k])) on
// slot `sl`: H2D of in[0, in_n), KZ, D2H of out[0, out_n).  in and out stay untouched by the caller until gz_wait
// (pinned buffers copy at the link's rate).
int gz_submit(GzDevice* d, int sl, const uint8_t* in, size_t in_n, const size_t* boff, const size_t* bclen,
              const uint32_t* bisize, const size_t* dout, size_t nb, uint8_t* out, size_t out_n, std::string& err) {
    GzSlot& s = d->slot[sl];
    if (s.busy) { err = "inflate slot in use"; return -1; }
    if (nb == 0) return 0;
    if (in_n >= ((size_t)1 << 32)) { err = "inflate batch too large"; return -1; }
    GZ_TRY(hipSetDevice(d->ordinal));
    if (in_n + kZInSlack > s.cap_in) {
        (void)hipFree(s.d_in);
        s.d_in = nullptr;
        s.cap_in = in_n + kZInSlack + (in_n >> 3);
        GZ_TRY(hipMalloc(&s.d_in, s.cap_in));
        GZ_TRY(hipMemsetAsync(s.d_in, 0, s.cap_in, s.stream));
    }
    if (out_n > s.cap_out) {
        (void)hipFree(s.d_out);
        s.d_out = nullptr;
        s.cap_out = out_n + (out_n >> 3);
        GZ_TRY(hipMalloc(&s.d_out, s.cap_out));
    }
    if (nb > s.cap_blk) {
        (void)hipFree(s.d_blk);
        s.d_blk = nullptr;
        s.cap_blk = nb + (nb >> 2) + 64;
        GZ_TRY(hipMalloc(&s.d_blk, s.cap_blk * sizeof(ZBlock)));
    }
    s.h_blk.resize(nb);
    for (size_t k = 0; k < nb; k++) {
        if (bisize[k] > (uint32_t)kZOutMax || dout[k] + bisize[k] > out_n || boff[k] + bclen[k] > in_n) {
            err = "BGZF block outside its batch";
            return -1;
        }
        s.h_blk[k] = ZBlock{(uint64_t)dout[k], (uint32_t)boff[k], (uint32_t)bclen[k], bisize[k], 0};
    }
    GZ_TRY(hipMemcpyAsync(s.d_in, in, in_n, hipMemcpyHostToDevice, s.stream));
    GZ_TRY(hipMemcpyAsync(s.d_blk, s.h_blk.data(), nb * sizeof(ZBlock), hipMemcpyHostToDevice, s.stream));
    GZ_TRY(hipMemsetAsync(s.d_err, 0, sizeof(unsigned long long), s.stream));
    GZ_TRY(hipMemsetAsync(s.d_err + 1, 0xFF, sizeof(unsigned long long), s.stream));
    hipLaunchKernelGGL(k_inflate, dim3((unsigned)nb), dim3(kZThreads), sizeof(ZLds), s.stream, (const uint8_t*)s.d_in,
                       (uint64_t)in_n, (const ZBlock*)s.d_blk, (int64_t)nb, s.d_out, s.d_err);
    GZ_TRY(hipGetLastError());
    GZ_TRY(hipMemcpyAsync(s.h_err, s.d_err, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s.stream));
    GZ_TRY(hipMemcpyAsync(out, s.d_out, out_n, hipMemcpyDeviceToHost, s.stream));
    s.busy = true;
    return 0;
}

// waits for slot sl's batch; -1 (err set) when a block failed to inflate to its ISIZE
int gz_wait(GzDevice* d, int sl, std::string& err) {
    GzSlot& s = d->slot[sl];
    if (!s.busy) return 0;
    s.busy = false;
    GZ_TRY(hipSetDevice(d->ordinal));
    GZ_TRY(hipStreamSynchronize(s.stream));
    if (s.h_err[0]) {
        err = "BGZF inflate failed (block " + std::to_string((long long)s.h_err[1] - 1) + " of the batch)";
        return -1;
    }
    return 0;
}

}  // namespace ngsep
