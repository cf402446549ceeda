// Host timing of the indel realigner's region replay (realign.cpp replay_region) on synthetic regions: 30x 150 bp reads
// around a 3-base deletion carried by half of them.  Build: make -C tools/replay_bench (PROF=1: gprof build).
#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../ngsepcore_amd/csrc/realign.hpp"

using namespace ngsep;

int main(int argc, char** argv) {
    const int n_regions = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int depth = argc > 2 ? std::atoi(argv[2]) : 30;
    std::mt19937_64 rng(7);
    const int L = 400000;
    std::string seq(L, 'A');
    const char* B = "ACGT";
    for (auto& c : seq) c = B[rng() & 3];
    RealignParams rp;
    double total_ms = 0;
    long long positions = 0, calls = 0;
    for (int k = 0; k < n_regions; k++) {
        const int X = 2000 + (int)(rng() % (uint64_t)(L - 4000));
        // reads starting in [X - 600, X + 300], depth / 150 per position
        std::vector<RawRead> reads;
        auto blk = std::make_shared<RawBlock>();
        const int nreads = 900 * depth / 150;
        blk->bytes.reset(new char[(size_t)nreads * (12 + 300)]);
        char* at = blk->bytes.get();
        std::vector<int> starts;
        for (int i = 0; i < nreads; i++) starts.push_back(X - 600 + (int)(rng() % 900));
        std::sort(starts.begin(), starts.end());
        for (int i = 0; i < nreads; i++) {
            RawRead r;
            const int f = starts[(size_t)i];
            const bool del = (rng() & 1) && f < X - 10 && f + 150 > X + 10;
            int32_t* ops = reinterpret_cast<int32_t*>(at);
            char* ch = at + 12;
            char* qu = ch + 150;
            at += 12 + 300;
            if (del) {
                const int a = X - f;                          // M bases before the deletion
                ops[0] = a * 8 + 3;                           // M: ref + read
                ops[1] = 3 * 8 + 1;                           // D: ref only
                ops[2] = (150 - a) * 8 + 3;
                r.n_ops = 3;
                for (int j = 0; j < a; j++) ch[j] = seq[(size_t)(f - 1 + j)];
                for (int j = a; j < 150; j++) ch[j] = seq[(size_t)(f - 1 + j + 3)];
                r.last = f + 150 + 3 - 1;
            } else {
                ops[0] = 150 * 8 + 3;
                r.n_ops = 1;
                for (int j = 0; j < 150; j++) ch[j] = seq[(size_t)(f - 1 + j)];
                r.last = f + 150 - 1;
            }
            for (int j = 0; j < 150; j++) qu[j] = (char)(33 + 30 + (int)(rng() % 8));
            r.first = f;
            r.flags = (rng() & 1) ? 16 : 0;
            r.len = 150;
            r.ops = ops;
            r.chars = ch;
            r.quals = qu;
            r.hold = blk;
            reads.push_back(r);
        }
        RegionOut out;
        const auto t0 = std::chrono::steady_clock::now();
        replay_region(seq, X - 700, X + 500, reads, rp, nullptr, nullptr, out);
        total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        positions += (long long)out.pos.size();
        calls += (long long)out.indels.size();
    }
    std::printf("%d regions, %lld positions, %lld indel calls: %.1f ms (%.0f ns per position)\n", n_regions, positions, calls,
                total_ms, total_ms * 1e6 / (double)std::max(1LL, positions));
    return 0;
}
