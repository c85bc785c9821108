// parse_table_probe.cpp (round 6): deflate_slow's parse driven by per-position match tables (first-max
// candidate within 128 / 32 chain steps, computed by interleaved chain walks) vs pdeflate.h's Parser (one
// walk at a time, inline). Checks the two symbol streams are identical and times both on fp32 weights.
//   g++ -O3 -march=native -std=c++17 -o /tmp/ptp tools/probe_src/parse_table_probe.cpp && /tmp/ptp 32
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
#include "../../fedn_amd/csrc/pdeflate.h"

using namespace pdef;

struct TabParser {
    const uint8_t* S;
    int64_t L;
    static constexpr int RB = 16, RS = 1 << RB, RM = RS - 1;
    struct Slot { uint32_t prev, key; };
    std::vector<uint32_t> head;
    std::vector<Slot> ring;
    int64_t ins = 0;     // positions < ins are inserted
    // per-position results for the current block
    static constexpr int BLK = 16384;
    int64_t blk0 = -1;
    std::vector<uint32_t> t128, t32;   // (len << 16) | dist, 0 = none
    std::vector<uint8_t> gate;         // hash_head != NIL && within MAX_DIST
    int64_t t = 0, mstart = 0; int64_t tot_steps = 0, tot_pos = 0, tot_keyhits = 0;
    int avail = 0, mlen = 2;
    TabParser(const uint8_t* s, int64_t l) : S(s), L(l), head(kHSize, 0), ring(RS, Slot{0, 0}), t128(BLK), t32(BLK), gate(BLK) {}
    static inline uint32_t load32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
    inline void insert(int64_t p) {
        const uint32_t h = hash3(S + p);
        ring[p & RM] = Slot{head[h], load32(S + p)};
        head[h] = (uint32_t)(p + 1);
    }
    void start(int64_t b) {
        const int64_t base = std::max<int64_t>(0, b - kWSize);
        for (int64_t p = base; p < b; ++p) insert(p);
        ins = b;
        t = b;
    }
    // tables for positions [b0, b0 + BLK) (all inserted first)
    void build(int64_t b0) {
        const int64_t e0 = std::min<int64_t>(L - 3, b0 + BLK);
        for (int64_t p = ins; p < e0; ++p) insert(p);
        ins = std::max(ins, e0);
        blk0 = b0;
        constexpr int G = 8;
        for (int64_t g = b0; g < e0; g += G) {
            const int n = (int)std::min<int64_t>(G, e0 - g);
            uint32_t cur[G], skey[G];
            int best128[G], best32[G], steps[G];
            uint32_t pos128[G], pos32[G];
            bool live[G];
            for (int i = 0; i < n; ++i) {
                const int64_t tt = g + i;
                const uint32_t hh = ring[tt & RM].prev;
                const bool ok = hh && tt - (int64_t)(hh - 1) <= kMaxDist;
                gate[tt - b0] = ok; ++tot_pos;
                cur[i] = hh;
                skey[i] = load32(S + tt);
                best128[i] = best32[i] = 2;
                pos128[i] = pos32[i] = 0;
                steps[i] = 0;
                live[i] = ok;
            }
            bool any = true;
            while (any) {
                any = false;
                for (int i = 0; i < n; ++i) {
                    if (!live[i]) continue;
                    const int64_t tt = g + i;
                    const int64_t p = (int64_t)cur[i] - 1;
                    const Slot sl = ring[p & RM];
                    ++steps[i]; ++tot_steps;
                    if (((sl.key ^ skey[i]) & 0x00FFFFFFu) == 0) {
                        ++tot_keyhits; const int len = kMinMatch + common255(S + tt + 3, S + p + 3);
                        if (len > best128[i]) {
                            best128[i] = len;
                            pos128[i] = (uint32_t)(tt - p);
                        }
                        if (steps[i] <= 32 && len > best32[i] && best32[i] < kNice) {
                            best32[i] = len;
                            pos32[i] = (uint32_t)(tt - p);
                        }
                        if (len >= kNice) { live[i] = false; continue; }
                    }
                    const uint32_t nx = sl.prev;
                    if (!nx || tt - (int64_t)(nx - 1) >= kMaxDist || steps[i] >= kChain) {
                        live[i] = false;
                        continue;
                    }
                    cur[i] = nx;
                    __builtin_prefetch(&ring[(nx - 1) & RM]);
                    any = true;
                }
            }
            for (int i = 0; i < n; ++i) {
                t128[g + i - b0] = best128[i] > 2 ? ((uint32_t)best128[i] << 16 | pos128[i]) : 0;
                t32[g + i - b0] = best32[i] > 2 ? ((uint32_t)best32[i] << 16 | pos32[i]) : 0;
            }
        }
    }
    inline void step(Syms& out) {
        if (blk0 < 0 || t >= blk0 + BLK || t < blk0) build(t);
        const int64_t i = t - blk0;
        const int prev_len = mlen;
        const int64_t prev_match = mstart;
        mlen = kMinMatch - 1;
        if (gate[i] && prev_len < kLazy) {
            const uint32_t e = prev_len >= kGood ? t32[i] : t128[i];
            const int len = (int)(e >> 16);
            if (len > prev_len) { mlen = len; mstart = t - (int64_t)(e & 0xFFFF); }
            else mlen = prev_len;
            if (mlen == kMinMatch && t - mstart > kTooFar) mlen = kMinMatch - 1;
        }
        if (prev_len >= kMinMatch && mlen <= prev_len) {
            out.match(prev_len, (int)(t - 1 - prev_match), t - 1);
            avail = 0;
            mlen = kMinMatch - 1;
            t += prev_len - 1;
        } else if (avail) {
            out.lit(S[t - 1], t - 1);
            ++t;
        } else {
            avail = 1;
            ++t;
        }
    }
};

int main(int argc, char** argv) {
    const int64_t L = (argc > 1 ? atoll(argv[1]) : 32) << 20;
    std::vector<uint8_t> S((size_t)L);
    std::mt19937 rng(1);
    std::normal_distribution<float> nd;
    for (int64_t i = 0; i + 4 <= L; i += 4) { float f = nd(rng); std::memcpy(&S[i], &f, 4); }
    const int64_t stop = L - 4096;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    Syms a, b;
    double t0 = now();
    { Parser P(S.data(), L); P.start(0); while (P.t < stop) P.step(a); }
    double t1 = now();
    TabParser T(S.data(), L); T.start(0); while (T.t < stop) T.step(b);
    printf("steps/pos %.2f keyhits/pos %.3f\n", (double)T.tot_steps / T.tot_pos, (double)T.tot_keyhits / T.tot_pos);
    double t2 = now();
    bool same = a.n == b.n && std::equal(a.w.begin(), a.w.begin() + a.n, b.w.begin());
    size_t firstdiff = 0;
    while (firstdiff < std::min(a.n, b.n) && a.w[firstdiff] == b.w[firstdiff]) ++firstdiff;
    printf("bytes %lld  parser %.3f s (%.1f ns/B)  table %.3f s (%.1f ns/B)  same %d  words %zu %zu firstdiff %zu\n",
           (long long)L, t1 - t0, (t1 - t0) / L * 1e9, t2 - t1, (t2 - t1) / L * 1e9, (int)same, a.n, b.n, firstdiff);
}
