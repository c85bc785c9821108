// pdeflate.h — the deflate stream numpy writes for one large npz member, computed on many threads.
//
// np.savez_compressed (numpyhelper.Helper.save, fedn/utils/helpers/plugins/numpyhelper.py:162)
// deflates each member with zlib at level 6 through one z_stream. That stream is a pure function of
// the bytes and of zlib 1.2.11's algorithm (deflate.c deflate_slow / longest_match / fill_window,
// trees.c), so it can be recomputed in parallel and come out byte-identical:
//
//  1. LZ77 parse, chunk-parallel. deflate_slow's parse at position t depends only on its lazy-match
//     state (match_available, match_length, match_start) and on the hash chains, and the chains
//     hold every earlier position (all are inserted), so a parse started at a chunk start with the
//     preceding 32 KiB inserted ("speculative") is the true parse from the first position where the
//     two agree on that state. Every chunk parses speculatively and marks the tops where its state
//     needs no match_start (match_length 2); the previous chunk continues its own (true) parse past
//     its end until it stands at such a top in the same state ("sync"), normally within a few bytes
//     (in periodic data the two may run out of phase to the end of the run).
//     Positions are handled as stream offsets; zlib's window coordinates only matter at two edges,
//     both handled exactly: a stored block is allowed only while its start is still in the window
//     (block_start >= 0, tracked through the slide schedule), and one hash-head corner right at a
//     window slide (checked; the member falls back to zlib when it occurs).
//  2. Window schedule, sequential and cheap: fill_window's calls (where they happen depends on the
//     parse and on numpy's write sizes), the slides they make, and a faithful replay of deflate_slow
//     with a real 64 KiB window over the stream's last ~100 KiB, where lookahead runs short and
//     matches may read stale window bytes.
//  3. Blocks: every 16383 symbols (lit_bufsize - 1 at memLevel 8). Each block's trees are built by
//     trees.c's exact algorithm (heap order with depth ties, gen_bitlen's overflow repair, scan_tree
//     / send_tree run-lengths) and the stored / fixed / dynamic choice made as _tr_flush_block
//     makes it; blocks are sized, placed at their bit offsets and encoded in parallel.
// Anything outside what this models makes the caller run zlib itself (FNPZ's exact fallback), so
// the output is zlib's bytes either way; tests/test_pdeflate.py compares against libz directly.
//
// Attribution. Byte-identical output means zlib's decisions reproduced exactly, so parts of this
// file follow zlib 1.2.11 closely: the tree construction (TreeBuilder::pqdownheap / gen_bitlen /
// build_tree, scan_tree, send_tree, the static tables and gen_codes: trees.c) and the tail replay
// (Tail::longest_match / fill_window / run: deflate.c's longest_match, fill_window and
// deflate_slow). Those parts are altered versions of zlib code — restructured for the chunked,
// stream-offset parse and parallel block encoding, not the original software — and carry zlib's
// notice:
//
//   Copyright (C) 1995-2017 Jean-loup Gailly and Mark Adler
//
//   This software is provided 'as-is', without any express or implied warranty. In no event will
//   the authors be held liable for any damages arising from the use of this software.
//
//   Permission is granted to anyone to use this software for any purpose, including commercial
//   applications, and to alter it and redistribute it freely, subject to the following
//   restrictions:
//   1. The origin of this software must not be misrepresented; you must not claim that you wrote
//      the original software. If you use this software in a product, an acknowledgment in the
//      product documentation would be appreciated but is not required.
//   2. Altered source versions must be plainly marked as such, and must not be misrepresented as
//      being the original software.
//   3. This notice may not be removed or altered from any source distribution.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <thread>
#include <utility>
#include <vector>

#include "fnpz_guard.h"

namespace pdef {

// ---- zlib 1.2.11 constants (deflate.h, deflate.c configuration_table[6], trees.c) ----------------
constexpr int kWSize = 1 << 15, kWMask = kWSize - 1;
constexpr int kHBits = 15, kHSize = 1 << kHBits, kHMask = kHSize - 1;
constexpr int kMinMatch = 3, kMaxMatch = 258;
constexpr int kMinLookahead = kMaxMatch + kMinMatch + 1;   // 262
constexpr int64_t kMaxDist = kWSize - kMinLookahead;       // 32506
constexpr int64_t kWindowSize = 2 * kWSize;                // 65536
constexpr int kTooFar = 4096;
constexpr int kGood = 8, kLazy = 16, kNice = 128, kChain = 128;
constexpr int64_t kBlockSyms = (1 << (8 + 6)) - 1;         // lit_bufsize - 1
constexpr int64_t kMinChunk = 1 << 18;                     // smallest chunk a member is cut into
constexpr int64_t kTailStop = 1024;                        // speculative parses stop this far before the end
constexpr int64_t kTailRec = 192 << 10;                    // recorded tops before the end (last chunk)
constexpr int kCkEvery = 256;                              // symbol checkpoints

// byte buffers whose resize leaves new bytes uninitialised: a deflate stream's output is written
// in full by the parallel encode (and a zlib stream's by zlib), so zero-filling it first — a serial
// pass that also takes every page fault on one thread — is wasted (round 6, profiles/r06_save_phases.log)
template <class T>
struct NoInit : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInit<U>;
    };
    NoInit() = default;
    template <class U>
    NoInit(const NoInit<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, NoInit<uint8_t>>;

inline uint32_t hash3(const uint8_t* p) { return (((uint32_t)p[0] << 10) ^ ((uint32_t)p[1] << 5) ^ p[2]) & kHMask; }

// ---- symbol streams: a literal is one u16 (< 256); a match is (0x8000 | len-3), dist -------------
struct Ck {
    uint32_t word;
    int64_t pos, sym;
};
struct Syms {
    std::vector<uint16_t> w;
    size_t n = 0;
    int64_t nsym = 0;
    std::vector<Ck> ck;   // before symbol k * kCkEvery: (word offset, position)
    inline void ensure(size_t k) {
        if (n + k > w.size()) w.resize(std::max(w.size() * 2, n + k + 4096));
    }
    inline void mark(int64_t pos) {
        if ((nsym & (kCkEvery - 1)) == 0) ck.push_back(Ck{(uint32_t)n, pos, nsym});
    }
    inline void lit(uint8_t c, int64_t pos) {
        mark(pos);
        ensure(1);
        w[n++] = c;
        ++nsym;
    }
    inline void match(int len, int dist, int64_t pos) {
        mark(pos);
        ensure(2);
        w[n++] = (uint16_t)(0x8000 | (len - kMinMatch));
        w[n++] = (uint16_t)dist;
        ++nsym;
    }
};
inline int sym_len(const uint16_t* w, size_t i) { return (w[i] & 0x8000) ? (w[i] & 0xFF) + kMinMatch : 1; }
inline int sym_words(const uint16_t* w, size_t i) { return (w[i] & 0x8000) ? 2 : 1; }

// deflate_slow's state at an iteration top, before INSERT_STRING
struct Rec {
    int64_t t, mstart, nsym;
    uint32_t word;
    int16_t mlen;
    uint8_t avail;
};

inline int common255(const uint8_t* a, const uint8_t* b) {   // equal leading bytes, at most 255
    int k = 0;
    for (; k + 8 <= 255; k += 8) {
        uint64_t x, y;
        std::memcpy(&x, a + k, 8);
        std::memcpy(&y, b + k, 8);
        if (x != y) return k + (__builtin_ctzll(x ^ y) >> 3);
    }
    for (; k < 255 && a[k] == b[k]; ++k) {
    }
    return k;
}

// ---- 1. the speculative / true parse in stream offsets ------------------------------------------
struct Parser {
    const uint8_t* S;
    int64_t L;
    int64_t base = 0;   // a position p is stored as p - base + 1; 0 is NIL (and stream position 0)
    // zlib's prev[] ring with each position's first 4 bytes beside its link: a chain step reads one
    // 8-byte slot, and most candidates (hash collisions, 3-byte matches) are rejected without
    // touching the stream — the candidates visited and counted are zlib's, only cheaper to reject
    struct Slot {
        uint32_t prev, key;
    };
    std::vector<uint32_t> head;
    std::vector<Slot> ring;
    int64_t t = 0, mstart = 0;
    int avail = 0, mlen = kMinMatch - 1;

    Parser(const uint8_t* s, int64_t l) : S(s), L(l), head(kHSize, 0), ring(kWSize, Slot{0, 0}) {}
    inline uint32_t enc(int64_t p) const { return p == 0 ? 0u : (uint32_t)(p - base + 1); }
    inline int64_t dec(uint32_t e) const { return (int64_t)e - 1 + base; }
    static inline uint32_t load32(const uint8_t* p) {
        uint32_t v;
        std::memcpy(&v, p, 4);
        return v;
    }
    inline uint32_t insert(int64_t p) {
        const uint32_t h = hash3(S + p), hh = head[h];
        ring[p & kWMask] = Slot{hh, load32(S + p)};
        head[h] = enc(p);
        return hh;
    }
    void rebase() {   // keep stored offsets in 32 bits on long parses (entries past the window drop)
        const int64_t nb = t - kWSize;
        auto fix = [&](uint32_t& e) {
            if (!e) return;
            const int64_t p = dec(e);
            e = p < nb ? 0u : (uint32_t)(p - nb + 1);
        };
        for (auto& e : head) fix(e);
        for (auto& e : ring) fix(e.prev);
        base = nb;
    }
    void start(int64_t b) {
        base = std::max<int64_t>(0, b - kWSize);
        for (int64_t p = base; p < b; ++p) insert(p);
        t = b;
        avail = 0;
        mlen = kMinMatch - 1;
        mstart = 0;
    }
    inline Rec rec(const Syms& s) const { return Rec{t, mstart, s.nsym, (uint32_t)s.n, (int16_t)mlen, (uint8_t)avail}; }
    inline bool same(const Rec& r) const {
        return r.t == t && r.avail == avail && r.mlen == mlen && (mlen < kMinMatch || r.mstart == mstart);
    }
    inline int longest(uint32_t cur, int prev_len) {
        int chain = kChain;
        if (prev_len >= kGood) chain >>= 2;
        const uint8_t* scan = S + t;
        int best = prev_len;
        uint8_t e1 = scan[best - 1], e0 = scan[best];
        const uint32_t skey = load32(scan);
        // a candidate beats best only if its first min(best + 1, 4) bytes equal scan's (bytes 0..2
        // agree for every same-hash candidate whose bytes 0..1 do, as zlib's check relies on)
        uint32_t kmask = best >= 3 ? 0xFFFFFFFFu : 0x00FFFFFFu;
        const int64_t limit = t - kMaxDist;
        int64_t cp = dec(cur);
        for (;;) {
            const Slot sl = ring[cp & kWMask];
            if (((sl.key ^ skey) & kmask) == 0) {
                const uint8_t* m = S + cp;
                if (best < 4 || (m[best] == e0 && m[best - 1] == e1)) {
                    const int len = kMinMatch + common255(scan + 3, m + 3);
                    if (len > best) {
                        mstart = cp;
                        best = len;
                        if (len >= kNice) break;
                        e1 = scan[best - 1];
                        e0 = scan[best];
                        kmask = 0xFFFFFFFFu;
                    }
                }
            }
            const uint32_t nx = sl.prev;
            if (!nx) break;
            cp = dec(nx);
            if (cp <= limit || --chain == 0) break;
        }
        return best;
    }
    // the chain walks a few positions ahead, started early: the first slot of t + 4's chain and the
    // second of t + 2's are fetched while this position is parsed (a walk is a chain of dependent
    // L2 loads, and the branch that ends each walk is hard to predict, so out-of-order execution
    // rarely gets to the next one on its own); addresses only, the parse is unchanged
    inline void prefetch_ahead() {
        const int64_t a = t + 4, b = t + 2;
        if (a + 3 <= L) {
            const uint32_t e = head[hash3(S + a)];
            if (e) __builtin_prefetch(&ring[(size_t)(dec(e) & kWMask)]);
        }
        if (b + 3 <= L) {
            const uint32_t e = head[hash3(S + b)];
            if (e) {
                const uint32_t n2 = ring[(size_t)(dec(e) & kWMask)].prev;
                if (n2) __builtin_prefetch(&ring[(size_t)(dec(n2) & kWMask)]);
            }
        }
    }
    // one deflate_slow iteration at top t (lookahead >= MIN_LOOKAHEAD)
    inline void step(Syms& out) {
        prefetch_ahead();
        const uint32_t hh = insert(t);
        const int prev_len = mlen;
        const int64_t prev_match = mstart;
        mlen = kMinMatch - 1;
        if (hh && prev_len < kLazy && t - dec(hh) <= kMaxDist) {
            mlen = longest(hh, prev_len);
            if (mlen == kMinMatch && t - mstart > kTooFar) mlen = kMinMatch - 1;
        }
        if (prev_len >= kMinMatch && mlen <= prev_len) {
            out.match(prev_len, (int)(t - 1 - prev_match), t - 1);
            const int64_t last = t + prev_len - 2;
            for (int64_t p = t + 1; p <= last; ++p) insert(p);
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
        if (t - base > (int64_t(1) << 31)) rebase();
    }
};

struct Chunk {
    int64_t b = 0, e = 0, stop = 0;
    bool last = false;
    Parser* P = nullptr;
    Syms spec, ext;
    // 2 bits per position of [b, stop): the speculative parse had a top there with match_length 2
    // and match_available 0 (bit 0) or 1 (bit 1) — the states a sync is looked for at
    std::vector<uint8_t> tops;
    std::vector<Rec> rec_tail;   // last chunk: every top of its final kTailRec bytes
    int64_t spec_p1 = 0;         // stream bytes the speculative symbols cover up to
    // stitch: c's own parse continued (ext) until it met chunk sync_chunk's speculative parse at
    // top sync_t; that parse's symbols from (sync_word, sync_sym, sync_pos) are the true ones
    bool synced = false;
    int sync_chunk = -1;
    int64_t sync_t = 0, sync_pos = 0, sync_sym = 0;
    size_t sync_word = 0, ext_words = 0;
    int64_t ext_syms = 0;
    bool ext_final = false;      // no sync anywhere: the extension runs to the end (and is recorded)
    int64_t ext_p1 = 0;
    inline int top_state(int64_t t) const {   // 0: no top with match_length 2; 1 + match_available
        const int64_t i = t - b;
        return (tops[(size_t)(i >> 2)] >> (2 * (i & 3))) & 3;
    }
};

// speculative parse of chunk c (the last chunk also records the full state of its final tops)
inline void parse_chunk(Chunk& c, const uint8_t* S, int64_t L) {
    c.P = new Parser(S, L);
    Parser& P = *c.P;
    P.start(c.b);
    c.stop = c.last ? L - kTailStop : c.e;
    const int64_t tail_from = c.last ? L - kTailRec : INT64_MAX;
    c.spec.w.resize((size_t)((c.stop - c.b) + 4096));
    c.tops.assign((size_t)((c.stop - c.b) / 4 + 1), 0);
    while (P.t < c.stop) {
        if (P.mlen == kMinMatch - 1) {
            const int64_t i = P.t - c.b;
            c.tops[(size_t)(i >> 2)] |= (uint8_t)((1 + P.avail) << (2 * (i & 3)));
        }
        if (P.t >= tail_from) c.rec_tail.push_back(P.rec(c.spec));
        P.step(c.spec);
    }
    c.spec_p1 = P.t - P.avail;
}

// the word offset / symbol index in s of the symbol that starts at position pos (false: none does)
inline bool locate(const Syms& s, int64_t pos, size_t& word, int64_t& sym) {
    const auto& ck = s.ck;
    size_t lo = 0, hi = ck.size();
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (ck[mid].pos <= pos) lo = mid + 1; else hi = mid;
    }
    if (lo == 0) return false;
    size_t w = ck[lo - 1].word;
    int64_t p = ck[lo - 1].pos, k = ck[lo - 1].sym;
    while (p < pos && w < s.n) {
        p += sym_len(s.w.data(), w);
        w += sym_words(s.w.data(), w);
        ++k;
    }
    if (p != pos) return false;
    word = w;
    sym = k;
    return true;
}

// continue chunk c's (true) parse through the chunks after it until it meets a speculative parse
// in a match_length-2 state at the same top, or reaches `until`; false if it did not
inline bool extend(Chunk& c, std::vector<Chunk>& C, int first, int64_t until) {
    Parser& P = *c.P;
    int k = first;
    while (P.t < until) {
        while (k < (int)C.size() && P.t >= C[k].stop) ++k;
        if (k >= (int)C.size()) return false;
        const Chunk& tg = C[k];
        if (P.mlen == kMinMatch - 1 && P.t >= tg.b && tg.top_state(P.t) == 1 + P.avail) {
            size_t w;
            int64_t sym;
            if (locate(tg.spec, P.t - P.avail, w, sym)) {
                c.synced = true;
                c.sync_chunk = k;
                c.sync_t = P.t;
                c.sync_pos = P.t - P.avail;
                c.sync_word = w;
                c.sync_sym = sym;
                c.ext_words = c.ext.n;
                c.ext_syms = c.ext.nsym;
                return true;
            }
        }
        P.step(c.ext);
    }
    return false;
}

// ---- 2. the true parse as runs of symbols; window schedule; the faithful tail ----------------------
struct Run {
    const Syms* s;
    size_t w0, w1;      // words
    int64_t s0, s1;     // symbol indices within s
    int64_t p0, p1;     // positions covered
    int64_t g0;         // global index of the first symbol
};

struct Cursor {   // a symbol of the true parse
    size_t run;
    size_t word;
    int64_t pos, sym;
};

class Runs {
public:
    std::vector<Run> r;
    void add(const Syms* s, size_t w0, size_t w1, int64_t s0, int64_t s1, int64_t p0, int64_t p1) {
        if (w1 <= w0) return;
        const int64_t g0 = r.empty() ? 0 : r.back().g0 + (r.back().s1 - r.back().s0);
        r.push_back(Run{s, w0, w1, s0, s1, p0, p1, g0});
    }
    int64_t total() const { return r.empty() ? 0 : r.back().g0 + (r.back().s1 - r.back().s0); }
    // the last checkpoint at or before (pos / sym) inside run k, as a cursor
    Cursor seek_pos(size_t k, int64_t pos) const {
        const Run& q = r[k];
        const auto& ck = q.s->ck;
        size_t lo = 0, hi = ck.size();
        while (lo < hi) {   // first checkpoint with pos > target
            const size_t mid = (lo + hi) / 2;
            if (ck[mid].pos <= pos) lo = mid + 1; else hi = mid;
        }
        Cursor c{k, q.w0, q.p0, q.s0};
        if (lo > 0 && ck[lo - 1].word >= q.w0 && ck[lo - 1].word < q.w1) c = Cursor{k, ck[lo - 1].word, ck[lo - 1].pos, ck[lo - 1].sym};
        return c;
    }
    Cursor seek_sym(size_t k, int64_t sym) const {
        const Run& q = r[k];
        const auto& ck = q.s->ck;
        const size_t i = (size_t)(sym / kCkEvery);
        Cursor c{k, q.w0, q.p0, q.s0};
        if (i < ck.size() && ck[i].sym >= q.s0 && ck[i].word < q.w1 && ck[i].sym <= sym) c = Cursor{k, ck[i].word, ck[i].pos, ck[i].sym};
        return c;
    }
    size_t run_of_pos(int64_t pos) const {
        size_t lo = 0, hi = r.size();
        while (lo < hi) {
            const size_t mid = (lo + hi) / 2;
            if (r[mid].p1 <= pos) lo = mid + 1; else hi = mid;
        }
        return lo;
    }
    size_t run_of_global(int64_t g) const {
        size_t lo = 0, hi = r.size();
        while (lo < hi) {
            const size_t mid = (lo + hi) / 2;
            if (r[mid].g0 + (r[mid].s1 - r[mid].s0) <= g) lo = mid + 1; else hi = mid;
        }
        return lo;
    }
    // first iteration top >= x (tops: every position except the interior of an emitted match past
    // its second byte); -1 if x lies beyond the runs
    int64_t top_at_or_after(int64_t x) const {
        const size_t k = run_of_pos(x);
        if (k >= r.size()) return -1;
        Cursor c = seek_pos(k, x);
        const uint16_t* w = r[k].s->w.data();
        for (;;) {
            const int len = sym_len(w, c.word);
            if (c.pos + len > x) return (len > 2 && x >= c.pos + 2) ? c.pos + len : x;
            c.pos += len;
            c.word += sym_words(w, c.word);
            if (c.word >= r[k].w1) return x;   // x is the first position of the next run
        }
    }
    // the symbol with global index g
    Cursor at_global(int64_t g) const {
        const size_t k = run_of_global(g);
        const Run& q = r[k];
        const int64_t sym = q.s0 + (g - q.g0);
        Cursor c = seek_sym(k, sym);
        const uint16_t* w = q.s->w.data();
        while (c.sym < sym) {
            c.pos += sym_len(w, c.word);
            c.word += sym_words(w, c.word);
            ++c.sym;
        }
        return c;
    }
};

// zlib's 64 KiB window as intervals of stream bytes: which stream offset each window index last
// received (by a read or by a slide's copy), -1 where nothing was written yet (zeros: zlib zeroes
// what lies past its high-water mark before it can be read). Tracks the bytes the tail's matches
// may read past the end of the data (stale bytes of earlier windows) without copying the stream.
struct WinMap {
    struct Iv {
        int64_t lo, hi, src;   // window [lo, hi) holds stream [src, src + hi - lo), or zeros (src < 0)
    };
    std::vector<Iv> iv{Iv{0, kWindowSize, -1}};
    void write(int64_t lo, int64_t hi, int64_t src) {
        if (hi <= lo) return;
        std::vector<Iv> out;
        for (const Iv& v : iv) {
            if (v.hi <= lo || v.lo >= hi) {
                out.push_back(v);
                continue;
            }
            if (v.lo < lo) out.push_back(Iv{v.lo, lo, v.src});
            if (v.hi > hi) out.push_back(Iv{hi, v.hi, v.src < 0 ? -1 : v.src + (hi - v.lo)});
        }
        out.push_back(Iv{lo, hi, src});
        std::sort(out.begin(), out.end(), [](const Iv& x, const Iv& y) { return x.lo < y.lo; });
        iv.swap(out);
    }
    void slide(int64_t n) {   // window[0, n) = window[wsize, wsize + n)
        std::vector<Iv> moved;
        for (const Iv& v : iv) {
            const int64_t lo = std::max<int64_t>(v.lo, kWSize), hi = std::min<int64_t>(v.hi, kWSize + n);
            if (hi > lo) moved.push_back(Iv{lo - kWSize, hi - kWSize, v.src < 0 ? -1 : v.src + (lo - v.lo)});
        }
        for (const Iv& v : moved) write(v.lo, v.hi, v.src);
    }
    void materialize(const uint8_t* S, uint8_t* win) const {
        for (const Iv& v : iv) {
            if (v.src < 0) std::memset(win + v.lo, 0, (size_t)(v.hi - v.lo));
            else std::memcpy(win + v.lo, S + v.src, (size_t)(v.hi - v.lo));
        }
    }
};

// numpy's deflate() input pieces and zlib's fill_window schedule over them
struct Feed {
    const std::vector<int64_t>* ends;   // cumulative ends of the deflate() inputs
    size_t seg = 0;                     // current input piece
    int64_t read_end = 0, w_base = 0;
    bool finishing = false;
    std::vector<int64_t> slides;        // tops where the window slid
    WinMap map;
    // fill_window's do-while at top t
    void fill(int64_t t) {
        for (;;) {
            int64_t more = kWindowSize - (read_end - w_base);
            if (t - w_base >= kWSize + kMaxDist) {
                map.slide(kWSize - more);   // zmemcpy(window, window + wsize, wsize - more)
                w_base += kWSize;
                more += kWSize;
                slides.push_back(t);
            }
            const int64_t avail_in = finishing ? 0 : (*ends)[seg] - read_end;
            if (avail_in == 0) break;
            const int64_t n = std::min(more, avail_in);
            map.write(read_end - w_base, read_end - w_base + n, read_end);
            read_end += n;
            if (!(read_end - t < kMinLookahead && (*ends)[seg] - read_end != 0)) break;
        }
    }
    // deflate_slow's loop top: fill while short of lookahead, moving on to the next deflate() call
    // (input piece) when one runs dry (need_more)
    void top(int64_t t) {
        while (read_end - t < kMinLookahead) {
            fill(t);
            if (read_end - t >= kMinLookahead) break;
            if (finishing) break;
            if (seg + 1 < ends->size()) ++seg;
            else finishing = true;   // the Z_FINISH call: no more input
        }
    }
};

// deflate_slow / longest_match / fill_window with a real window, from a recorded top to the end of
// the stream (zlib 1.2.11 semantics, window coordinates)
struct Tail {
    const uint8_t* S;
    int64_t L;
    Feed& F;
    std::vector<uint8_t> win;
    std::vector<uint16_t> head, prev;
    int64_t strstart = 0, lookahead = 0, match_start = 0, prev_match = 0;
    int match_length = kMinMatch - 1, prev_length = kMinMatch - 1, match_available = 0;
    uint32_t ins_h = 0;
    Syms out;
    bool final_literal = false;

    Tail(const uint8_t* s, int64_t l, Feed& f) : S(s), L(l), F(f), win(kWindowSize + 1024, 0), head(kHSize, 0), prev(kWSize, 0) {}
    inline void update_hash(uint8_t c) { ins_h = ((ins_h << 5) ^ c) & kHMask; }
    inline uint16_t insert_string(int64_t str) {
        update_hash(win[str + kMinMatch - 1]);
        const uint16_t hh = head[ins_h];
        prev[str & kWMask] = hh;
        head[ins_h] = (uint16_t)str;
        return hh;
    }
    // state at top r.t before its fill check: the window as F's schedule left it
    void start(const Rec& r) {
        const int64_t W = F.w_base;
        F.map.materialize(S, win.data());
        for (int64_t p = W; p < r.t; ++p) {
            const int64_t i = p - W;
            const uint32_t h = hash3(win.data() + i);
            prev[i & kWMask] = head[h];
            head[h] = (uint16_t)i;
        }
        strstart = r.t - W;
        lookahead = F.read_end - r.t;
        ins_h = (((uint32_t)win[strstart - 1] << 10) ^ ((uint32_t)win[strstart] << 5) ^ win[strstart + 1]) & kHMask;
        match_available = r.avail;
        match_length = r.mlen;
        match_start = r.mstart - W;
    }
    void fill_window() {
        do {
            int64_t more = kWindowSize - lookahead - strstart;
            if (strstart >= kWSize + kMaxDist) {
                std::memcpy(win.data(), win.data() + kWSize, (size_t)(kWSize - more));
                match_start -= kWSize;
                strstart -= kWSize;
                F.w_base += kWSize;
                F.slides.push_back(F.w_base + strstart);
                for (auto& m : head) m = (uint16_t)(m >= kWSize ? m - kWSize : 0);
                for (auto& m : prev) m = (uint16_t)(m >= kWSize ? m - kWSize : 0);
                more += kWSize;
            }
            const int64_t avail_in = F.finishing ? 0 : (*F.ends)[F.seg] - F.read_end;
            if (avail_in == 0) break;
            const int64_t n = std::min(more, avail_in);
            std::memcpy(win.data() + strstart + lookahead, S + F.read_end, (size_t)n);
            F.read_end += n;
            lookahead += n;
            if (lookahead >= kMinMatch) {   // s->insert is 0 here
                ins_h = win[strstart];
                update_hash(win[strstart + 1]);
            }
        } while (lookahead < kMinLookahead && (*F.ends)[F.seg] - F.read_end != 0 && !F.finishing);
        // high_water: the window has been full, nothing to zero
    }
    int longest_match(int64_t cur_match) {
        int chain_length = kChain;
        const uint8_t* scan = win.data() + strstart;
        int best_len = prev_length;
        int nice_match = kNice;
        const int64_t limit = strstart > kMaxDist ? strstart - kMaxDist : 0;
        const uint8_t* strend = win.data() + strstart + kMaxMatch;
        uint8_t scan_end1 = scan[best_len - 1], scan_end = scan[best_len];
        if (prev_length >= kGood) chain_length >>= 2;
        if (nice_match > lookahead) nice_match = (int)lookahead;
        do {
            const uint8_t* match = win.data() + cur_match;
            if (match[best_len] != scan_end || match[best_len - 1] != scan_end1 || match[0] != scan[0] ||
                match[1] != scan[1])
                continue;
            {
                const uint8_t* s2 = scan + 2;
                const uint8_t* m2 = match + 2;
                do {
                } while (*++s2 == *++m2 && *++s2 == *++m2 && *++s2 == *++m2 && *++s2 == *++m2 && *++s2 == *++m2 &&
                         *++s2 == *++m2 && *++s2 == *++m2 && *++s2 == *++m2 && s2 < strend);
                const int len = kMaxMatch - (int)(strend - s2);
                if (len > best_len) {
                    match_start = cur_match;
                    best_len = len;
                    if (len >= nice_match) break;
                    scan_end1 = scan[best_len - 1];
                    scan_end = scan[best_len];
                }
            }
        } while ((cur_match = prev[cur_match & kWMask]) > limit && --chain_length != 0);
        if (best_len <= lookahead) return best_len;
        return (int)lookahead;
    }
    void run() {
        for (;;) {
            if (lookahead < kMinLookahead) {
                for (;;) {   // fill; a dry input piece moves to the next deflate() call
                    fill_window();
                    if (lookahead >= kMinLookahead || F.finishing) break;
                    if (F.seg + 1 < F.ends->size()) ++F.seg;
                    else F.finishing = true;
                }
                if (lookahead == 0) break;
            }
            int64_t hash_head = 0;
            if (lookahead >= kMinMatch) hash_head = insert_string(strstart);
            prev_length = match_length;
            prev_match = match_start;
            match_length = kMinMatch - 1;
            if (hash_head != 0 && prev_length < kLazy && strstart - hash_head <= kMaxDist) {
                match_length = longest_match(hash_head);
                if (match_length <= 5 && match_length == kMinMatch && strstart - match_start > kTooFar)
                    match_length = kMinMatch - 1;
            }
            if (prev_length >= kMinMatch && match_length <= prev_length) {
                const int64_t max_insert = strstart + lookahead - kMinMatch;
                out.match(prev_length, (int)(strstart - 1 - prev_match), F.w_base + strstart - 1);
                lookahead -= prev_length - 1;
                prev_length -= 2;
                do {
                    if (++strstart <= max_insert) insert_string(strstart);
                } while (--prev_length != 0);
                match_available = 0;
                match_length = kMinMatch - 1;
                ++strstart;
            } else if (match_available) {
                out.lit(win[strstart - 1], F.w_base + strstart - 1);
                ++strstart;
                --lookahead;
            } else {
                match_available = 1;
                ++strstart;
                --lookahead;
            }
        }
        if (match_available) {
            out.lit(win[strstart - 1], F.w_base + strstart - 1);
            final_literal = true;
            match_available = 0;
        }
        out.mark(F.w_base + strstart);
    }
};

// ---- 3. trees.c -----------------------------------------------------------------------------------
constexpr int kLCodes = 286, kDCodes = 30, kBLCodes = 19, kHeap = 2 * kLCodes + 1, kMaxBits = 15, kMaxBLBits = 7;
constexpr int kEndBlock = 256;
const int kExtraLBits[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const int kExtraDBits[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
const int kExtraBLBits[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
const uint8_t kBLOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Static {
    uint8_t length_code[256], dist_code[512];
    int base_length[29], base_dist[30];
    uint16_t sl_len[288], sl_code[288], sd_len[30], sd_code[30];
    static uint32_t reverse(uint32_t code, int len) {
        uint32_t r = 0;
        do {
            r |= code & 1;
            code >>= 1;
            r <<= 1;
        } while (--len > 0);
        return r >> 1;
    }
    static void gen_codes(const uint16_t* len, uint16_t* code, int max_code, const uint16_t* bl_count) {
        uint16_t next[kMaxBits + 1];
        uint32_t c = 0;
        for (int bits = 1; bits <= kMaxBits; ++bits) {
            c = (c + bl_count[bits - 1]) << 1;
            next[bits] = (uint16_t)c;
        }
        for (int n = 0; n <= max_code; ++n) {
            const int l = len[n];
            if (l == 0) continue;
            code[n] = (uint16_t)reverse(next[l]++, l);
        }
    }
    Static() {
        int length = 0, code;
        for (code = 0; code < 28; ++code) {
            base_length[code] = length;
            for (int n = 0; n < (1 << kExtraLBits[code]); ++n) length_code[length++] = (uint8_t)code;
        }
        length_code[length - 1] = (uint8_t)code;   // length 258: code 285, not 284 + 5 bits
        base_length[28] = 0;
        int dist = 0;
        for (code = 0; code < 16; ++code) {
            base_dist[code] = dist;
            for (int n = 0; n < (1 << kExtraDBits[code]); ++n) dist_code[dist++] = (uint8_t)code;
        }
        dist >>= 7;
        for (; code < kDCodes; ++code) {
            base_dist[code] = dist << 7;
            for (int n = 0; n < (1 << (kExtraDBits[code] - 7)); ++n) dist_code[256 + dist++] = (uint8_t)code;
        }
        uint16_t bl_count[kMaxBits + 1] = {0};
        for (int n = 0; n < 288; ++n) {
            sl_len[n] = n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8;
            bl_count[sl_len[n]]++;
        }
        gen_codes(sl_len, sl_code, 287, bl_count);
        for (int n = 0; n < kDCodes; ++n) {
            sd_len[n] = 5;
            sd_code[n] = (uint16_t)reverse((uint32_t)n, 5);
        }
    }
    inline int d_code(int dist) const { return dist < 256 ? dist_code[dist] : dist_code[256 + (dist >> 7)]; }
};
inline const Static& tables() {
    static const Static s;
    return s;
}

struct TreeDesc {
    uint16_t freq[kHeap], len[kHeap], dad[kHeap], code[kHeap];
    int max_code = 0;
};

struct TreeBuilder {   // deflate_state's tree-building fields
    int heap[kHeap];
    int heap_len = 0, heap_max = 0;
    uint8_t depth[kHeap];
    uint16_t bl_count[kMaxBits + 1];
    uint64_t opt_len = 0, static_len = 0;

    inline bool smaller(const TreeDesc& t, int n, int m) const {
        return t.freq[n] < t.freq[m] || (t.freq[n] == t.freq[m] && depth[n] <= depth[m]);
    }
    void pqdownheap(const TreeDesc& t, int k) {
        const int v = heap[k];
        int j = k << 1;
        while (j <= heap_len) {
            if (j < heap_len && smaller(t, heap[j + 1], heap[j])) j++;
            if (smaller(t, v, heap[j])) break;
            heap[k] = heap[j];
            k = j;
            j <<= 1;
        }
        heap[k] = v;
    }
    void gen_bitlen(TreeDesc& t, const uint16_t* stree, const int* extra, int base, int max_length) {
        const int max_code = t.max_code;
        int overflow = 0;
        for (int bits = 0; bits <= kMaxBits; ++bits) bl_count[bits] = 0;
        t.len[heap[heap_max]] = 0;
        int h;
        for (h = heap_max + 1; h < kHeap; ++h) {
            const int n = heap[h];
            int bits = t.len[t.dad[n]] + 1;
            if (bits > max_length) bits = max_length, overflow++;
            t.len[n] = (uint16_t)bits;
            if (n > max_code) continue;
            bl_count[bits]++;
            int xbits = 0;
            if (n >= base) xbits = extra[n - base];
            const uint64_t f = t.freq[n];
            opt_len += f * (uint64_t)(bits + xbits);
            if (stree) static_len += f * (uint64_t)(stree[n] + xbits);
        }
        if (overflow == 0) return;
        do {
            int bits = max_length - 1;
            while (bl_count[bits] == 0) bits--;
            bl_count[bits]--;
            bl_count[bits + 1] += 2;
            bl_count[max_length]--;
            overflow -= 2;
        } while (overflow > 0);
        for (int bits = max_length; bits != 0; bits--) {
            int n = bl_count[bits];
            while (n != 0) {
                const int m = heap[--h];
                if (m > max_code) continue;
                if ((unsigned)t.len[m] != (unsigned)bits) {
                    opt_len += ((uint64_t)bits - t.len[m]) * t.freq[m];
                    t.len[m] = (uint16_t)bits;
                }
                n--;
            }
        }
    }
    void build_tree(TreeDesc& t, const uint16_t* stree, const int* extra, int base, int elems, int max_length) {
        int max_code = -1;
        heap_len = 0;
        heap_max = kHeap;
        for (int n = 0; n < elems; ++n) {
            if (t.freq[n] != 0) {
                heap[++heap_len] = max_code = n;
                depth[n] = 0;
            } else {
                t.len[n] = 0;
            }
        }
        while (heap_len < 2) {
            const int node = heap[++heap_len] = (max_code < 2 ? ++max_code : 0);
            t.freq[node] = 1;
            depth[node] = 0;
            opt_len--;
            if (stree) static_len -= stree[node];
        }
        t.max_code = max_code;
        for (int n = heap_len / 2; n >= 1; n--) pqdownheap(t, n);
        int node = elems;
        do {
            const int n = heap[1];
            heap[1] = heap[heap_len--];
            pqdownheap(t, 1);
            const int m = heap[1];
            heap[--heap_max] = n;
            heap[--heap_max] = m;
            t.freq[node] = (uint16_t)(t.freq[n] + t.freq[m]);
            depth[node] = (uint8_t)((depth[n] >= depth[m] ? depth[n] : depth[m]) + 1);
            t.dad[n] = t.dad[m] = (uint16_t)node;
            heap[1] = node++;
            pqdownheap(t, 1);
        } while (heap_len >= 2);
        heap[--heap_max] = heap[1];
        gen_bitlen(t, stree, extra, base, max_length);
        Static::gen_codes(t.len, t.code, max_code, bl_count);
    }
};

inline void scan_tree(TreeDesc& tree, int max_code, TreeDesc& bl) {
    int prevlen = -1, nextlen = tree.len[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    tree.len[max_code + 1] = 0xffff;   // guard
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = tree.len[n + 1];
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            bl.freq[curlen] = (uint16_t)(bl.freq[curlen] + count);
        } else if (curlen != 0) {
            if (curlen != prevlen) bl.freq[curlen]++;
            bl.freq[16]++;
        } else if (count <= 10) {
            bl.freq[17]++;
        } else {
            bl.freq[18]++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

struct BitW {
    uint8_t* p;
    uint64_t acc = 0;
    int nb = 0;
    explicit BitW(uint8_t* out, int phase) : p(out), nb(phase) {}
    inline void put(uint32_t v, int n) {
        acc |= (uint64_t)v << nb;
        nb += n;
        if (nb >= 32) {
            std::memcpy(p, &acc, 4);   // little-endian host
            p += 4;
            acc >>= 32;
            nb -= 32;
        }
    }
    inline void align() {   // bi_windup
        while (nb > 0) {
            *p++ = (uint8_t)acc;
            acc >>= 8;
            nb -= 8;
        }
        nb = 0;
        acc = 0;
    }
    inline void flush_partial() {   // the last partial bytes (bits beyond nb are zero)
        while (nb > 0) {
            *p++ = (uint8_t)acc;
            acc >>= 8;
            nb -= 8;
        }
    }
};

inline void send_tree(BitW& bw, const TreeDesc& tree, int max_code, const TreeDesc& bl) {
    int prevlen = -1, nextlen = tree.len[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) max_count = 138, min_count = 3;
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = tree.len[n + 1];
        if (++count < max_count && curlen == nextlen) {
            continue;
        } else if (count < min_count) {
            do {
                bw.put(bl.code[curlen], bl.len[curlen]);
            } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) {
                bw.put(bl.code[curlen], bl.len[curlen]);
                count--;
            }
            bw.put(bl.code[16], bl.len[16]);
            bw.put((uint32_t)(count - 3), 2);
        } else if (count <= 10) {
            bw.put(bl.code[17], bl.len[17]);
            bw.put((uint32_t)(count - 3), 3);
        } else {
            bw.put(bl.code[18], bl.len[18]);
            bw.put((uint32_t)(count - 11), 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) max_count = 138, min_count = 3;
        else if (curlen == nextlen) max_count = 6, min_count = 3;
        else max_count = 7, min_count = 4;
    }
}

enum BlockType { kStored = 0, kFixed = 1, kDynamic = 2 };

struct Block {
    int64_t g0 = 0, g1 = 0;        // global symbols [g0, g1)
    int64_t p0 = 0, p1 = 0;        // stream bytes covered
    bool last = false, buf_ok = false;
    int type = kDynamic;
    int64_t bits = 0;              // encoded size (stored: set at placement)
    int64_t off = 0;               // global bit offset
    std::vector<uint8_t> bytes;    // encoded at its phase
};

// what encoding a block needs after planning: its trees' code lengths and where its symbols start
struct Plan {
    uint8_t llen[kLCodes + 2], dlen[kDCodes + 2], bllen[kBLCodes];
    int16_t lmax = 0, dmax = 0, maxbl = 0;
    size_t run = 0, word = 0;
};

struct Encoder {
    const Runs& R;
    const uint8_t* S;
    explicit Encoder(const Runs& r, const uint8_t* s) : R(r), S(s) {}

    // f(is_match, literal or len - 3, dist) for the block's symbols, from the cursor (run, word)
    template <class F>
    inline void each_symbol(const Block& b, size_t k, size_t word, F&& f) const {
        int64_t left = b.g1 - b.g0;
        while (left > 0) {
            const Run& q = R.r[k];
            const uint16_t* w = q.s->w.data();
            const size_t w1 = q.w1;
            while (word < w1 && left > 0) {
                const uint16_t v = w[word];
                if (v & 0x8000) {
                    f(true, v & 0xFF, (int)w[word + 1]);
                    word += 2;
                } else {
                    f(false, v, 0);
                    word += 1;
                }
                --left;
            }
            if (++k < R.r.size()) word = R.r[k].w0;
        }
    }
    // trees and type (as _tr_flush_block decides); the dynamic / fixed size in bits
    void plan(Block& b, Plan& pl) const {
        const Static& st = tables();
        TreeDesc lt, dt, bt;
        TreeBuilder tb;
        std::memset(lt.freq, 0, sizeof(lt.freq));
        std::memset(dt.freq, 0, sizeof(dt.freq));
        std::memset(bt.freq, 0, sizeof(bt.freq));
        lt.freq[kEndBlock] = 1;
        if (b.g1 > b.g0) {
            const Cursor c = R.at_global(b.g0);
            pl.run = c.run;
            pl.word = c.word;
            each_symbol(b, pl.run, pl.word, [&](bool m, int a, int d) {
                if (!m) {
                    lt.freq[a]++;
                } else {
                    lt.freq[st.length_code[a] + 257]++;
                    dt.freq[st.d_code(d - 1)]++;
                }
            });
        }
        tb.opt_len = tb.static_len = 0;
        tb.build_tree(lt, st.sl_len, kExtraLBits, 257, kLCodes, kMaxBits);
        tb.build_tree(dt, st.sd_len, kExtraDBits, 0, kDCodes, kMaxBits);
        scan_tree(lt, lt.max_code, bt);
        scan_tree(dt, dt.max_code, bt);
        tb.build_tree(bt, nullptr, kExtraBLBits, 0, kBLCodes, kMaxBLBits);
        int max_blindex;
        for (max_blindex = kBLCodes - 1; max_blindex >= 3; max_blindex--)
            if (bt.len[kBLOrder[max_blindex]] != 0) break;
        tb.opt_len += 3 * ((uint64_t)max_blindex + 1) + 5 + 5 + 4;
        uint64_t opt_lenb = (tb.opt_len + 3 + 7) >> 3;
        const uint64_t static_lenb = (tb.static_len + 3 + 7) >> 3;
        if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
        const uint64_t stored_len = (uint64_t)(b.p1 - b.p0);
        if (stored_len + 4 <= opt_lenb && b.buf_ok) {
            b.type = kStored;
            b.bits = -1;
        } else if (static_lenb == opt_lenb) {
            b.type = kFixed;
            b.bits = 3 + (int64_t)tb.static_len;
        } else {
            b.type = kDynamic;
            b.bits = 3 + (int64_t)tb.opt_len;
        }
        pl.lmax = (int16_t)lt.max_code;
        pl.dmax = (int16_t)dt.max_code;
        pl.maxbl = (int16_t)max_blindex;
        for (int n = 0; n <= lt.max_code; ++n) pl.llen[n] = (uint8_t)lt.len[n];
        for (int n = 0; n <= dt.max_code; ++n) pl.dlen[n] = (uint8_t)dt.len[n];
        for (int n = 0; n < kBLCodes; ++n) pl.bllen[n] = (uint8_t)bt.len[n];
    }
    static void codes_of(const uint8_t* lens, int max_code, uint16_t* len, uint16_t* code) {
        uint16_t bl_count[kMaxBits + 1] = {0};
        for (int n = 0; n <= max_code; ++n) {
            len[n] = lens[n];
            bl_count[lens[n]]++;
        }
        bl_count[0] = 0;
        Static::gen_codes(len, code, max_code, bl_count);
    }
    // encode at bit phase b.off % 8 into b.bytes; returns the bits written (header included)
    int64_t encode(Block& b, const Plan& pl) const {
        const Static& st = tables();
        const int phase = (int)(b.off & 7);
        const int64_t nbits = b.bits;
        b.bytes.resize((size_t)((phase + nbits + 7) / 8 + 16));
        b.bytes[0] = 0;
        BitW bw(b.bytes.data(), phase);
        if (b.type == kStored) {
            bw.put((0 << 1) + (b.last ? 1 : 0), 3);
            bw.align();
            const uint32_t n = (uint32_t)(b.p1 - b.p0);
            bw.put(n & 0xFFFF, 16);
            bw.put(~n & 0xFFFF, 16);
            bw.flush_partial();
            std::memcpy(bw.p, S + b.p0, (size_t)n);
            return nbits;
        }
        TreeDesc lt, dt, bt;
        const uint16_t *lcode, *llen, *dcode, *dlen;
        if (b.type == kFixed) {
            bw.put((1 << 1) + (b.last ? 1 : 0), 3);
            lcode = st.sl_code, llen = st.sl_len, dcode = st.sd_code, dlen = st.sd_len;
        } else {
            bw.put((2 << 1) + (b.last ? 1 : 0), 3);
            codes_of(pl.llen, pl.lmax, lt.len, lt.code);
            codes_of(pl.dlen, pl.dmax, dt.len, dt.code);
            codes_of(pl.bllen, kBLCodes - 1, bt.len, bt.code);
            lt.len[pl.lmax + 1] = 0xffff;   // scan_tree's guards, as send_tree reads them
            dt.len[pl.dmax + 1] = 0xffff;
            const int lcodes = pl.lmax + 1, dcodes = pl.dmax + 1, blcodes = pl.maxbl + 1;
            bw.put((uint32_t)(lcodes - 257), 5);
            bw.put((uint32_t)(dcodes - 1), 5);
            bw.put((uint32_t)(blcodes - 4), 4);
            for (int rank = 0; rank < blcodes; rank++) bw.put(bt.len[kBLOrder[rank]], 3);
            send_tree(bw, lt, lcodes - 1, bt);
            send_tree(bw, dt, dcodes - 1, bt);
            lcode = lt.code, llen = lt.len, dcode = dt.code, dlen = dt.len;
        }
        if (b.g1 > b.g0)
            each_symbol(b, pl.run, pl.word, [&](bool m, int a, int d) {
                if (!m) {
                    bw.put(lcode[a], llen[a]);
                    return;
                }
                int code = st.length_code[a];
                bw.put(lcode[code + 257], llen[code + 257]);
                int extra = kExtraLBits[code];
                if (extra) bw.put((uint32_t)(a - st.base_length[code]), extra);
                const int dist = d - 1;
                code = st.d_code(dist);
                bw.put(dcode[code], dlen[code]);
                extra = kExtraDBits[code];
                if (extra) bw.put((uint32_t)(dist - st.base_dist[code]), extra);
            });
        bw.put(lcode[kEndBlock], llen[kEndBlock]);
        const int64_t written = (int64_t)(bw.p - b.bytes.data()) * 8 + bw.nb - phase;
        bw.flush_partial();
        return written;
    }
};

// ---- driver ----------------------------------------------------------------------------------------
template <class F>
inline void parallel(int n, int threads, F&& f) {   // a worker's exception is rethrown here
    fnpz_internal::run_parallel(n, threads, std::forward<F>(f));
}

// Release big buffers off the caller's critical path: returning 1-2 GB to the OS (munmap, serial under
// the process's mmap lock) took ~0.1 s at the end of a 100 M-param save (profiles/r06_save_phases.log).
// The object is moved into a detached thread that drops it; if no thread can be had, it is dropped here.
template <class T>
inline void free_later(T&& obj) {
    try {
        std::thread([o = std::move(obj)]() mutable { T().swap(o); }).detach();
    } catch (const std::exception&) {
    }
}

struct Stats {
    int chunks = 0, fixups = 0, blocks = 0;
    double t_parse = 0, t_sync = 0, t_sched = 0, t_plan = 0, t_encode = 0;
    int64_t tail_from = 0;
    int64_t out_len = 0;               // bytes of the stream (in out, or at dst)
    const char* fallback = nullptr;   // why the caller must run zlib itself
};

// The raw deflate stream zlib 1.2.11 (level 6, memLevel 8, default strategy, wbits -15) produces for
// S[0, L) fed as deflate(Z_NO_FLUSH) calls ending at `ends` and then deflate(Z_FINISH). False (with
// st->fallback set) if this input needs zlib itself. The stream goes to `out`, or — with dst — straight
// to dst[0, st->out_len) (false, "no room", if it needs more than dst_cap bytes): the archive writer
// encodes a big member in place, with no copy of the stream afterwards.
inline bool deflate_exact(const uint8_t* S, int64_t L, const std::vector<int64_t>& ends, int threads, int64_t chunk,
                          Bytes& out, Stats* st, uint8_t* dst = nullptr, int64_t dst_cap = 0) {
    Stats dummy;
    if (!st) st = &dummy;
    if (chunk < kMinChunk) chunk = kMinChunk;
    if (L < 2 * chunk || L < 2 * kTailRec || ends.empty() || ends.back() != L) {
        st->fallback = "too small";
        return false;
    }
    // a whole number of chunks per thread (the parse is most of the time: a last round with a few
    // chunks would leave the other threads idle), each near the requested size
    int64_t T0 = std::min<int64_t>(L / chunk, 1 << 20);
    if (threads > 1 && T0 > threads) {
        const int64_t k = std::max<int64_t>(1, (T0 + threads / 2) / threads);
        const int64_t Tk = std::min<int64_t>(k * threads, L / kMinChunk);
        if (Tk >= 2 && 2 * kTailRec <= L / Tk * Tk) T0 = Tk, chunk = L / Tk;
    }
    const int T = (int)T0;
    std::vector<Chunk> C((size_t)T);
    for (int i = 0; i < T; ++i) {
        C[i].b = (int64_t)i * chunk;
        C[i].e = i + 1 < T ? (int64_t)(i + 1) * chunk : L;
        C[i].last = i + 1 == T;
    }
    st->chunks = T;
    struct Free {
        std::vector<Chunk>& c;
        ~Free() {
            for (auto& x : c) delete x.P;
        }
    } free_parsers{C};
    // 1. speculative parses, then each chunk extends its own parse into the next until they meet;
    // one that has not met by the end of the next chunk goes on (in order) through the chunks after
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t0 = now();
    parallel(T, threads, [&](int i) { parse_chunk(C[i], S, L); });
    st->t_parse = now() - t0;
    t0 = now();
    // (syncs are looked for before the tail region only: a parse that has not met another there
    // becomes the tail's source itself, its final tops recorded)
    parallel(T - 1, threads, [&](int i) { extend(C[i], C, i + 1, std::min(C[i + 1].stop, L - kTailRec)); });
    for (int i = 0; i + 1 < T;) {
        if (!C[i].synced) {
            ++st->fixups;
            if (!extend(C[i], C, i + 1, L - kTailRec)) {   // periodic to the end: this parse is the rest
                Chunk& k = C[i];
                Parser& P = *k.P;
                while (P.t < L - kTailStop) {
                    if (P.t >= L - kTailRec) k.rec_tail.push_back(P.rec(k.ext));
                    P.step(k.ext);
                }
                k.ext_final = true;
                k.ext_p1 = P.t - P.avail;
                break;
            }
        }
        i = C[i].sync_chunk;
    }
    st->t_sync = now() - t0;
    t0 = now();
    // the chain of runs (the last chunk's spec is cut at the tail hand-over below)
    Runs R;
    int c = 0;
    size_t w0 = 0;
    int64_t s0 = 0, p0 = 0;
    // the parse the tail hands over from: the last chunk's speculative one, or an extension that
    // never met one
    const Syms* src = nullptr;
    const std::vector<Rec>* src_rec = nullptr;
    int64_t src_p1 = 0;
    for (;;) {
        Chunk& k = C[c];
        if (k.last) {
            src = &k.spec, src_rec = &k.rec_tail, src_p1 = k.spec_p1;
            break;
        }
        R.add(&k.spec, w0, k.spec.n, s0, k.spec.nsym, p0, k.spec_p1);
        if (k.ext_final) {
            src = &k.ext, src_rec = &k.rec_tail, src_p1 = k.ext_p1;
            w0 = 0, s0 = 0, p0 = k.spec_p1;
            break;
        }
        R.add(&k.ext, 0, k.ext_words, 0, k.ext_syms, k.spec_p1, k.sync_pos);
        c = k.sync_chunk;
        w0 = k.sync_word;
        s0 = k.sync_sym;
        p0 = k.sync_pos;
    }
    // 2. the window schedule (fill calls and slides) up to the tail's first recorded top at or after
    // the source's sync point; the tail is replayed from there with a real window
    const auto& RT = *src_rec;
    size_t hi_idx = 0;
    while (hi_idx < RT.size() && RT[hi_idx].t < p0) ++hi_idx;
    if (hi_idx >= RT.size()) {
        st->fallback = "no recorded top for the tail";
        return false;
    }
    const Rec* handover = &RT[hi_idx];
    Feed F{&ends};
    {
        Runs Q = R;   // provisional: the whole source parse, for top queries
        Q.add(src, w0, src->n, s0, src->nsym, p0, src_p1);
        int64_t t = 0;
        while (t < handover->t) {
            F.top(t);
            // the slide corner: a slide exactly at wsize + MAX_DIST whose hash head is the new window
            // start (zlib sees NIL there, stream offsets would not)
            if (!F.slides.empty() && F.slides.back() == t && t - (F.w_base - kWSize) == kWSize + kMaxDist) {
                const uint32_t h = hash3(S + t);
                int64_t q = t - 1;
                while (q > F.w_base && hash3(S + q) != h) --q;
                if (q == F.w_base && hash3(S + q) == h) {
                    st->fallback = "slide corner";
                    return false;
                }
            }
            t = Q.top_at_or_after(F.read_end - kMinLookahead + 1);   // the next top short of lookahead
            if (t < 0) break;
        }
    }
    st->tail_from = handover->t;
    R.add(src, w0, handover->word, s0, handover->nsym, p0, handover->t - handover->avail);
    Tail tail(S, L, F);
    tail.start(*handover);
    tail.run();
    R.add(&tail.out, 0, tail.out.n, 0, tail.out.nsym, handover->t - handover->avail, L);
    st->t_sched = now() - t0;
    t0 = now();
    // 3. blocks
    const int64_t N = R.total();
    std::vector<Block> B;
    {
        int64_t g = 0;
        while (true) {
            const int64_t nxt = g + kBlockSyms;
            if (nxt < N || (nxt == N && !tail.final_literal)) {
                Block b;
                b.g0 = g;
                b.g1 = nxt;
                B.push_back(b);
                g = nxt;
            } else {
                Block b;
                b.g0 = g;
                b.g1 = N;
                b.last = true;
                B.push_back(b);
                break;
            }
        }
    }
    st->blocks = (int)B.size();
    const std::vector<int64_t>& slides = F.slides;
    auto w_base_at = [&](int64_t top) {   // slides at tops <= top
        return (int64_t)(std::upper_bound(slides.begin(), slides.end(), top) - slides.begin()) * kWSize;
    };
    // positions: each block ends where its last symbol ends; the window base at its flush decides
    // whether a stored block is allowed (block_start >= 0 in window coordinates)
    std::vector<int64_t> flush_base(B.size());
    parallel((int)B.size(), threads, [&](int i) {
        Block& b = B[i];
        if (b.last || b.g1 <= b.g0) {
            b.p1 = L;
            flush_base[i] = F.w_base;
            return;
        }
        const Cursor e = R.at_global(b.g1 - 1);
        b.p1 = e.pos + sym_len(R.r[e.run].s->w.data(), e.word);
        flush_base[i] = w_base_at(e.pos + 1);   // the iteration that tallied it
    });
    for (size_t i = 0; i < B.size(); ++i) {
        B[i].p0 = i ? B[i - 1].p1 : 0;
        B[i].buf_ok = B[i].p0 >= flush_base[i];
    }
    std::vector<Plan> plans(B.size());
    Encoder E(R, S);
    parallel((int)B.size(), threads, [&](int i) { E.plan(B[i], plans[i]); });
    st->t_plan = now() - t0;
    t0 = now();
    int64_t off = 0;
    for (auto& b : B) {
        b.off = off;
        if (b.type == kStored) {
            const int64_t after_hdr = off + 3;
            const int64_t aligned = (after_hdr + 7) & ~int64_t(7);
            b.bits = aligned - off + 32 + 8 * (b.p1 - b.p0);
            if (b.p1 - b.p0 > 0xFFFF) {
                st->fallback = "stored block over 64 KiB";
                return false;
            }
        }
        off += b.bits;
    }
    const int64_t total_bits = off;
    std::atomic<int> bad{0};
    const int64_t nbytes = (total_bits + 7) / 8;
    if (dst && nbytes > dst_cap) {
        st->fallback = "no room";
        return false;
    }
    if (!dst) out.resize((size_t)nbytes);       // every byte is written below (no zero fill)
    uint8_t* const O = dst ? dst : out.data();
    st->out_len = nbytes;
    parallel((int)B.size(), threads, [&](int i) {
        Block& b = B[i];
        const int64_t got = E.encode(b, plans[i]);
        if (got != b.bits) bad.fetch_add(1);
        // bytes after the first go straight out; the shared first byte is merged below
        const int64_t first = b.off >> 3, lastb = (b.off + b.bits - 1) >> 3;
        if (lastb > first) std::memcpy(O + first + 1, b.bytes.data() + 1, (size_t)(lastb - first));
    });
    if (bad.load()) {
        st->fallback = "internal size mismatch";
        return false;
    }
    for (auto& b : B) {
        const int64_t first = b.off >> 3;
        if ((b.off & 7) == 0) O[first] = b.bytes[0];
        else O[first] |= b.bytes[0];
        std::vector<uint8_t>().swap(b.bytes);
    }
    st->t_encode = now() - t0;
    for (auto& x : C) {                 // the parsers (small), then the symbol streams off the critical path
        delete x.P;
        x.P = nullptr;
    }
    free_later(std::move(C));
    return true;
}

}  // namespace pdef
