// Raw DEFLATE (RFC 1951) decoder and CRC-32 for the npz codec's whole-member reads.
//
// FEDn's clients write updates with np.savez_compressed (numpyhelper.py:144-169): every member is ONE
// deflate stream, so its decode runs on one core and bounds Helper.load / load_model_update. zlib's
// inflate moves one symbol per table lookup through a 32-bit window it refills a byte at a time;
// this decoder keeps a 64-bit bit buffer refilled with one unaligned load, decodes up to three
// literals per refill through 11-bit root tables (one lookup for all codes of <= 11 bits), and copies
// matches 8 bytes at a time. It is resumable at any output position (run() stops when the output
// window is full and continues on the next call, a match split across calls included), so the .npy
// header and the payload land in separate buffers and the CRC is taken over each piece while it is
// still in cache. CRC-32 (the zip polynomial, reflected) folds 64 bytes per step with carry-less
// multiplies (PCLMULQDQ) where the CPU has them.
//
// Acceptance follows zlib: over-subscribed codes, incomplete codes (except a single one-bit code),
// a literal/length code without end-of-block, repeat codes with no previous length, distances
// before the start of the output, invalid symbols (286/287, 30/31) and truncated input are errors.
#pragma once

#include <algorithm>
#include <vector>
#include <cstddef>
#include <cstdint>
#include <cstring>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace fnpz_fast {

// ---------------------------------------------------------------------------------------
// CRC-32 (0x04C11DB7 reflected; zlib's crc32 convention: pass the previous return value)
// ---------------------------------------------------------------------------------------
struct CrcTables {
    uint32_t t[8][256];
    CrcTables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
    }
};

inline const CrcTables& crc_tables() {
    static const CrcTables tabs;
    return tabs;
}

// slicing-by-8 over the bit-inverted state
inline uint32_t crc32_sb8(uint32_t c, const uint8_t* p, size_t n) {
    const CrcTables& T = crc_tables();
    while (n >= 8) {
        uint32_t lo, hi;
        std::memcpy(&lo, p, 4);
        std::memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = T.t[7][lo & 0xFF] ^ T.t[6][(lo >> 8) & 0xFF] ^ T.t[5][(lo >> 16) & 0xFF] ^ T.t[4][lo >> 24] ^
            T.t[3][hi & 0xFF] ^ T.t[2][(hi >> 8) & 0xFF] ^ T.t[1][(hi >> 16) & 0xFF] ^ T.t[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = T.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    return c;
}

#if defined(__x86_64__)
// Attribution: this routine follows the published PCLMULQDQ CRC folding method — V. Gopal et al.,
// "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ Instruction" (Intel white paper,
// 2009) — in the form of Chromium's zlib crc32_sse42_simd_() (third_party/zlib/crc32_simd.c,
// Copyright 2017 The Chromium Authors, BSD-style license: "Use of this source code is governed by
// a BSD-style license that can be found in the Chromium source repository LICENSE file"), whose
// constant names (k1k2, k3k4, k5k0, poly, mask32) and fold / Barrett sequence it keeps. The
// constants are the CRC-32 (0xEDB88320) values that method defines.
// Fold-by-4 over 128-bit lanes, then 128 -> 64 -> 32 bits by Barrett reduction (the constants are
// x^(4*128+64) mod P, x^(4*128) mod P, x^(128+64) mod P, x^128 mod P, x^64 mod P, P' and mu for the
// reflected polynomial). ``n`` is a multiple of 16 and at least 64; ``c`` the bit-inverted state.
__attribute__((target("pclmul,sse4.1"))) inline uint32_t crc32_clmul(uint32_t c, const uint8_t* p, size_t n) {
    const __m128i k1k2 = _mm_set_epi64x(0x01c6e41596LL, 0x0154442bd4LL);
    const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009eLL, 0x01751997d0LL);
    const __m128i k5k0 = _mm_set_epi64x(0, 0x0163cd6124LL);
    const __m128i poly = _mm_set_epi64x(0x01f7011641LL, 0x01db710641LL);
    const __m128i mask32 = _mm_setr_epi32(-1, 0, -1, 0);
    __m128i x1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    __m128i x2 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16));
    __m128i x3 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 32));
    __m128i x4 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 48));
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)c));
    p += 64;
    n -= 64;
    while (n >= 64) {
        const __m128i x5 = _mm_clmulepi64_si128(x1, k1k2, 0x00), x6 = _mm_clmulepi64_si128(x2, k1k2, 0x00);
        const __m128i x7 = _mm_clmulepi64_si128(x3, k1k2, 0x00), x8 = _mm_clmulepi64_si128(x4, k1k2, 0x00);
        x1 = _mm_clmulepi64_si128(x1, k1k2, 0x11);
        x2 = _mm_clmulepi64_si128(x2, k1k2, 0x11);
        x3 = _mm_clmulepi64_si128(x3, k1k2, 0x11);
        x4 = _mm_clmulepi64_si128(x4, k1k2, 0x11);
        x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128(reinterpret_cast<const __m128i*>(p)));
        x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16)));
        x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 32)));
        x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 48)));
        p += 64;
        n -= 64;
    }
    __m128i x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k3k4, 0x11), x2), x5);
    x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k3k4, 0x11), x3), x5);
    x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k3k4, 0x11), x4), x5);
    while (n >= 16) {
        x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00);
        x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k3k4, 0x11),
                                         _mm_loadu_si128(reinterpret_cast<const __m128i*>(p))), x5);
        p += 16;
        n -= 16;
    }
    // 128 -> 64 bits
    __m128i x2b = _mm_clmulepi64_si128(x1, k3k4, 0x10);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2b);
    x2b = _mm_srli_si128(x1, 4);
    x1 = _mm_and_si128(x1, mask32);
    x1 = _mm_xor_si128(_mm_clmulepi64_si128(x1, k5k0, 0x00), x2b);
    // Barrett reduction to 32 bits
    x2b = _mm_and_si128(x1, mask32);
    x2b = _mm_clmulepi64_si128(x2b, poly, 0x10);
    x2b = _mm_and_si128(x2b, mask32);
    x2b = _mm_clmulepi64_si128(x2b, poly, 0x00);
    x1 = _mm_xor_si128(x1, x2b);
    return (uint32_t)_mm_extract_epi32(x1, 1);
}

inline bool have_clmul() {
    static const bool ok = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    return ok;
}
#endif

// zlib-compatible: crc32(0, p, n) is the CRC of p; crc32(crc32(0, a), b) that of a || b
inline uint32_t crc32(uint32_t crc, const uint8_t* p, size_t n) {
    uint32_t c = ~crc;
#if defined(__x86_64__)
    if (n >= 64 && have_clmul()) {
        const size_t m = n & ~(size_t)15;
        c = crc32_clmul(c, p, m);
        p += m;
        n -= m;
    }
#endif
    return ~crc32_sb8(c, p, n);
}

// ---------------------------------------------------------------------------------------
// DEFLATE decoder
// ---------------------------------------------------------------------------------------
// decode table entry: bits 0-4 code length (bits consumed), 8-11 extra bits (or a subtable's index
// bits), 16-30 value (literal byte, length / distance base, subtable offset), and one flag per kind
// so the hot loop tests a single bit: bit 31 literal (the sign: one test), 5 subtable, 6
// end-of-block, 7 length, 12 distance; no flag = an invalid code
enum : uint32_t { K_INVALID = 0, K_LIT = 1, K_LEN = 2, K_EOB = 3, K_SUB = 4, K_DIST = 5 };
constexpr uint32_t F_LIT = 1u << 31, F_SUB = 1u << 5, F_EOB = 1u << 6, F_LEN = 1u << 7, F_DIST = 1u << 12;
#ifndef FNPZ_LIT_ROOT
#define FNPZ_LIT_ROOT 11                  // root bits of the literal/length table (tools: build variants)
#endif
constexpr int kLitRoot = FNPZ_LIT_ROOT, kDistRoot = 8, kPreRoot = 7;
constexpr int kLitTable = (1 << kLitRoot) + 288 * (1 << (15 - kLitRoot)), kDistTable = (1 << kDistRoot) + 32 * 128;

inline uint32_t entry(uint32_t len, uint32_t kind, uint32_t extra, uint32_t value) {
    static const uint32_t flag[6] = {0, F_LIT, F_LEN, F_EOB, F_SUB, F_DIST};
    return len | flag[kind] | (extra << 8) | (value << 16);
}
inline uint32_t e_len(uint32_t e) { return e & 31; }
inline uint32_t e_kind(uint32_t e) {
    return (e & F_LIT) ? K_LIT : (e & F_SUB) ? K_SUB : (e & F_LEN) ? K_LEN : (e & F_EOB) ? K_EOB : (e & F_DIST) ? K_DIST : K_INVALID;
}
inline uint32_t e_extra(uint32_t e) { return (e >> 8) & 15; }
inline uint32_t e_value(uint32_t e) { return (e >> 16) & 0x7FFF; }

static const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                       193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

enum class Alphabet { kLitLen, kDist, kPre };

inline uint32_t sym_entry(Alphabet a, int sym, uint32_t len) {
    switch (a) {
        case Alphabet::kLitLen:
            if (sym < 256) return entry(len, K_LIT, 0, (uint32_t)sym);
            if (sym == 256) return entry(len, K_EOB, 0, 0);
            if (sym <= 285) return entry(len, K_LEN, kLenExtra[sym - 257], kLenBase[sym - 257]);
            return entry(len, K_INVALID, 0, 0);
        case Alphabet::kDist:
            if (sym < 30) return entry(len, K_DIST, kDistExtra[sym], kDistBase[sym]);
            return entry(len, K_INVALID, 0, 0);
        default:
            return entry(len, K_LIT, 0, (uint32_t)sym);
    }
}

struct Rev8 {
    uint8_t t[256];
    Rev8() {
        for (int i = 0; i < 256; ++i) {
            int r = 0;
            for (int b = 0; b < 8; ++b) r |= ((i >> b) & 1) << (7 - b);
            t[i] = (uint8_t)r;
        }
    }
};

// the low n (<= 16) bits of c, reversed (deflate packs Huffman codes most-significant bit first)
inline uint32_t reverse_bits(uint32_t c, int n) {
    static const Rev8 rev;
    return (((uint32_t)rev.t[c & 0xFF] << 8) | rev.t[(c >> 8) & 0xFF]) >> (16 - n);
}

// Canonical Huffman table of ``n`` code lengths (0 = unused) with a ``root``-bit first level and
// second-level subtables for longer codes. Returns false for a set zlib rejects.
inline bool build_table(const uint8_t* lens, int n, Alphabet a, int root, uint32_t* table, int cap) {
    int count[16] = {0};
    int maxlen = 0;
    for (int s = 0; s < n; ++s) {
        if (lens[s] > 15) return false;
        count[lens[s]]++;
        if (lens[s] > maxlen) maxlen = lens[s];
    }
    if (maxlen == 0) {                                                    // no codes (an all-literal block's distances)
        std::memset(table, 0, sizeof(uint32_t) * (size_t)(1 << root));   // K_INVALID everywhere
        return a != Alphabet::kPre;
    }
    count[0] = 0;
    int left = 1;
    for (int l = 1; l <= 15; ++l) {
        left <<= 1;
        left -= count[l];
        if (left < 0) return false;                                        // over-subscribed
    }
    if (left > 0 && (a == Alphabet::kPre || maxlen != 1)) return false;   // incomplete (zlib's rule)
    // a complete code fills every entry below; only the one incomplete case zlib allows (a single
    // one-bit code) leaves entries that must read as invalid
    if (left > 0) std::memset(table, 0, sizeof(uint32_t) * (size_t)(1 << root));
    int next[16];
    int code = 0;
    for (int l = 1; l <= 15; ++l) {
        code = (code + count[l - 1]) << 1;
        next[l] = code;
    }
    // subtable geometry: the longest code under each root prefix
    static thread_local uint8_t sublen[1 << kLitRoot];
    static thread_local int32_t suboff[1 << kLitRoot];
    const int rsize = 1 << root;
    if (maxlen > root) {
        std::memset(sublen, 0, (size_t)rsize);
        int tmp[16];
        std::memcpy(tmp, next, sizeof(tmp));
        for (int s = 0; s < n; ++s) {
            const int l = lens[s];
            if (l > root) {
                const uint32_t rev = reverse_bits((uint32_t)tmp[l], l);
                const uint32_t pre = rev & (uint32_t)(rsize - 1);
                if (l - root > sublen[pre]) sublen[pre] = (uint8_t)(l - root);
            }
            if (l) tmp[l]++;
        }
        int off = rsize;
        for (int p = 0; p < rsize; ++p) {
            if (!sublen[p]) continue;
            suboff[p] = off;
            off += 1 << sublen[p];
            if (off > cap) return false;
            table[p] = entry(0, K_SUB, sublen[p], (uint32_t)suboff[p]);     // (complete: filled below)
        }
    }
    for (int s = 0; s < n; ++s) {
        const int l = lens[s];
        if (!l) continue;
        const uint32_t rev = reverse_bits((uint32_t)next[l]++, l);
        const uint32_t e = sym_entry(a, s, (uint32_t)l);
        if (l <= root) {
            for (uint32_t i = rev; i < (uint32_t)rsize; i += 1u << l) table[i] = e;
        } else {
            const uint32_t pre = rev & (uint32_t)(rsize - 1);
            const int sb = sublen[pre];
            uint32_t* sub = table + suboff[pre];
            for (uint32_t i = rev >> root; i < (1u << sb); i += 1u << (l - root)) sub[i] = e;
        }
    }
    return true;
}

class Inflate {
  public:
    enum Status { kOk = 0, kFull = 1, kEnd = 2, kNeed = 3, kStop = 4, kSwitch = 5, kCorrupt = -1 };
    static constexpr uint64_t kNoStop = ~(uint64_t)0;

    Inflate(const uint8_t* in, size_t n) : in_(in), in_end_(in + n), in_start_(in) {}

    // Streaming input (an archive arriving in pieces): the unconsumed input continues at [in, end)
    // — the bytes after the last call's input_pos(), possibly moved. Not ``final``: more input may
    // follow, so run() returns kNeed instead of decoding a symbol or block header that might run
    // past ``end`` (it keeps >= 56 bits, or >= 700 bytes before a block header, buffered ahead).
    void set_input(const uint8_t* in, const uint8_t* end, bool final) {
        in_ = in;
        in_end_ = end;
        in_start_ = in;
        more_ = !final;
    }
    // the next input byte not loaded into the bit buffer yet
    const uint8_t* input_pos() const { return in_; }

    // ---- parallel decode of one stream (npz_codec.cpp inflate_parallel) ----------------------
    // Restart at bit ``bit`` of the input (a block header there), every state reset.
    void restart_at(uint64_t bit) {
        in_ = in_start_ + bit / 8;
        bits_ = 0;
        nbits_ = 0;
        zeros_ = 0;
        state_ = kHeader;
        final_ = false;
        more_ = false;
        stored_left_ = 0;
        pend_len_ = pend_dist_ = 0;
        err_line_ = 0;
        last_marker_ = 32767;                                   // run_markers(): the window's markers
        if (bit % 8) {
            need((unsigned)(bit % 8));
            drop((unsigned)(bit % 8));
        }
    }
    // Could a dynamic-Huffman block header start at input bit ``bit``? The cheap field checks only
    // (type 2, <= 286 literal/length and <= 30 distance codes, a complete precode); the block
    // finder then parses and trial-decodes the survivors.
    static bool maybe_dynamic_header(const uint8_t* base, size_t n, uint64_t bit) {
        const size_t byte = (size_t)(bit / 8);
        if (byte + 11 > n) return false;
        uint64_t v;
        std::memcpy(&v, base + byte, 8);
        v >>= bit % 8;                                          // >= 56 valid bits
        if (((v >> 1) & 3) != 2) return false;
        if (((v >> 3) & 31) > 29 || ((v >> 8) & 31) > 29) return false;
        const int hclen = (int)((v >> 13) & 15) + 4;
        static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        // the precode lengths: bits 17 .. 17 + 3 * hclen (up to 57 of them) — one 64-bit load holds
        // 64 - ((bit % 8) + 1) >= 56, so the 19th length's last bit comes from the next byte then
        uint64_t w;
        std::memcpy(&w, base + byte + 2, 8);
        const int sh = (int)(bit % 8) + 1;
        w >>= sh;
        if (sh > 7) w |= (uint64_t)base[byte + 10] << (64 - sh);
        int count[8] = {0};
        for (int i = 0; i < hclen; ++i) count[(w >> (3 * i)) & 7]++;
        (void)order;
        int left = 1;
        for (int l = 1; l <= 7; ++l) {
            left = (left << 1) - count[l];
            if (left < 0) return false;
        }
        return left == 0;                                       // zlib: the precode must be complete
    }

    // run() / run_markers() return kStop at the block header at input bit ``bit`` (kCorrupt if a
    // block runs past it: it was not a block boundary of this stream)
    void stop_at(uint64_t bit) { stop_bit_ = bit; }
    uint64_t bit_pos() const { return (uint64_t)(in_ - in_start_) * 8 + (uint64_t)zeros_ * 8 - nbits_; }

    // Marker mode: decode with the 32 KiB before the start unknown. ``out`` starts with 32768
    // markers, value 256 + i standing for byte i of that unknown window; literals append their
    // byte, copies copy values (markers included), so every output value is a byte or the marker
    // of the window byte it equals. Returns kSwitch once the last 32 KiB of output hold no marker
    // (the byte decoder can take over: run() with those bytes as its window), kStop / kEnd /
    // kCorrupt as run(), kFull past ``max_out`` values.
    int run_markers(std::vector<uint16_t>& out, size_t max_out) {
        for (;;) {
            if (out.size() >= 65536 && out.size() - 1 - last_marker_ >= 32768) return kSwitch;
            if (out.size() >= max_out) return kFull;
            if (state_ == kHeader) {
                if (stop_bit_ != kNoStop) {
                    const uint64_t b = bit_pos();
                    if (b == stop_bit_) return kStop;
                    if (b > stop_bit_) return corrupt(__LINE__);
                }
                if (final_) return kEnd;
                if (!need(3)) return corrupt(__LINE__);
                final_ = (bits_ & 1) != 0;
                const uint32_t type = (uint32_t)(bits_ >> 1) & 3;
                drop(3);
                if (type == 0) {
                    if (!start_stored()) return corrupt(__LINE__);
                } else if (type == 1) {
                    fixed_tables();
                    state_ = kHuff;
                } else if (type == 2) {
                    if (!dynamic_tables()) return corrupt(__LINE__);
                    state_ = kHuff;
                } else {
                    return corrupt(__LINE__);
                }
                continue;
            }
            if (state_ == kStored) {
                while (stored_left_ && in_ < in_end_ && out.size() < max_out) {
                    out.push_back(*in_++);
                    --stored_left_;
                }
                if (stored_left_) {
                    if (out.size() >= max_out) return kFull;
                    return corrupt(__LINE__);
                }
                state_ = kHeader;
                continue;
            }
            // one Huffman symbol
            if (!refill_slow()) return corrupt(__LINE__);
            const uint32_t e = lit_entry();
            if (e & F_LIT) {
                drop(e_len(e));
                if (overran()) return corrupt(__LINE__);
                out.push_back((uint16_t)e_value(e));
                continue;
            }
            if (e & F_EOB) {
                drop(e_len(e));
                if (overran()) return corrupt(__LINE__);
                state_ = kHeader;
                continue;
            }
            if (!(e & F_LEN)) return corrupt(__LINE__);
            drop(e_len(e));
            const uint32_t xb = e_extra(e);
            const size_t len = e_value(e) + ((uint32_t)bits_ & ((1u << xb) - 1));
            drop(xb);
            const uint32_t d = dist_entry();
            if (!(d & F_DIST)) return corrupt(__LINE__);
            drop(e_len(d));
            const uint32_t db = e_extra(d);
            const size_t dist = e_value(d) + ((uint32_t)bits_ & ((1u << db) - 1));
            drop(db);
            if (overran() || dist > out.size()) return corrupt(__LINE__);
            for (size_t k = 0; k < len; ++k) {
                const uint16_t v = out[out.size() - dist];
                if (v >= 256) last_marker_ = out.size();
                out.push_back(v);
            }
        }
    }

    // Decode into [*out, out_end): returns kFull when the window is full (call again with the next
    // window), kEnd after the final block (the stream's output is complete), kCorrupt on an invalid
    // or truncated stream. ``win_start``: the first byte back-references may reach (the output's
    // start, or any point with >= 32 KiB of output before it in the same buffer). *out is advanced.
    int run(uint8_t** outp, uint8_t* out_end, const uint8_t* win_start) {
        uint8_t* out = *outp;
        int rc = kOk;
        for (;;) {
            if (pend_len_) {                                      // a match split by the last window
                if (pend_dist_ > (size_t)(out - win_start)) { rc = corrupt(__LINE__); break; }
                while (pend_len_ && out < out_end) {
                    *out = out[-(ptrdiff_t)pend_dist_];
                    ++out;
                    --pend_len_;
                }
                if (pend_len_) { rc = kFull; break; }
            }
            if (state_ == kHeader) {
                if (stop_bit_ != kNoStop) {
                    const uint64_t b = bit_pos();
                    if (b == stop_bit_) { rc = kStop; break; }
                    if (b > stop_bit_) { rc = corrupt(__LINE__); break; }
                }
                if (final_) { rc = kEnd; break; }
                // a full window at the end of a non-final range (a block of a sync-flushed stream,
                // read on its own): nothing more to decode here
                if (out == out_end && !input_left(3)) { rc = kFull; break; }
                // a dynamic header is < 600 bytes: with more input to come, start a block only
                // when it cannot run past the input at hand
                if (more_ && !input_left(8 * 700)) { rc = kNeed; break; }
                if (!need(3)) { rc = corrupt(__LINE__); break; }
                final_ = (bits_ & 1) != 0;
                const uint32_t type = (uint32_t)(bits_ >> 1) & 3;
                drop(3);
                if (type == 0) {
                    if (!start_stored()) { rc = corrupt(__LINE__); break; }
                } else if (type == 1) {
                    fixed_tables();
                    state_ = kHuff;
                } else if (type == 2) {
                    if (!dynamic_tables()) { rc = corrupt(__LINE__); break; }
                    state_ = kHuff;
                } else {
                    rc = corrupt(__LINE__);
                    break;
                }
            }
            if (state_ == kStored) {
                const size_t room = (size_t)(out_end - out);
                const size_t k = std::min<size_t>({stored_left_, room, (size_t)(in_end_ - in_)});
                std::memcpy(out, in_, k);
                in_ += k;
                out += k;
                stored_left_ -= k;
                if (stored_left_) {
                    if (out == out_end) { rc = kFull; break; }
                    rc = more_ ? kNeed : corrupt(__LINE__);   // the input ran out inside the block
                    break;
                }
                state_ = kHeader;
                continue;
            }
            if (state_ == kHuff) {
                const int r = huffman(&out, out_end, win_start);
                if (r != kOk) { rc = r; break; }
                state_ = kHeader;                                  // end of block
            }
        }
        *outp = out;
        return rc;
    }

    // the decoder line that found the stream invalid (0: none), for error messages
    int error_line() const { return err_line_; }

    // input bytes the decode has consumed (after kEnd: the stream's length, its last byte included)
    size_t consumed() const {
        const size_t loaded = (size_t)(in_ - in_start_) * 8 + (size_t)zeros_ * 8;
        return (loaded - nbits_ + 7) / 8;
    }

  private:
    enum State { kHeader, kStored, kHuff };
    const uint8_t* in_;
    const uint8_t* in_end_;
    const uint8_t* in_start_;
    uint64_t bits_ = 0;
    unsigned nbits_ = 0;
    unsigned zeros_ = 0;                 // zero bytes fed past the end of the input (<= 8)
    State state_ = kHeader;
    bool final_ = false;
    bool more_ = false;                  // streaming input: more may follow the current end
    size_t stored_left_ = 0;
    size_t pend_len_ = 0, pend_dist_ = 0;
    int err_line_ = 0;
    uint64_t stop_bit_ = kNoStop;
    size_t last_marker_ = 0;             // run_markers(): index of the last marker written
    uint32_t lit_[kLitTable];
    uint32_t dist_[kDistTable];

    int corrupt(int line) {
        if (!err_line_) err_line_ = line;
        return kCorrupt;
    }
    // slow refill (a byte at a time, zeros past the end of the input) to 56..63 bits (never 64: the
    // fast refill shifts by nbits_). It fails only when a 9th phantom byte would be needed: 64
    // phantom bits against < 56 buffered means the decode has already consumed bits past the end,
    // i.e. the stream is truncated. Consuming phantom bits is caught by overran() where it matters.
    bool refill_slow() {
        while (nbits_ < 56) {
            if (in_ < in_end_) {
                bits_ |= (uint64_t)*in_++ << nbits_;
            } else {
                if (zeros_ >= 8) return false;
                ++zeros_;
            }
            nbits_ += 8;
        }
        return true;
    }
    // load real input bytes up to 56..63 buffered bits; whether that many are there
    bool fill_real() {
        while (nbits_ < 56 && in_ < in_end_) {
            bits_ |= (uint64_t)*in_++ << nbits_;
            nbits_ += 8;
        }
        return nbits_ >= 56;
    }
    // at least n real (not phantom) input bits not consumed yet
    bool input_left(unsigned n) const {
        return (size_t)(in_end_ - in_) * 8 + nbits_ >= (size_t)n + (size_t)zeros_ * 8;
    }
    // at least n (<= 56) bits buffered
    bool need(unsigned n) { return nbits_ >= n || refill_slow(); }
    void drop(unsigned n) {
        bits_ >>= n;
        nbits_ -= n;
    }
    bool overran() const { return (size_t)zeros_ * 8 > (size_t)nbits_; }

    bool start_stored() {
        drop(nbits_ & 7);                                           // to a byte boundary
        if (!need(32)) return false;
        const uint32_t len = (uint32_t)bits_ & 0xFFFF, nlen = (uint32_t)(bits_ >> 16) & 0xFFFF;
        drop(32);
        if (len != (~nlen & 0xFFFF)) return false;
        if (overran()) return false;
        // give back the whole bytes still buffered, then copy straight from the input
        const unsigned back = nbits_ / 8;
        const unsigned phantom = std::min(back, zeros_);
        in_ -= (back - phantom);
        zeros_ -= phantom;
        bits_ = 0;
        nbits_ = 0;
        if (zeros_) return false;
        stored_left_ = len;
        state_ = kStored;
        return true;
    }

    void fixed_tables() {
        uint8_t l[288 + 32];
        for (int i = 0; i < 144; ++i) l[i] = 8;
        for (int i = 144; i < 256; ++i) l[i] = 9;
        for (int i = 256; i < 280; ++i) l[i] = 7;
        for (int i = 280; i < 288; ++i) l[i] = 8;
        for (int i = 0; i < 32; ++i) l[288 + i] = 5;
        build_table(l, 288, Alphabet::kLitLen, kLitRoot, lit_, kLitTable);
        build_table(l + 288, 32, Alphabet::kDist, kDistRoot, dist_, kDistTable);
    }

    bool dynamic_tables() {
        static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        if (!need(14)) return false;
        const int hlit = (int)(bits_ & 31) + 257, hdist = (int)((bits_ >> 5) & 31) + 1, hclen = (int)((bits_ >> 10) & 15) + 4;
        drop(14);
        if (hlit > 286 || hdist > 30) return false;                // zlib: "too many length or distance symbols"
        uint8_t pl[19] = {0};
        for (int i = 0; i < hclen; ++i) {
            if (!need(3)) return false;
            pl[order[i]] = (uint8_t)(bits_ & 7);
            drop(3);
        }
        uint32_t pre[1 << kPreRoot];
        if (!build_table(pl, 19, Alphabet::kPre, kPreRoot, pre, 1 << kPreRoot)) return false;
        uint8_t l[286 + 30];
        int i = 0;
        while (i < hlit + hdist) {
            if (!need(7 + 7)) return false;                         // a code and its repeat bits
            const uint32_t e = pre[bits_ & ((1u << kPreRoot) - 1)];
            if (e_kind(e) == K_INVALID) return false;
            drop(e_len(e));
            const uint32_t sym = e_value(e);
            if (sym < 16) {
                l[i++] = (uint8_t)sym;
                continue;
            }
            int rep;
            uint8_t v = 0;
            if (sym == 16) {
                if (i == 0) return false;
                rep = 3 + (int)(bits_ & 3);
                drop(2);
                v = l[i - 1];
            } else if (sym == 17) {
                rep = 3 + (int)(bits_ & 7);
                drop(3);
            } else {
                rep = 11 + (int)(bits_ & 127);
                drop(7);
            }
            if (i + rep > hlit + hdist) return false;
            while (rep--) l[i++] = v;
        }
        if (overran()) return false;
        if (l[256] == 0) return false;                              // no end-of-block code
        if (!build_table(l, hlit, Alphabet::kLitLen, kLitRoot, lit_, kLitTable)) return false;
        if (!build_table(l + hlit, hdist, Alphabet::kDist, kDistRoot, dist_, kDistTable)) return false;
        return true;
    }

    static inline uint64_t load64(const uint8_t* p) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        return v;
    }

    inline uint32_t lit_entry() const {
        uint32_t e = lit_[bits_ & ((1u << kLitRoot) - 1)];
        if (e_kind(e) == K_SUB) e = lit_[e_value(e) + ((bits_ >> kLitRoot) & ((1u << e_extra(e)) - 1))];
        return e;
    }
    inline uint32_t dist_entry() const {
        uint32_t e = dist_[bits_ & ((1u << kDistRoot) - 1)];
        if (e_kind(e) == K_SUB) e = dist_[e_value(e) + ((bits_ >> kDistRoot) & ((1u << e_extra(e)) - 1))];
        return e;
    }

    // The fast loop: bit buffer, input pointer and tables in locals (a byte store through ``out``
    // may alias any member, so members would be reloaded after every literal). Runs while >= 16
    // input bytes remain (branch-free refills) and the window has room for the longest match plus
    // an 8-byte overcopy. Returns 1 at end-of-block, 0 when those margins run out (the careful path
    // takes over), -1 on an invalid code or distance (err line set).
    __attribute__((always_inline)) inline int fast_loop_body(uint8_t** outp, uint8_t* out_end, const uint8_t* win_start) {
        uint8_t* out = *outp;
        const uint8_t* in = in_;
        const uint8_t* const in_stop = in_end_ - 16;
        uint64_t bits = bits_;
        unsigned nbits = nbits_;
        const uint32_t* const lit = lit_;
        const uint32_t* const dst = dist_;
        uint8_t* const out_stop = out_end - (258 + 16);
        int ret = 0;
#define FNPZ_REFILL()                          \
    do {                                       \
        bits |= load64(in) << nbits;           \
        in += (63 - nbits) >> 3;               \
        nbits |= 56;                           \
    } while (0)
#define FNPZ_LIT(e)                                                                                  \
    do {                                                                                             \
        e = lit[bits & ((1u << kLitRoot) - 1)];                                                      \
        if (__builtin_expect((e & F_SUB) != 0, 0))                                                   \
            e = lit[e_value(e) + ((bits >> kLitRoot) & ((1u << e_extra(e)) - 1))];                   \
    } while (0)
        if (zeros_) return 0;                                  // phantom bytes buffered: careful path only
        while (in <= in_stop && out <= out_stop) {
            FNPZ_REFILL();
            uint32_t e;
            FNPZ_LIT(e);
            if (e & F_LIT) {                          // up to three literals per refill
                bits >>= e_len(e);
                nbits -= e_len(e);
                *out++ = (uint8_t)e_value(e);
                FNPZ_LIT(e);
                if (e & F_LIT) {
                    bits >>= e_len(e);
                    nbits -= e_len(e);
                    *out++ = (uint8_t)e_value(e);
                    FNPZ_LIT(e);
                    if (e & F_LIT) {
                        bits >>= e_len(e);
                        nbits -= e_len(e);
                        *out++ = (uint8_t)e_value(e);
                        continue;
                    }
                }
                if (nbits < 48) FNPZ_REFILL();                 // a length / distance pair: <= 48 bits
            }
            if (__builtin_expect((e & F_LEN) != 0, 1)) {
                bits >>= e_len(e);
                nbits -= e_len(e);
                const uint32_t xb = e_extra(e);
                const size_t len = e_value(e) + ((uint32_t)bits & ((1u << xb) - 1));
                bits >>= xb;
                nbits -= xb;
                uint32_t d = dst[bits & ((1u << kDistRoot) - 1)];
                if (__builtin_expect((d & F_SUB) != 0, 0))
                    d = dst[e_value(d) + ((bits >> kDistRoot) & ((1u << e_extra(d)) - 1))];
                if (!(d & F_DIST)) { ret = -1; err_line_ = err_line_ ? err_line_ : __LINE__; break; }
                bits >>= e_len(d);
                nbits -= e_len(d);
                const uint32_t db = e_extra(d);
                const size_t dist = e_value(d) + ((uint32_t)bits & ((1u << db) - 1));
                bits >>= db;
                nbits -= db;
                if (dist > (size_t)(out - win_start)) { ret = -1; err_line_ = err_line_ ? err_line_ : __LINE__; break; }
                const uint8_t* src = out - dist;
                uint8_t* end = out + len;
                if (dist >= 8) {
                    do {
                        std::memcpy(out, src, 8);
                        out += 8;
                        src += 8;
                    } while (out < end);
                } else if (dist == 1) {
                    std::memset(out, src[0], len);
                } else {
                    for (uint8_t* o = out; o < end; ++o) *o = o[-(ptrdiff_t)dist];
                }
                out = end;
                continue;
            }
            if (e & F_LIT) {                                   // reached only after the second refill
                bits >>= e_len(e);
                nbits -= e_len(e);
                *out++ = (uint8_t)e_value(e);
                continue;
            }
            if (e & F_EOB) {
                bits >>= e_len(e);
                nbits -= e_len(e);
                ret = 1;
                break;
            }
            ret = -1;
            err_line_ = err_line_ ? err_line_ : __LINE__;
            break;
        }
#undef FNPZ_LIT
#undef FNPZ_REFILL
        in_ = in;
        bits_ = bits;
        nbits_ = nbits;
        *outp = out;
        return ret;
    }

    int fast_loop_base(uint8_t** outp, uint8_t* out_end, const uint8_t* win_start) {
        return fast_loop_body(outp, out_end, win_start);
    }
#if defined(__x86_64__)
    // the same loop with BMI2's flag-free variable shifts (shrx): the bit buffer's shift by a code
    // length read from the table is on the critical path of every symbol
    __attribute__((target("bmi2"))) int fast_loop_bmi2(uint8_t** outp, uint8_t* out_end, const uint8_t* win_start) {
        return fast_loop_body(outp, out_end, win_start);
    }
    static bool have_bmi2() {
        static const bool ok = __builtin_cpu_supports("bmi2");
        return ok;
    }
#endif
    int fast_loop(uint8_t** outp, uint8_t* out_end, const uint8_t* win_start) {
#if defined(__x86_64__)
        if (have_bmi2()) return fast_loop_bmi2(outp, out_end, win_start);
#endif
        return fast_loop_base(outp, out_end, win_start);
    }

    // one Huffman block's symbols: kOk at its end-of-block, kFull / kCorrupt as run()
    int huffman(uint8_t** outp, uint8_t* out_end, const uint8_t* win_start) {
        uint8_t* out = *outp;
        int rc = kOk;
        for (;;) {
            const int f = fast_loop(&out, out_end, win_start);
            if (f == 1) break;
            if (f < 0) { rc = kCorrupt; break; }
            // careful path: the input's or the window's last bytes (>= 56 bits buffered: a whole
            // length / distance pair, <= 48 bits, fits)
            if (more_ && !fill_real()) { rc = kNeed; break; }     // wait for input, nothing consumed
            if (!refill_slow()) { rc = corrupt(__LINE__); break; }
            const uint32_t e = lit_entry();
            const uint32_t k = e_kind(e);
            if (k == K_INVALID) { rc = corrupt(__LINE__); break; }
            if (k == K_LIT) {
                if (out >= out_end) { rc = kFull; break; }          // not consumed: resumes here
                drop(e_len(e));
                if (overran()) { rc = corrupt(__LINE__); break; }
                *out++ = (uint8_t)e_value(e);
                continue;
            }
            if (k == K_EOB) {
                drop(e_len(e));
                if (overran()) rc = corrupt(__LINE__);
                break;
            }
            if (k != K_LEN) { rc = corrupt(__LINE__); break; }
            if (out >= out_end) { rc = kFull; break; }
            drop(e_len(e));
            const uint32_t xb = e_extra(e);
            const size_t len = e_value(e) + ((uint32_t)bits_ & ((1u << xb) - 1));
            drop(xb);
            const uint32_t d = dist_entry();
            if (e_kind(d) != K_DIST) { rc = corrupt(__LINE__); break; }
            drop(e_len(d));
            const uint32_t db = e_extra(d);
            const size_t dist = e_value(d) + ((uint32_t)bits_ & ((1u << db) - 1));
            drop(db);
            if (overran()) { rc = corrupt(__LINE__); break; }
            if (dist > (size_t)(out - win_start)) { rc = corrupt(__LINE__); break; }
            size_t n = len;
            while (n && out < out_end) {
                *out = out[-(ptrdiff_t)dist];
                ++out;
                --n;
            }
            if (n) {
                pend_len_ = n;
                pend_dist_ = dist;
                rc = kFull;
                *outp = out;
                return rc;                                            // state stays kHuff
            }
        }
        *outp = out;
        return rc;
    }
};

}  // namespace fnpz_fast
