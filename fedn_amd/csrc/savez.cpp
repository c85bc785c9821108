// savez.cpp — numpy-identical npz writer (fnpz_savez, include/fednpz.h).
//
// numpyhelper.Helper.save is np.savez_compressed (fedn/utils/helpers/plugins/numpyhelper.py:
// 144-169, the call at :162), and that archive is a deterministic byte stream: numpy's _savez
// opens every member with zipfile.ZipFile.open(key + ".npy", "w", force_zip64=True) and
// numpy.lib.format.write_array writes the .npy header in one write and then the payload in
// writes of 16 MiB // itemsize elements; zipfile feeds each write to
// zlib.compressobj(Z_DEFAULT_COMPRESSION, DEFLATED, -15) (level 6, memLevel 8, default
// strategy), CRCs it, finishes the stream, seeks back and rewrites the local header with the
// real sizes. This file replays exactly that byte sequence: the same deflate() calls into
// the same libz (the process's libz.so.1 — CPython's zlib module links it too), and
// zipfile's headers field for field (CPython 3.10 zipfile.py: ZipInfo.FileHeader,
// ZipFile._write_end_record). Members deflate in parallel; each member's stream is
// sequential, as numpy's is (fnpz_savez's single-stream parallel mode lives in
// pdeflate.h).

#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/fednpz.h"
#include "fnpz_guard.h"
#include "inflate.h"
#include "pdeflate.h"


namespace {

using fnpz_internal::set_error;

// members of at least this many bytes take pdeflate.h's single-stream parallel path
std::atomic<int64_t> g_par_min{32ll << 20}, g_par_chunk{4ll << 20};
std::atomic<int64_t> g_par_ok{0}, g_par_fallback{0};
thread_local const char* g_par_reason = nullptr;

// ---- which libz pdeflate.h may stand in for ------------------------------------------------------
// pdeflate.h reproduces zlib 1.2.11's level-6 stream. Small members always go through the process's
// libz (deflate_member); a big member's bytes come from pdeflate.h only while that libz is one
// pdeflate.h is known to match: its zlibVersion() is a modelled version, it is the libz Python's zlib
// module runs (zlib.ZLIB_RUNTIME_VERSION, handed in by codec.py: numpy's archive comes from THAT
// libz), and a self-test — one 1.5 MiB member through both, compared byte for byte — agrees. Any
// other libz (zlib-ng-compat, Chromium's, a later release) sends every member through deflate_member,
// so an archive never mixes two deflaters. Evaluated once, at the first big member.
const char* const kModelledZlib[] = {"1.2.11"};
std::mutex g_zl_mu;
std::atomic<int> g_zl_state{-1};   // -1 not evaluated, 0 off (zlib for every member), 1 pdeflate.h allowed
std::string g_zl_expect;           // Python's zlib.ZLIB_RUNTIME_VERSION ("" = not told)
int g_zl_force = 0;                // test hook: 1 = as if the check failed
std::string g_zl_reason = "not evaluated";

// the last big member's phases (s), for fnpz_savez_stats: the input copy, pdeflate.h's five phases,
// the CRC, and (per call) the archive assembly
enum { kStCopy, kStParse, kStSync, kStSched, kStPlan, kStEncode, kStCrc, kStAssemble, kStTotal, kStN };
std::mutex g_st_mu;
double g_st[kStN] = {0};
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the member's deflate() inputs as cumulative ends: the header, then numpy's writes
std::vector<int64_t> input_ends(int64_t hlen, int64_t nbytes, int64_t seg) {
    std::vector<int64_t> ends{hlen};
    if (seg <= 0) seg = std::max<int64_t>(nbytes, 1);
    for (int64_t b = 0; b < nbytes; b += seg) ends.push_back(hlen + std::min(nbytes, b + seg));
    return ends;
}

void put16(uint8_t*& p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p += 2; }
void put32(uint8_t*& p, uint32_t v) { for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i)); p += 4; }
void put64(uint8_t*& p, uint64_t v) { for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i)); p += 8; }

constexpr uint64_t kZip64Limit = (1ull << 31) - 1;   // zipfile.ZIP64_LIMIT
constexpr uint64_t kFileCountLimit = (1u << 16) - 1; // zipfile.ZIP_FILECOUNT_LIMIT
// the limits fnpz_savez applies (fnpz_savez_zip_limits: tests compare the ZIP64 branches with numpy
// run under a zipfile whose limits are patched to the same small values)
std::atomic<uint64_t> g_zip64_limit{kZip64Limit}, g_filecount_limit{kFileCountLimit};
constexpr uint16_t kDosDate = (0 << 9) | (1 << 5) | 1; // ZipInfo's default date_time 1980-01-01 00:00:00
constexpr uint16_t kDefaultVersion = 20, kZip64Version = 45;
constexpr uint32_t kExternalAttr = 0600u << 16;      // zipfile: "?rw-------"

struct Member {
    const char* name;
    const uint8_t* header;
    int64_t hlen;
    const uint8_t* data;
    int64_t nbytes;
    int64_t seg;                // numpy's write size (bytes); <= 0: one write
    pdef::Bytes out;            // the raw deflate stream (empty when it was encoded in place)
    uint32_t crc = 0;
    int rc = Z_OK;
    int64_t comp = -1;          // the stream's length once encoded in place (>= 0), else out.size()
    int64_t stream_len() const { return comp >= 0 ? comp : (int64_t)out.size(); }
};

// the same stream from pdeflate.h on `threads` threads; false: the caller runs zlib (also when the
// extra memory this path holds — a copy of the member and its symbol streams — cannot be had: the
// streaming zlib path needs only its output)
bool deflate_member_parallel_unchecked(Member& m, int threads, uint8_t* dst, int64_t dst_cap) try {
    const double t_start = now_s();
    const int64_t L = m.hlen + m.nbytes;
    std::unique_ptr<uint8_t[]> buf(new uint8_t[(size_t)L]);   // no zero fill: every byte is copied in
    uint8_t* const S = buf.get();
    std::memcpy(S, m.header, (size_t)m.hlen);
    const int64_t piece = 8 << 20;
    pdef::parallel((int)((m.nbytes + piece - 1) / piece), threads, [&](int i) {
        const int64_t b = (int64_t)i * piece;
        std::memcpy(S + m.hlen + b, m.data + b, (size_t)std::min(piece, m.nbytes - b));
    });
    const double t_copied = now_s();
    pdef::Stats st;
    const bool ok = pdef::deflate_exact(S, L, input_ends(m.hlen, m.nbytes, m.seg), threads, g_par_chunk.load(),
                                        m.out, &st, dst, dst_cap);
    (ok ? g_par_ok : g_par_fallback).fetch_add(1);
    g_par_reason = st.fallback;
    if (!ok) return false;
    if (dst) m.comp = st.out_len;
    const double t_deflated = now_s();
    // CRC-32 by pieces, combined
    const int np = (int)((L + piece - 1) / piece);
    std::vector<uint32_t> crcs((size_t)np);
    pdef::parallel(np, threads, [&](int i) {
        const int64_t b = (int64_t)i * piece;
        crcs[i] = fnpz_fast::crc32(0, S + b, (size_t)std::min(piece, L - b));
    });
    uLong crc = crcs[0];
    for (int i = 1; i < np; ++i) crc = crc32_combine(crc, crcs[i], (z_off_t)std::min(piece, L - (int64_t)i * piece));
    m.crc = (uint32_t)crc;
    m.rc = Z_OK;
    pdef::free_later(std::move(buf));   // the member's copy is returned to the OS off the critical path
    const double t_end = now_s();
    std::lock_guard<std::mutex> lk(g_st_mu);
    g_st[kStCopy] = t_copied - t_start;
    g_st[kStParse] = st.t_parse;
    g_st[kStSync] = st.t_sync;
    g_st[kStSched] = st.t_sched;
    g_st[kStPlan] = st.t_plan;
    g_st[kStEncode] = st.t_encode;
    g_st[kStCrc] = t_end - t_deflated;
    return true;
} catch (const std::bad_alloc&) {
    pdef::Bytes().swap(m.out);
    g_par_fallback.fetch_add(1);
    g_par_reason = "out of memory";
    return false;
} catch (const std::system_error&) {   // a worker thread could not be started
    pdef::Bytes().swap(m.out);
    g_par_fallback.fetch_add(1);
    g_par_reason = "no thread";
    return false;
}

// zlib.compressobj(-1, DEFLATED, -15).compress(w) for each write w, then .flush()
void deflate_member(Member& m) {
    z_stream zs{};
    if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, -MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
        m.rc = Z_MEM_ERROR;
        return;
    }
    const uint64_t raw = (uint64_t)(m.hlen + m.nbytes);
    m.out.resize((size_t)(raw + raw / 1000 + (raw >> 14) * 5 + 1024));   // >= deflateBound's stored worst case
    size_t used = 0;
    auto run = [&](const uint8_t* in, uint64_t n, int flush) -> bool {
        // CPython passes at most UINT_MAX input bytes per deflate() call (arrange_input_buffer)
        do {
            const uInt take = (uInt)std::min<uint64_t>(n, 0xFFFFFFFFu);
            zs.next_in = const_cast<Bytef*>(in);
            zs.avail_in = take;
            const bool last_piece = take == n;
            for (;;) {
                if (m.out.size() - used < 64) m.out.resize(m.out.size() * 2);
                zs.next_out = m.out.data() + used;
                const size_t room = std::min<size_t>(m.out.size() - used, 0xFFFFFFFFu);
                zs.avail_out = (uInt)room;
                const int rc = deflate(&zs, last_piece ? flush : Z_NO_FLUSH);
                used += room - zs.avail_out;
                if (rc == Z_STREAM_END) return true;
                if (rc != Z_OK && rc != Z_BUF_ERROR) return false;
                if (zs.avail_in == 0 && zs.avail_out != 0 && !(last_piece && flush == Z_FINISH)) break;
            }
            in += take;
            n -= take;
        } while (n > 0);
        return true;
    };
    bool ok = run(m.header, (uint64_t)m.hlen, Z_NO_FLUSH);
    m.crc = fnpz_fast::crc32(0, m.header, (size_t)m.hlen);
    const int64_t seg = m.seg > 0 ? m.seg : std::max<int64_t>(m.nbytes, 1);
    for (int64_t b = 0; ok && b < m.nbytes; b += seg) {
        const int64_t n = std::min(seg, m.nbytes - b);
        ok = run(m.data + b, (uint64_t)n, Z_NO_FLUSH);
        m.crc = fnpz_fast::crc32(m.crc, m.data + b, (size_t)n);
    }
    ok = ok && run(nullptr, 0, Z_FINISH);
    deflateEnd(&zs);
    m.out.resize(used);
    m.rc = ok ? Z_OK : Z_STREAM_ERROR;
}

// Why this process's libz may not be replaced by pdeflate.h ("" = it may). The self-test member is a
// .npy-like header and 1.5 MiB written in 256 KiB pieces: float32-like noise, a zero run (258-byte
// matches), a short period (lazy matches, chains at their limit) and repeated text, so the chunked
// parse, the syncs, the tail replay and all three block types are exercised against this libz.
std::string zlib_check_locked() {
    const char* v = zlibVersion();
    bool known = false;
    for (const char* k : kModelledZlib) known = known || std::strcmp(v, k) == 0;
    if (!known) return std::string("libz ") + v + " is not a version pdeflate.h models (1.2.11)";
    if (!g_zl_expect.empty() && g_zl_expect != v)
        return "Python's zlib runs libz " + g_zl_expect + ", this library links " + v;
    const int64_t n = 3 << 19;
    const char* dict = "{'descr': '<f4', 'fortran_order': False, 'shape': (393216,), }";
    std::vector<uint8_t> hdr(128, ' ');
    std::memcpy(hdr.data(), dict, std::strlen(dict));
    hdr.back() = '\n';
    std::vector<uint8_t> data((size_t)n);
    uint32_t x = 2463534242u;
    const char* text = "federated averaging of client updates, round after round; ";
    for (int64_t i = 0; i < n; i += 4) {
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        const int64_t part = i / (n / 8);
        uint32_t w;
        if (part == 2) w = 0;                                              // zero run
        else if (part == 5) w = 0x3c000000u | (uint32_t)((i / 4) % 7) << 8; // short period
        else if (part == 6) std::memcpy(&w, text + (i % 56), 4);           // text
        else w = 0x3c000000u | (x & 0x01ffffffu);                          // small float32 weights
        std::memcpy(&data[(size_t)i], &w, 4);
    }
    Member z{"t", hdr.data(), (int64_t)hdr.size(), data.data(), n, 256 << 10};
    deflate_member(z);
    if (z.rc != Z_OK) return "self-test: this libz failed to deflate";
    const int64_t L = z.hlen + n;
    std::vector<uint8_t> S((size_t)L);
    std::memcpy(S.data(), hdr.data(), hdr.size());
    std::memcpy(S.data() + hdr.size(), data.data(), (size_t)n);
    pdef::Bytes out;
    pdef::Stats st;
    if (!pdef::deflate_exact(S.data(), L, input_ends(z.hlen, n, z.seg), 4, pdef::kMinChunk, out, &st))
        return std::string("self-test: pdeflate.h fell back (") + (st.fallback ? st.fallback : "?") + ")";
    if (out != z.out) return std::string("self-test: pdeflate.h's stream differs from libz ") + v + "'s";
    return "";
}

// whether big members may take pdeflate.h (evaluated once; re-evaluated after fnpz_savez_zlib_expect)
bool zlib_modelled() {
    const int s = g_zl_state.load(std::memory_order_acquire);
    if (s >= 0) return s == 1;
    std::lock_guard<std::mutex> lk(g_zl_mu);
    if (g_zl_state.load() < 0) {
        std::string why;
        try {
            why = g_zl_force ? std::string("forced off (fnpz_savez_zlib_expect test hook)") : zlib_check_locked();
        } catch (const std::exception&) {   // no memory for the self-test: zlib this time, ask again later
            return false;
        }
        g_zl_reason = why.empty() ? std::string("libz ") + zlibVersion() + ": pdeflate.h matches it (self-test passed)"
                                  : why;
        g_zl_state.store(why.empty() ? 1 : 0, std::memory_order_release);
    }
    return g_zl_state.load() == 1;
}

// MemAvailable from /proc/meminfo (bytes), or -1 if it cannot be read
int64_t mem_available() {
    FILE* f = std::fopen("/proc/meminfo", "r");
    if (!f) return -1;
    char line[256];
    long long kb = -1;
    while (std::fgets(line, sizeof(line), f))
        if (std::sscanf(line, "MemAvailable: %lld kB", &kb) == 1) break;
    std::fclose(f);
    return kb < 0 ? -1 : (int64_t)kb * 1024;
}

bool deflate_member_parallel(Member& m, int threads, uint8_t* dst, int64_t dst_cap) {
    if (!zlib_modelled()) {
        g_par_reason = "libz not modelled";
        return false;
    }
    // the parallel path holds a copy of the member and its symbol streams (2 bytes per input byte on
    // weights) besides the output both paths hold — ~4x the member at its peak, 5.3x with the caller's
    // archive buffer (tools/big_save_check.py): where that would not fit in the host's available
    // memory, the streaming zlib path writes the same bytes (the reference streams too)
    const int64_t avail = mem_available();
    if (avail >= 0 && 5 * (m.hlen + m.nbytes) > avail) {
        g_par_fallback.fetch_add(1);
        g_par_reason = "memory";
        return false;
    }
    return deflate_member_parallel_unchecked(m, threads, dst, dst_cap);
}

}  // namespace

extern "C" int fnpz_savez(int n, const char* const* names, const uint8_t* const* headers, const int64_t* header_lens,
                          const void* const* datas, const int64_t* nbytes, const int64_t* seg_bytes, int threads,
                          uint8_t* out, int64_t out_cap, int64_t* out_len) {
    const double t_call = now_s();
    return fnpz_internal::guard("fnpz_savez", [&]() -> int {
        if (n < 0 || !out || !out_len || (n > 0 && (!names || !headers || !header_lens || !datas || !nbytes)))
            return set_error(FNPZ_EINVAL, "fnpz_savez: bad arguments");
        std::vector<Member> ms((size_t)n);
        for (int i = 0; i < n; ++i) {
            const size_t nl = std::strlen(names[i]);
            if (nl + 4 > 0xFFFF || header_lens[i] < 0 || nbytes[i] < 0 || (nbytes[i] > 0 && !datas[i]))
                return set_error(FNPZ_EINVAL, "fnpz_savez: bad member %d", i);
            ms[i] = Member{names[i], headers[i], header_lens[i], static_cast<const uint8_t*>(datas[i]), nbytes[i],
                           seg_bytes ? seg_bytes[i] : 0};
        }
        // big members take pdeflate.h's stream on every thread; the rest are deflated member-parallel
        // FIRST (largest first, so one long stream does not start last), so that when the archive is laid
        // out in order every big member's place is known and its stream is encoded straight into it (no
        // copy of the stream afterwards). Big: at least min_member bytes, or at least four chunks and more
        // than an even share of the archive per thread (member-parallel, that member alone would outlast
        // the rest of the archive spread over the other threads)
        int64_t total = 0;
        for (const Member& m : ms) total += m.hlen + m.nbytes;
        const int64_t floor = 4 * g_par_chunk.load();
        std::vector<int> order;
        std::vector<char> is_big((size_t)n, 0);
        for (int i = 0; i < n; ++i) {
            const int64_t sz = ms[i].hlen + ms[i].nbytes;
            if (threads > 1 && (sz >= g_par_min.load() || (sz >= floor && sz * threads > total))) is_big[i] = 1;
            else order.push_back(i);
        }
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return ms[a].nbytes > ms[b].nbytes; });
        fnpz_internal::run_parallel((int)order.size(), std::max(1, threads), [&](int k) { deflate_member(ms[order[k]]); });
        auto check = [&](int i) -> int {
            if (ms[i].rc == Z_MEM_ERROR) return set_error(FNPZ_ENOMEM, "fnpz_savez: zlib out of memory on member %d", i);
            if (ms[i].rc != Z_OK) return set_error(FNPZ_ECORRUPT, "fnpz_savez: deflate failed on member %d", i);
            return FNPZ_OK;
        };
        for (int i : order)
            if (const int rc = check(i)) return rc;

        uint8_t* p = out;
        uint8_t* const lim = out + out_cap;
        const uint64_t zip64_limit = g_zip64_limit.load(), filecount_limit = g_filecount_limit.load();
        std::vector<uint64_t> offs((size_t)n);
        std::vector<uint64_t> comps((size_t)n);
        std::vector<uint16_t> ver((size_t)n);
        std::vector<uint8_t*> dst((size_t)n);
        double t_asm = now_s(), t_big = 0;
        for (int i = 0; i < n; ++i) {
            Member& m = ms[i];
            const size_t nl = std::strlen(m.name) + 4;
            if ((int64_t)(30 + nl + 20) > lim - p) return set_error(FNPZ_ENOSPC, "fnpz_savez: output buffer too small");
            if (is_big[i]) {                    // encoded in place behind its local header, else zlib's stream
                const double t0 = now_s();
                uint8_t* at = p + 30 + nl + 20;
                if (!deflate_member_parallel(m, threads, at, lim - at)) deflate_member(m);
                if (const int rc = check(i)) return rc;
                t_big += now_s() - t0;
            }
            const uint64_t raw = (uint64_t)(m.hlen + m.nbytes), comp = (uint64_t)m.stream_len();
            if ((int64_t)(30 + nl + 20 + comp) > lim - p) return set_error(FNPZ_ENOSPC, "fnpz_savez: output buffer too small");
            // ZipInfo.FileHeader(zip64=True) as _ZipWriteFile.close rewrites it
            const bool big = raw > zip64_limit || comp > zip64_limit;
            ver[i] = big ? kZip64Version : kDefaultVersion;
            offs[i] = (uint64_t)(p - out);
            comps[i] = comp;
            put32(p, 0x04034b50);
            put16(p, ver[i]);
            put16(p, 0);                        // flag bits (seekable output: no data descriptor)
            put16(p, Z_DEFLATED);
            put16(p, 0);                        // DOS time
            put16(p, kDosDate);
            put32(p, m.crc);
            put32(p, big ? 0xFFFFFFFFu : (uint32_t)comp);
            put32(p, big ? 0xFFFFFFFFu : (uint32_t)raw);
            put16(p, (uint16_t)nl);
            put16(p, 20);
            std::memcpy(p, m.name, nl - 4);
            std::memcpy(p + nl - 4, ".npy", 4);
            p += nl;
            put16(p, 1);
            put16(p, 16);
            put64(p, raw);
            put64(p, comp);
            dst[i] = p;
            p += comp;
        }
        // the deflate streams into place, in 8 MiB pieces on every thread (one 370 MB member copied
        // by one thread, page faults on the fresh output included, was a serial ~0.1 s of the save)
        {
            const int64_t piece = 8 << 20;
            std::vector<std::pair<int, int64_t>> pieces;
            for (int i = 0; i < n; ++i)   // (a stream encoded in place has no bytes here)
                for (int64_t b = 0; b < (int64_t)ms[i].out.size(); b += piece) pieces.emplace_back(i, b);
            fnpz_internal::run_parallel((int)pieces.size(), std::max(1, threads), [&](int k) {
                const int i = pieces[k].first;
                const int64_t b = pieces[k].second;
                std::memcpy(dst[i] + b, ms[i].out.data() + b, (size_t)std::min<int64_t>(piece, ms[i].out.size() - b));
            });
            for (Member& m : ms) pdef::Bytes().swap(m.out);
        }
        const uint64_t cd_off = (uint64_t)(p - out);
        for (int i = 0; i < n; ++i) {   // ZipFile._write_end_record
            const Member& m = ms[i];
            const size_t nl = std::strlen(m.name) + 4;
            const uint64_t raw = (uint64_t)(m.hlen + m.nbytes);
            const uint64_t csize = comps[i];
            uint64_t extra[3];
            int ne = 0;
            const bool big = raw > zip64_limit || csize > zip64_limit;
            if (big) extra[ne++] = raw, extra[ne++] = csize;
            if (offs[i] > zip64_limit) extra[ne++] = offs[i];
            const uint16_t v = ne ? std::max<uint16_t>(kZip64Version, ver[i]) : ver[i];
            if ((int64_t)(46 + nl + 4 + 8 * ne) > lim - p) return set_error(FNPZ_ENOSPC, "fnpz_savez: output buffer too small");
            put32(p, 0x02014b50);
            put16(p, (uint16_t)(v | (3 << 8)));  // create_version | create_system (unix)
            put16(p, v);                          // extract_version
            put16(p, 0);
            put16(p, Z_DEFLATED);
            put16(p, 0);
            put16(p, kDosDate);
            put32(p, m.crc);
            put32(p, big ? 0xFFFFFFFFu : (uint32_t)csize);
            put32(p, big ? 0xFFFFFFFFu : (uint32_t)raw);
            put16(p, (uint16_t)nl);
            put16(p, (uint16_t)(ne ? 4 + 8 * ne : 0));
            put16(p, 0);                          // comment
            put16(p, 0);                          // disk number start
            put16(p, 0);                          // internal attributes
            put32(p, kExternalAttr);
            put32(p, offs[i] > zip64_limit ? 0xFFFFFFFFu : (uint32_t)offs[i]);
            std::memcpy(p, m.name, nl - 4);
            std::memcpy(p + nl - 4, ".npy", 4);
            p += nl;
            if (ne) {
                put16(p, 1);
                put16(p, (uint16_t)(8 * ne));
                for (int k = 0; k < ne; ++k) put64(p, extra[k]);
            }
        }
        const uint64_t pos2 = (uint64_t)(p - out);
        const uint64_t cd_size = pos2 - cd_off;
        uint64_t count = (uint64_t)n, size = cd_size, offset = cd_off;
        if (count > filecount_limit || cd_off > zip64_limit || cd_size > zip64_limit) {
            if (56 + 20 > lim - p) return set_error(FNPZ_ENOSPC, "fnpz_savez: output buffer too small");
            put32(p, 0x06064b50);
            put64(p, 44);
            put16(p, kZip64Version);
            put16(p, kZip64Version);
            put32(p, 0);
            put32(p, 0);
            put64(p, count);
            put64(p, count);
            put64(p, cd_size);
            put64(p, cd_off);
            put32(p, 0x07064b50);
            put32(p, 0);
            put64(p, pos2);
            put32(p, 1);
            count = std::min<uint64_t>(count, 0xFFFF);
            size = std::min<uint64_t>(size, 0xFFFFFFFFu);
            offset = std::min<uint64_t>(offset, 0xFFFFFFFFu);
        }
        if (22 > lim - p) return set_error(FNPZ_ENOSPC, "fnpz_savez: output buffer too small");
        put32(p, 0x06054b50);
        put16(p, 0);
        put16(p, 0);
        put16(p, (uint16_t)count);
        put16(p, (uint16_t)count);
        put32(p, (uint32_t)size);
        put32(p, (uint32_t)offset);
        put16(p, 0);
        *out_len = (int64_t)(p - out);
        {
            std::lock_guard<std::mutex> lk(g_st_mu);
            g_st[kStAssemble] = now_s() - t_asm - t_big;   // the big members' deflates are their own phases
            g_st[kStTotal] = now_s() - t_call;
        }
        return FNPZ_OK;
    });
}

extern "C" void fnpz_savez_zlib_expect(const char* runtime_version, int force_zlib) {
    std::lock_guard<std::mutex> lk(g_zl_mu);
    if (runtime_version) g_zl_expect = runtime_version;
    if (force_zlib >= 0) g_zl_force = force_zlib ? 1 : 0;
    g_zl_state.store(-1);
    g_zl_reason = "not evaluated";
}

extern "C" int fnpz_savez_zlib_status(char* reason, int64_t cap) {
    const bool on = zlib_modelled();
    if (reason && cap > 0) {
        std::lock_guard<std::mutex> lk(g_zl_mu);
        const size_t k = std::min<size_t>(g_zl_reason.size(), (size_t)cap - 1);
        std::memcpy(reason, g_zl_reason.data(), k);
        reason[k] = 0;
    }
    return on ? 1 : 0;
}

extern "C" int fnpz_savez_stats(double* out, int n) {
    if (!out || n <= 0) return kStN;
    std::lock_guard<std::mutex> lk(g_st_mu);
    const int k = std::min(n, (int)kStN);
    for (int i = 0; i < k; ++i) out[i] = g_st[i];
    return k;
}

extern "C" void fnpz_savez_config(int64_t min_member, int64_t chunk, int64_t* parallel, int64_t* fallback) {
    if (min_member > 0) g_par_min.store(min_member);
    if (chunk > 0) g_par_chunk.store(chunk);
    if (parallel) *parallel = g_par_ok.load();
    if (fallback) *fallback = g_par_fallback.load();
}

extern "C" void fnpz_savez_zip_limits(int64_t zip64_limit, int64_t filecount_limit) {
    g_zip64_limit.store(zip64_limit > 0 ? (uint64_t)zip64_limit : kZip64Limit);
    g_filecount_limit.store(filecount_limit > 0 ? (uint64_t)filecount_limit : kFileCountLimit);
}

extern "C" int fnpz_deflate_exact(const uint8_t* in, int64_t len, const int64_t* ends, int nends, int threads,
                                  int64_t chunk, uint8_t* out, int64_t out_cap, int64_t* out_len) {
    return fnpz_internal::guard("fnpz_deflate_exact", [&]() -> int {
        if (!in || len <= 0 || !ends || nends <= 0 || !out || !out_len || ends[nends - 1] != len)
            return set_error(FNPZ_EINVAL, "fnpz_deflate_exact: bad arguments");
        std::vector<int64_t> e(ends, ends + nends);
        pdef::Bytes res;
        pdef::Stats st;
        if (!pdef::deflate_exact(in, len, e, std::max(1, threads), chunk, res, &st))
            return set_error(FNPZ_EFALLBACK, "fnpz_deflate_exact: %s", st.fallback ? st.fallback : "fallback");
        if ((int64_t)res.size() > out_cap) return set_error(FNPZ_ENOSPC, "fnpz_deflate_exact: output buffer too small");
        std::memcpy(out, res.data(), res.size());
        *out_len = (int64_t)res.size();
        set_error(FNPZ_OK, "chunks %d fixups %d blocks %d tail_from %lld parse %.3f sync %.3f sched %.3f plan %.3f encode %.3f",
                  st.chunks, st.fixups, st.blocks, (long long)st.tail_from, st.t_parse, st.t_sync, st.t_sched, st.t_plan,
                  st.t_encode);
        return FNPZ_OK;
    });
}

// the parallel decoder's block-header pre-check (inflate.h Inflate::maybe_dynamic_header), for tests
extern "C" int fnpz_probe_dynamic_header(const uint8_t* in, int64_t len, int64_t bit) {
    if (!in || len < 0 || bit < 0) return 0;
    return fnpz_fast::Inflate::maybe_dynamic_header(in, (size_t)len, (uint64_t)bit) ? 1 : 0;
}
