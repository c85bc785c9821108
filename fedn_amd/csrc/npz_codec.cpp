// npz_codec.cpp — native .npz codec for FEDn's model wire format (see include/fednpz.h).
//
// Reader: ZIP / ZIP64 central directory -> per member local header -> raw-inflate the
// .npy preamble + header dict (parsed for descr / fortran_order / shape), then inflate the
// payload straight into the caller's buffer (no temp file, no intermediate bytes object,
// no copy), CRC-32 checked; members decode in parallel.
// Writer: every member's uncompressed stream (npy header + payload) is cut into blocks
// that deflate independently and in parallel (no shared window; non-final blocks end in
// Z_SYNC_FLUSH, the last in Z_FINISH), so their concatenation is one valid deflate stream;
// block CRC-32s are combined, and a block index in a private extra field lets fnpz_read
// inflate the blocks in parallel too. Container layout follows numpy's savez_compressed
// (ZIP64 extras on every member, names "<key>.npy").

#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fednpz.h"
#include "fnpz_guard.h"
#include "inflate.h"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace

namespace fnpz_internal {   // the error slot the other translation units (savez.cpp) report through
int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}
}  // namespace fnpz_internal

namespace {

uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
void wr16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
void wr32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i)); }
void wr64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i)); }

constexpr uint32_t kLocalSig = 0x04034b50, kCentralSig = 0x02014b50, kEocdSig = 0x06054b50;
constexpr uint32_t kZ64EocdSig = 0x06064b50, kZ64LocSig = 0x07064b50;
constexpr uInt kChunk = 1u << 30;   // zlib's avail_* are 32-bit

// ---------------------------------------------------------------------------------------
// inflate helper: a raw-deflate stream consumed in pieces into successive outputs
// ---------------------------------------------------------------------------------------
struct Inflater {
    z_stream zs{};
    const uint8_t* src;
    int64_t left;
    bool ok = false;
    Inflater(const uint8_t* s, int64_t n) : src(s), left(n) { ok = inflateInit2(&zs, -MAX_WBITS) == Z_OK; }
    ~Inflater() {
        if (ok) inflateEnd(&zs);
    }
    // fill exactly `n` bytes of out; returns false on a corrupt / short stream
    bool fill(uint8_t* out, int64_t n) {
        while (n > 0) {
            if (zs.avail_in == 0 && left > 0) {
                zs.next_in = const_cast<Bytef*>(src);
                zs.avail_in = (uInt)std::min<int64_t>(left, kChunk);
                src += zs.avail_in;
                left -= zs.avail_in;
            }
            zs.next_out = out;
            zs.avail_out = (uInt)std::min<int64_t>(n, kChunk);
            const uInt before = zs.avail_out;
            const int rc = inflate(&zs, Z_NO_FLUSH);
            const uInt got = before - zs.avail_out;
            out += got;
            n -= got;
            if (rc == Z_STREAM_END) return n == 0;
            if (rc != Z_OK && !(rc == Z_BUF_ERROR && got > 0)) return false;
            if (got == 0 && zs.avail_in == 0 && left == 0) return false;
        }
        return true;
    }
};

// source of a member's uncompressed bytes: stored or deflated
struct MemberReader {
    const uint8_t* data;
    int64_t comp;
    int method;
    int64_t pos = 0;
    Inflater* inf = nullptr;
    MemberReader(const uint8_t* d, int64_t c, int m) : data(d), comp(c), method(m) {
        if (method == 8) inf = new Inflater(d, c);
    }
    ~MemberReader() { delete inf; }
    bool ready() const { return method == 0 || (inf && inf->ok); }
    bool read(uint8_t* out, int64_t n) {
        if (method == 0) {
            if (pos + n > comp) return false;
            std::memcpy(out, data + pos, (size_t)n);
            pos += n;
            return true;
        }
        return inf->fill(out, n);
    }
};

// ---------------------------------------------------------------------------------------
// .npy header dict parser: {'descr': '<f4', 'fortran_order': False, 'shape': (3, 4), }
// ---------------------------------------------------------------------------------------
bool parse_npy_dict(const std::string& h, fnpz_entry* e) {
    auto key = [&](const char* k) -> size_t {
        size_t p = h.find(std::string("'") + k + "'");
        if (p == std::string::npos) return p;
        p = h.find(':', p);
        return p == std::string::npos ? p : p + 1;
    };
    size_t p = key("descr");
    if (p == std::string::npos) return false;
    while (p < h.size() && h[p] == ' ') ++p;
    if (p >= h.size() || (h[p] != '\'' && h[p] != '"')) return false;   // structured dtypes (lists) unsupported
    const char q = h[p];
    const size_t end = h.find(q, p + 1);
    if (end == std::string::npos || end - p - 1 >= sizeof(e->descr)) return false;
    std::memcpy(e->descr, h.data() + p + 1, end - p - 1);
    e->descr[end - p - 1] = 0;
    p = key("fortran_order");
    if (p == std::string::npos) return false;
    while (p < h.size() && h[p] == ' ') ++p;
    e->fortran_order = h.compare(p, 4, "True") == 0 ? 1 : 0;
    p = key("shape");
    if (p == std::string::npos) return false;
    p = h.find('(', p);
    const size_t close = h.find(')', p);
    if (p == std::string::npos || close == std::string::npos) return false;
    e->ndim = 0;
    size_t i = p + 1;
    while (i < close) {
        while (i < close && (h[i] == ' ' || h[i] == ',')) ++i;
        if (i >= close) break;
        if (h[i] < '0' || h[i] > '9') return false;
        int64_t v = 0;
        while (i < close && h[i] >= '0' && h[i] <= '9') v = v * 10 + (h[i++] - '0');
        if (e->ndim >= FNPZ_MAX_DIMS) return false;
        e->shape[e->ndim++] = v;
    }
    return true;
}

int64_t descr_itemsize(const char* d) {
    // '<f4', '|u1', '<c16', '|S5', '<U6' ...: the digits after the kind letter are bytes,
    // except for 'U' (UCS-4 characters: 4 bytes each)
    const char* p = d;
    char kind = 0;
    while (*p && (*p < '0' || *p > '9')) kind = *p++;
    const int64_t n = *p ? std::atoll(p) : 0;
    return kind == 'U' ? 4 * n : n;
}

// ---------------------------------------------------------------------------------------
// central directory
// ---------------------------------------------------------------------------------------
struct CdEntry {
    std::string name;
    int method;
    uint32_t crc;
    uint64_t comp, uncomp, local_off;
};

// Block index extra field written by fnpz_write (ID 0x5046, "FP"): u32 count, u32 pad,
// u64 raw block size, then count + 1 u64 offsets of each independently deflated block
// inside the member's compressed data. Readers that do not know the ID skip it (APPNOTE
// 4.5.2); fnpz_read uses it to inflate the blocks of one member in parallel.
constexpr uint16_t kIndexId = 0x5046;
constexpr int kMaxIndexBlocks = 8000;   // keeps the local extra field < 64 KiB

int read_central(const uint8_t* a, int64_t len, std::vector<CdEntry>& out) {
    if (len < 22) return fail(FNPZ_EFORMAT, "not a zip archive (too short)");
    int64_t eocd = -1;
    for (int64_t p = len - 22; p >= std::max<int64_t>(0, len - 22 - 65535); --p)
        if (rd32(a + p) == kEocdSig) {
            eocd = p;
            break;
        }
    if (eocd < 0) return fail(FNPZ_EFORMAT, "no end-of-central-directory record");
    uint64_t n = rd16(a + eocd + 10), cd_size = rd32(a + eocd + 12), cd_off = rd32(a + eocd + 16);
    if (eocd >= 20 && rd32(a + eocd - 20) == kZ64LocSig) {
        const uint64_t z64 = rd64(a + eocd - 20 + 8);
        if (z64 + 56 > (uint64_t)len || rd32(a + z64) != kZ64EocdSig) return fail(FNPZ_EFORMAT, "bad ZIP64 EOCD");
        n = rd64(a + z64 + 32);
        cd_size = rd64(a + z64 + 40);
        cd_off = rd64(a + z64 + 48);
    }
    if (cd_off + cd_size > (uint64_t)len) return fail(FNPZ_EFORMAT, "central directory out of range");
    const uint8_t* p = a + cd_off;
    const uint8_t* end = p + cd_size;
    for (uint64_t i = 0; i < n; ++i) {
        if (p + 46 > end || rd32(p) != kCentralSig) return fail(FNPZ_EFORMAT, "bad central directory entry %llu", (unsigned long long)i);
        CdEntry e;
        const uint16_t flags = rd16(p + 8);
        if (flags & 1) return fail(FNPZ_EFORMAT, "encrypted members are not supported");
        e.method = rd16(p + 10);
        e.crc = rd32(p + 16);
        e.comp = rd32(p + 20);
        e.uncomp = rd32(p + 24);
        const uint16_t nl = rd16(p + 28), xl = rd16(p + 30), cl = rd16(p + 32);
        e.local_off = rd32(p + 42);
        if (p + 46 + nl + xl + cl > end) return fail(FNPZ_EFORMAT, "truncated central directory");
        e.name.assign(reinterpret_cast<const char*>(p + 46), nl);
        const uint8_t* x = p + 46 + nl;
        const uint8_t* xe = x + xl;
        while (x + 4 <= xe) {
            const uint16_t id = rd16(x), sz = rd16(x + 2);
            if (id == 1) {
                const uint8_t* f = x + 4;
                if (e.uncomp == 0xFFFFFFFFu && f + 8 <= x + 4 + sz) { e.uncomp = rd64(f); f += 8; }
                if (e.comp == 0xFFFFFFFFu && f + 8 <= x + 4 + sz) { e.comp = rd64(f); f += 8; }
                if (e.local_off == 0xFFFFFFFFu && f + 8 <= x + 4 + sz) { e.local_off = rd64(f); f += 8; }
            }
            x += 4 + sz;
        }
        out.push_back(e);
        p += 46 + nl + xl + cl;
    }
    return FNPZ_OK;
}

int resolve_entry(const uint8_t* a, int64_t len, const CdEntry& c, fnpz_entry* e) {
    std::memset(e, 0, sizeof(*e));
    if (c.method != 0 && c.method != 8) return fail(FNPZ_EFORMAT, "%s: compression method %d unsupported", c.name.c_str(), c.method);
    if (c.local_off + 30 > (uint64_t)len || rd32(a + c.local_off) != kLocalSig) return fail(FNPZ_EFORMAT, "%s: bad local header", c.name.c_str());
    const uint16_t lnl = rd16(a + c.local_off + 26), lxl = rd16(a + c.local_off + 28);
    const uint64_t data = c.local_off + 30 + lnl + lxl;
    if (data + c.comp > (uint64_t)len) return fail(FNPZ_EFORMAT, "%s: member data out of range", c.name.c_str());
    std::string nm = c.name;
    if (nm.size() >= 4 && nm.compare(nm.size() - 4, 4, ".npy") == 0) nm.resize(nm.size() - 4);
    if (nm.size() >= sizeof(e->name)) return fail(FNPZ_EFORMAT, "member name too long");
    std::memcpy(e->name, nm.data(), nm.size());
    e->method = c.method;
    e->crc32 = c.crc;
    e->comp_size = (int64_t)c.comp;
    e->uncomp_size = (int64_t)c.uncomp;
    e->data_offset = (int64_t)data;
    e->index_offset = 0;
    e->index_count = 0;
    if (data <= (uint64_t)len) {
        const uint8_t* x = a + c.local_off + 30 + lnl;
        const uint8_t* xe = x + lxl;
        while (x + 4 <= xe) {
            const uint16_t id = rd16(x), sz = rd16(x + 2);
            if (id == kIndexId && sz >= 16 && x + 4 + sz <= xe) {
                const uint32_t cnt = rd32(x + 4);
                if (cnt > 0 && (uint64_t)sz == 16 + 8ull * (cnt + 1) && rd64(x + 4 + 16 + 8ull * cnt) == c.comp) {
                    e->index_offset = (int64_t)(x + 4 - a);
                    e->index_count = (int32_t)cnt;
                }
            }
            x += 4 + sz;
        }
    }
    // .npy preamble: magic(6) major minor len (2 or 4) then the header dict
    MemberReader r(a + data, e->comp_size, c.method);
    if (!r.ready()) return fail(FNPZ_ECORRUPT, "%s: inflate init failed", c.name.c_str());
    uint8_t pre[12];
    if (!r.read(pre, 10) || std::memcmp(pre, "\x93NUMPY", 6) != 0) return fail(FNPZ_EFORMAT, "%s: not a .npy member", c.name.c_str());
    int64_t hlen, hoff;
    if (pre[6] == 1) {
        hlen = rd16(pre + 8);
        hoff = 10;
    } else if (pre[6] == 2 || pre[6] == 3) {
        if (!r.read(pre + 10, 2)) return fail(FNPZ_ECORRUPT, "%s: short header", c.name.c_str());
        hlen = rd32(pre + 8);
        hoff = 12;
    } else {
        return fail(FNPZ_EFORMAT, "%s: .npy version %d unsupported", c.name.c_str(), pre[6]);
    }
    std::string h((size_t)hlen, '\0');
    if (!r.read(reinterpret_cast<uint8_t*>(&h[0]), hlen)) return fail(FNPZ_ECORRUPT, "%s: short header", c.name.c_str());
    if (!parse_npy_dict(h, e)) return fail(FNPZ_EFORMAT, "%s: unsupported .npy header %s", c.name.c_str(), h.c_str());
    e->npy_header = hoff + hlen;
    int64_t count = 1;
    for (int d = 0; d < e->ndim; ++d) count *= e->shape[d];
    e->nbytes = count * descr_itemsize(e->descr);
    if (e->npy_header + e->nbytes != e->uncomp_size)
        return fail(FNPZ_EFORMAT, "%s: size mismatch (header says %lld payload bytes, member holds %lld)", c.name.c_str(),
                    (long long)e->nbytes, (long long)(e->uncomp_size - e->npy_header));
    return FNPZ_OK;
}

// Inflate one raw-deflate range whose output is exactly ``hlen`` bytes into ``hdr`` followed by
// ``dlen`` bytes into ``dst`` (fnpz_fast::Inflate, inflate.h), CRC-32 folded in over 256 KiB
// pieces while they are in cache. The header and the first 64 KiB of payload are decoded into a
// scratch buffer first, so that every later back-reference (<= 32 KiB) stays inside ``dst``.
// Returns 0, or -1 with ``*line`` = the decoder's verdict line (0: the stream ended early).
int inflate_split(const uint8_t* in, int64_t inlen, uint8_t* hdr, int64_t hlen, uint8_t* dst, int64_t dlen,
                  uint32_t* crc, int* line) {
    std::unique_ptr<fnpz_fast::Inflate> dec(new fnpz_fast::Inflate(in, (size_t)inlen));
    uint32_t c = *crc;
    *line = 0;
    auto fill = [&](uint8_t* lo, uint8_t* hi, const uint8_t* win) -> bool {
        uint8_t* o = lo;
        const int rc = dec->run(&o, hi, win);
        if (rc == fnpz_fast::Inflate::kCorrupt) *line = dec->error_line();
        return rc != fnpz_fast::Inflate::kCorrupt && o == hi;
    };
    int64_t done = 0;
    if (hlen > 0) {
        const int64_t first = std::min<int64_t>(dlen, 64 << 10);
        std::vector<uint8_t> tmp((size_t)(hlen + first));
        if (!fill(tmp.data(), tmp.data() + tmp.size(), tmp.data())) return -1;
        c = fnpz_fast::crc32(c, tmp.data(), tmp.size());
        std::memcpy(hdr, tmp.data(), (size_t)hlen);
        if (first > 0) std::memcpy(dst, tmp.data() + hlen, (size_t)first);
        done = first;
    }
    constexpr int64_t kPiece = 256 << 10;
    while (done < dlen) {
        const int64_t k = std::min<int64_t>(kPiece, dlen - done);
        if (!fill(dst + done, dst + done + k, dst)) return -1;
        c = fnpz_fast::crc32(c, dst + done, (size_t)k);
        done += k;
    }
    *crc = c;
    return 0;
}

// ---------------------------------------------------------------------------------------
// One deflate stream decoded on several threads (FEDn's np.savez_compressed writes one stream
// per tensor; a model dominated by one large tensor would decode on one core). The compressed
// bytes are cut into ``threads`` ranges; in each range after the first, the first position where
// a dynamic-Huffman block header parses and trial-decodes is taken as a chunk start. Chunk t
// decodes from its start to the next chunk's start — it must arrive EXACTLY at that bit on a block
// header, which proves by induction from the stream's own start that every chunk start is a real
// block boundary. A chunk begins in marker mode (its 32 KiB of history unknown: copies from it
// carry markers, Inflate::run_markers) until its last 32 KiB hold no marker, then runs the byte
// decoder; once the chunks before it are known its markers are replaced by the bytes they stand
// for. The member's CRC-32 over the assembled output is the final check. Any failure (no block
// found, a chunk that does not meet the next start, a marker before the stream's start, a CRC
// mismatch) returns -1 and the caller decodes the stream sequentially: the result never depends
// on the speculation.
// ---------------------------------------------------------------------------------------
struct GrowBuf {                                  // uninitialised, growable byte buffer
    std::unique_ptr<uint8_t[]> p;
    size_t cap = 0;
    void reserve_keep(size_t need, size_t keep) {
        if (need <= cap) return;
        size_t c = std::max(need, cap + cap / 2);
        std::unique_ptr<uint8_t[]> q(new uint8_t[c]);
        if (keep) std::memcpy(q.get(), p.get(), keep);
        p.swap(q);
        cap = c;
    }
};

struct ParChunk {
    uint64_t start = 0;                          // input bit of the block header it starts at
    std::vector<uint16_t> mark;                  // marker-mode output; [0, 32768) the unknown window
    GrowBuf body;                                // byte-mode output; [0, hist) the window it started with
    size_t hist = 0, body_len = 0;
    std::vector<uint8_t> prefix;                 // mark's output resolved to bytes
    int rc = 0;
    size_t len() const { return prefix.size() + (body_len - hist); }
    size_t cap_left() const { return body.cap - body_len; }
};

// byte-mode decode into c.body from c.body_len until a stop / the end
int par_bytes(fnpz_fast::Inflate& d, ParChunk& c, size_t expect) {
    for (;;) {
        if (c.cap_left() < (1u << 20)) c.body.reserve_keep(c.body_len + std::max<size_t>(expect / 4, 4u << 20), c.body_len);
        uint8_t* o = c.body.p.get() + c.body_len;
        const int rc = d.run(&o, c.body.p.get() + c.body.cap, c.body.p.get());
        c.body_len = (size_t)(o - c.body.p.get());
        if (rc == fnpz_fast::Inflate::kFull) continue;
        return rc;
    }
}

// the ``want`` (<= 32768) bytes of logical output right before chunk t, into the end of win[32768]
void chunk_tail(const std::vector<ParChunk>& ch, int t, size_t want, uint8_t* win) {
    size_t got = 0;
    for (int u = t - 1; u >= 0 && got < want; --u) {
        const ParChunk& c = ch[u];
        // chunk u's output: prefix, then body[hist, body_len)
        const size_t blen = c.body_len - c.hist;
        size_t k = std::min(want - got, blen);
        if (k) std::memcpy(win + 32768 - got - k, c.body.p.get() + c.body_len - k, k);
        got += k;
        if (got < want) {
            k = std::min(want - got, c.prefix.size());
            if (k) std::memcpy(win + 32768 - got - k, c.prefix.data() + c.prefix.size() - k, k);
            got += k;
        }
    }
}

template <class F>
void parallel_for(int n, int threads, F&& f);

// The parallel decode's phases run on one process-wide pool: a burst of updates read at once (the
// staging workers decode every ModelUpdate as it arrives) queues its chunks on the same workers,
// so no core idles while any decode has chunks left and no decode is left on one thread because an
// earlier one holds the rest. Jobs are served in arrival order; a caller works on its own job's
// indices too, so a job always completes (also nested in fnpz_read's member tasks, and in a forked
// child, which gets a fresh pool like CopyPool).
class DecodePool {
   public:
    static DecodePool& get() {
        static std::mutex m;
        static DecodePool* pool = nullptr;
        static pid_t owner = 0;
        std::lock_guard<std::mutex> lk(m);
        if (!pool || owner != getpid()) {
            pool = new DecodePool();               // never destroyed: parked workers end with the process
            owner = getpid();
        }
        return *pool;
    }
    template <class F>
    void run(int n, int want, F&& f) {
        if (n <= 0) return;
        if (want <= 1 || n == 1) {
            for (int i = 0; i < n; ++i) f(i);
            return;
        }
        auto job = std::make_shared<Job>();
        job->n = n;
        job->f = [&f](int i) { f(i); };
        {
            std::lock_guard<std::mutex> lk(mu_);
            const int w = std::min(want, kMaxThreads) - 1;
            try {
                for (; workers_ < w; ++workers_) std::thread([this] { work(); }).detach();
            } catch (...) {
                // no more threads: the pool's and the caller's finish the job
            }
            queue_.push_back(job);
        }
        cv_.notify_all();
        for (int i; (i = claim(job.get())) >= 0;) finish(*job, i);
        std::unique_lock<std::mutex> lk(job->mu);
        job->cv.wait(lk, [&] { return job->done == job->n; });
        job->err.rethrow();   // a worker's exception, on the calling thread
    }

   private:
    static constexpr int kMaxThreads = 64;
    struct Job {
        int n = 0, next = 0, done = 0;   // next: under the pool's lock; done: under mu
        std::function<void(int)> f;      // the caller's body, alive until done == n
        fnpz_internal::FirstError err;   // the first exception of any index (the rest still run)
        std::mutex mu;
        std::condition_variable cv;
    };
    int claim(Job* j) {                    // the next index of j, or -1; a fully claimed job leaves the queue
        std::lock_guard<std::mutex> lk(mu_);
        if (j->next >= j->n) return -1;
        const int i = j->next++;
        if (j->next == j->n)
            for (auto it = queue_.begin(); it != queue_.end(); ++it)
                if (it->get() == j) {
                    queue_.erase(it);
                    break;
                }
        return i;
    }
    static void finish(Job& j, int i) {
        try {
            j.f(i);
        } catch (...) {
            j.err.capture();
        }
        std::lock_guard<std::mutex> lk(j.mu);
        if (++j.done == j.n) j.cv.notify_all();
    }
    void work() {
        for (;;) {
            std::shared_ptr<Job> j;
            int i;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return !queue_.empty(); });
                j = queue_.front();            // holds the job past its caller's wait
                i = j->next++;
                if (j->next == j->n) queue_.pop_front();
            }
            finish(*j, i);
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Job>> queue_;
    int workers_ = 0;
};

template <class F>
void decode_for(int n, int threads, F&& f) {
    DecodePool::get().run(n, threads, std::forward<F>(f));
}

// fnpz_parallel_config: streams of at least g_par_min compressed bytes, chunks of at least
// g_par_chunk; counters of the decodes that went parallel / fell back
std::atomic<int64_t> g_par_min{16 << 20}, g_par_chunk{4 << 20}, g_par_ok{0}, g_par_fallback{0};
std::atomic<int> g_par_inflight{0};             // large deflated members being decoded

int inflate_parallel(const uint8_t* in, int64_t inlen, uint8_t* hdr, int64_t hlen, uint8_t* dst, int64_t dlen,
                     int threads, uint32_t* crc_out) {
    using fnpz_fast::Inflate;
    const int64_t min_chunk = std::max<int64_t>(g_par_chunk.load(), 64 << 10);
    const int T = (int)std::min<int64_t>(threads, inlen / min_chunk);
    if (T < 2) return -1;
    // a stream that starts with a stored or fixed-code block (deflate's choice for incompressible
    // bytes, or Z_FIXED) is not split: chunk starts are searched as dynamic-block headers only
    if (((in[0] >> 1) & 3) != 2) return -1;
    const uint64_t total = (uint64_t)(hlen + dlen);
    // 1. chunk starts: the first block header in each range that parses and trial-decodes
    std::vector<uint64_t> starts((size_t)T, 0);
    std::vector<char> found((size_t)T, 0);
    decode_for(T - 1, T - 1, [&](int j) {
        const int t = j + 1;
        const uint64_t lo = (uint64_t)inlen * (uint64_t)t / (uint64_t)T * 8;
        // zlib ends a block every 16 K symbols (<= ~30 KB of dynamic codes): 128 KiB of search finds
        // one, and bounds the time lost on stretches without dynamic blocks (stored ones)
        const uint64_t hi = std::min<uint64_t>((uint64_t)inlen * (uint64_t)(t + 1) / (uint64_t)T * 8, lo + (1ull << 20));
        std::unique_ptr<Inflate> d(new Inflate(in, (size_t)inlen));
        std::vector<uint16_t> scratch;
        for (uint64_t b = lo; b < hi; ++b) {
            if (!Inflate::maybe_dynamic_header(in, (size_t)inlen, b)) continue;
            d->restart_at(b);
            scratch.resize(32768);
            for (int i = 0; i < 32768; ++i) scratch[(size_t)i] = (uint16_t)(256 + i);
            const int rc = d->run_markers(scratch, 32768 + 16384);
            if (rc == Inflate::kFull || (rc == Inflate::kEnd && scratch.size() > 32768)) {
                starts[(size_t)t] = b;
                found[(size_t)t] = 1;
                return;
            }
        }
    });
    std::vector<uint64_t> st(1, 0);
    for (int t = 1; t < T; ++t)
        if (found[(size_t)t] && starts[(size_t)t] > st.back()) st.push_back(starts[(size_t)t]);
    const int C = (int)st.size();
    if (C < 2) return -1;
    // 2. every chunk from its start to the next one's
    std::vector<ParChunk> ch((size_t)C);
    const size_t expect = (size_t)(total / (uint64_t)C) + (1u << 20);
    decode_for(C, C, [&](int t) {
        ParChunk& c = ch[(size_t)t];
        std::unique_ptr<Inflate> d(new Inflate(in, (size_t)inlen));
        d->restart_at(st[(size_t)t]);
        d->stop_at(t + 1 < C ? st[(size_t)t + 1] : Inflate::kNoStop);
        if (t == 0) {
            c.rc = par_bytes(*d, c, expect);
            return;
        }
        c.mark.resize(32768);
        for (int i = 0; i < 32768; ++i) c.mark[(size_t)i] = (uint16_t)(256 + i);
        int rc = d->run_markers(c.mark, std::min<size_t>((size_t)total, 64u << 20) + 32768);
        if (rc == Inflate::kSwitch) {                             // the last 32 KiB hold bytes only
            c.body.reserve_keep(expect + 32768, 0);
            const size_t m = c.mark.size();
            for (size_t i = 0; i < 32768; ++i) c.body.p[i] = (uint8_t)c.mark[m - 32768 + i];
            c.hist = c.body_len = 32768;
            rc = par_bytes(*d, c, expect);
        }
        c.rc = rc;
    });
    uint64_t sum = 0;
    for (int t = 0; t < C; ++t) {
        const ParChunk& c = ch[(size_t)t];
        if (c.rc != (t + 1 < C ? Inflate::kStop : Inflate::kEnd)) return -1;
        sum += (c.mark.empty() ? 0 : c.mark.size() - 32768) + (c.body_len - c.hist);
    }
    if (sum != total) return -1;
    // 3. markers -> bytes, chunk by chunk (each needs the 32 KiB before it)
    std::vector<uint64_t> off((size_t)C + 1, 0);
    std::vector<uint8_t> win(32768);
    for (int t = 0; t < C; ++t) {
        ParChunk& c = ch[(size_t)t];
        if (t > 0) {
            const size_t avail = (size_t)std::min<uint64_t>(32768, off[(size_t)t]);
            chunk_tail(ch, t, avail, win.data());
            // output = mark[32768, m) resolved, then body[hist, body_len) (body[0, hist) repeats the
            // mark's last 32 KiB as the byte decoder's window)
            const size_t m = c.mark.size();
            c.prefix.resize(m - 32768);
            for (size_t i = 32768; i < m; ++i) {
                const uint16_t v = c.mark[i];
                if (v < 256) {
                    c.prefix[i - 32768] = (uint8_t)v;
                } else {
                    const size_t w = (size_t)(v - 256);
                    if (w < 32768 - avail) return -1;            // a reference before the stream's start
                    c.prefix[i - 32768] = win[w];
                }
            }
            std::vector<uint16_t>().swap(c.mark);
        }
        off[(size_t)t + 1] = off[(size_t)t] + c.len();
    }
    // 4. into [hdr | dst], CRC-32 per chunk, combined in order
    std::vector<uint32_t> crcs((size_t)C, 0);
    decode_for(C, C, [&](int t) {
        const ParChunk& c = ch[(size_t)t];
        uint64_t o = off[(size_t)t];
        uint32_t cr = 0;
        auto put = [&](const uint8_t* src, size_t n) {
            cr = fnpz_fast::crc32(cr, src, n);
            while (n) {
                if (o < (uint64_t)hlen) {
                    const size_t k = (size_t)std::min<uint64_t>(n, (uint64_t)hlen - o);
                    std::memcpy(hdr + o, src, k);
                    o += k, src += k, n -= k;
                } else {
                    std::memcpy(dst + (o - (uint64_t)hlen), src, n);
                    o += n;
                    n = 0;
                }
            }
        };
        if (!c.prefix.empty()) put(c.prefix.data(), c.prefix.size());
        if (c.body_len > c.hist) put(c.body.p.get() + c.hist, c.body_len - c.hist);
        crcs[(size_t)t] = cr;
    });
    uLong crc = crcs[0];
    for (int t = 1; t < C; ++t) crc = crc32_combine(crc, crcs[(size_t)t], (z_off_t)ch[(size_t)t].len());
    *crc_out = (uint32_t)crc;
    return 0;
}

int decode_one(const uint8_t* a, const fnpz_entry& e, void* dst, char* err, size_t errlen, int threads) {
    uint8_t* out = static_cast<uint8_t*>(dst);
    std::vector<uint8_t> hdr((size_t)e.npy_header);
    uint32_t crc = 0;
    // concurrent reads (the staging workers decode several updates at once) share DecodePool's
    // threads: each parallel decode queues its chunks there. Once ``threads`` large members are
    // being decoded at once every core has one, and a member decodes in order (the split's search,
    // markers and copy cost ~15 % more core time than the in-order decode)
    struct Inflight {
        const int ahead = g_par_inflight++;
        ~Inflight() { --g_par_inflight; }
    };
    const bool large = e.method == 8 && e.comp_size >= g_par_min.load() &&
                       e.comp_size >= 2 * std::max<int64_t>(g_par_chunk.load(), 64 << 10);
    std::unique_ptr<Inflight> inflight(large ? new Inflight() : nullptr);
    if (large && threads > 1 && inflight->ahead < threads) {
        uint32_t pc = 0;
        const bool ok = inflate_parallel(a + e.data_offset, e.comp_size, hdr.data(), e.npy_header, out, e.nbytes,
                                         threads, &pc) == 0 && pc == e.crc32;
        if (ok) {
            g_par_ok++;
            return FNPZ_OK;
        }
        g_par_fallback++;                // the speculation did not hold (or the stream is bad): in order
    }
    if (e.method == 8) {
        int line = 0;
        if (inflate_split(a + e.data_offset, e.comp_size, hdr.data(), e.npy_header, out, e.nbytes, &crc, &line))
            return snprintf(err, errlen, "%.200s: corrupt or truncated deflate stream (inflate.h:%d)", e.name, line),
                   FNPZ_ECORRUPT;
    } else {
        if (e.npy_header + e.nbytes > e.comp_size) return snprintf(err, errlen, "%s: truncated member", e.name), FNPZ_ECORRUPT;
        if (e.npy_header > 0) std::memcpy(hdr.data(), a + e.data_offset, (size_t)e.npy_header);
        if (e.nbytes > 0) std::memcpy(out, a + e.data_offset + e.npy_header, (size_t)e.nbytes);
        crc = fnpz_fast::crc32(fnpz_fast::crc32(0, hdr.data(), hdr.size()), out, (size_t)e.nbytes);
    }
    if (crc != e.crc32) return snprintf(err, errlen, "%s: CRC-32 mismatch", e.name), FNPZ_ECORRUPT;
    return FNPZ_OK;
}

template <class F>
void parallel_for(int n, int threads, F&& f) {
    fnpz_internal::run_parallel(n, threads, std::forward<F>(f));
}

// ---------------------------------------------------------------------------------------
// writer
// ---------------------------------------------------------------------------------------
struct Block {
    int member;
    int64_t begin, len;          // range in the member's virtual stream (header + payload)
    bool last;
    std::vector<uint8_t> out;
    uLong crc = 0;
    int rc = Z_OK;
};

struct MemberSrc {
    const uint8_t* header;
    int64_t hlen;
    const uint8_t* data;
    int64_t nbytes;
    // copy virtual-stream range [b, b+n) into dst
    void gather(int64_t b, int64_t n, uint8_t* dst) const {
        if (b < hlen) {
            const int64_t k = std::min(n, hlen - b);
            std::memcpy(dst, header + b, (size_t)k);
            dst += k;
            b += k;
            n -= k;
        }
        if (n > 0) std::memcpy(dst, data + (b - hlen), (size_t)n);
    }
    const uint8_t* direct(int64_t b, int64_t n) const { return b >= hlen ? data + (b - hlen) : (b + n <= hlen ? header + b : nullptr); }
};

// one deflate pass of [in, in + n) as a (sync-flushed or final) raw stream; false on a zlib error
bool deflate_into(const uint8_t* in, int64_t n, bool last, int level, int strategy, std::vector<uint8_t>& out) {
    z_stream zs{};
    if (deflateInit2(&zs, level, Z_DEFLATED, -MAX_WBITS, 8, strategy) != Z_OK) return false;
    // zlib 1.2.11's deflateBound assumes a stored fallback, which Z_FIXED does not take (fixed codes can
    // expand incompressible bytes by 1/8): size for that too
    out.resize(std::max<size_t>(deflateBound(&zs, (uLong)n), (size_t)(n + n / 8 + n / 64)) + 64);
    zs.next_in = const_cast<Bytef*>(in);
    zs.avail_in = (uInt)n;
    zs.next_out = out.data();
    zs.avail_out = (uInt)out.size();
    const int rc = deflate(&zs, last ? Z_FINISH : Z_SYNC_FLUSH);
    const bool ok = last ? rc == Z_STREAM_END : (rc == Z_OK && zs.avail_in == 0);
    out.resize(out.size() - zs.avail_out);
    deflateEnd(&zs);
    return ok;
}

// FNPZ_STRATEGY_AUTO: run-length matching only (zlib's Z_RLE) — on model weights (fp32 / bf16 values,
// sparse or not) as small as the default strategy or smaller and 3-8x faster, as their bytes hardly
// repeat beyond runs; a block that shrinks below 60 % (structured data: integer ramps, tiled
// patterns, where longer matches pay) is deflated again with the default strategy at level 1 and the
// smaller of the two kept
void deflate_block(const MemberSrc& m, Block& blk, int level, int strategy) {
    std::vector<uint8_t> tmp;
    const uint8_t* in = m.direct(blk.begin, blk.len);
    if (!in) {
        tmp.resize((size_t)blk.len);
        m.gather(blk.begin, blk.len, tmp.data());
        in = tmp.data();
    }
    blk.crc = fnpz_fast::crc32(0, in, (size_t)blk.len);
    const bool autos = strategy == FNPZ_STRATEGY_AUTO;
    if (!deflate_into(in, blk.len, blk.last, level, autos && level > 0 ? Z_RLE : (autos ? Z_DEFAULT_STRATEGY : strategy),
                      blk.out)) {
        blk.rc = Z_BUF_ERROR;
        return;
    }
    blk.rc = Z_OK;
    if (autos && level > 0 && (double)blk.out.size() < 0.6 * (double)blk.len) {
        std::vector<uint8_t> alt;
        if (deflate_into(in, blk.len, blk.last, 1, Z_DEFAULT_STRATEGY, alt) && alt.size() < blk.out.size())
            blk.out.swap(alt);
    }
}

// ---------------------------------------------------------------------------------------
// streaming reader: the archive arrives front to back in pieces (an upload's chunks), so
// members are read from their LOCAL headers as they come; the central directory at the end
// is only recognised, never needed. Payload bytes are inflated straight into the caller's
// window (e.g. a pinned slot); the CRC-32 covers the .npy header and payload as in the zip.
// ---------------------------------------------------------------------------------------
constexpr uint32_t kDescSig = 0x08074b50;
constexpr size_t kMaxNpyHeader = 1u << 20;

}  // namespace

struct fnpz_stream {
    std::vector<uint8_t> in;            // buffered input; in[pos:] not consumed yet
    size_t pos = 0;
    enum State { HDR, NPY, DATA, DESC, END } st = HDR;
    std::string name;
    uint16_t flags = 0;
    int method = 0;
    uint32_t crc_want = 0;
    uint64_t raw_left = 0;              // stored member: bytes still to read
    bool zip64 = false;
    z_stream zs{};
    bool zinit = false;
    bool zend = false;                  // the member's data ended
    uLong crc = 0;
    std::vector<uint8_t> pend;          // inflated bytes not delivered yet (header + first payload)
    size_t pend_pos = 0;
    int64_t left = 0;                   // payload bytes still to deliver
    int err = 0;
    // deflated members whose compressed size the local header gives (no data descriptor): the
    // codec's own decoder (inflate.h), fed as the archive arrives, decoding into ``hist`` — the last
    // 32 KiB of output stay there as the back-reference window, the callers' windows are separate
    std::unique_ptr<fnpz_fast::Inflate> fdec;
    bool fast = false;
    bool fend = false;                  // the decoder passed the member's final block
    uint64_t comp_left = 0;             // compressed bytes of the member not handed to the decoder
    std::vector<uint8_t> hist;
    size_t hp = 0, hd = 0;              // hist[0, hp) decoded; [hd, hp) not delivered yet
    static constexpr size_t kHistCap = (1u << 20) + (32u << 10), kWindow = 32u << 10;

    ~fnpz_stream() {
        if (zinit) inflateEnd(&zs);
    }
    size_t avail() const { return in.size() - pos; }

    int64_t produce_fast(uint8_t* dst, int64_t cap) {
        if (hd == hp && !fend) {
            if (hp + 512 > hist.size()) {                          // keep the window, make room
                const size_t keep = std::min(hp, kWindow);
                std::memmove(hist.data(), hist.data() + hp - keep, keep);
                hp = hd = keep;
            }
            const uint8_t* base = in.data() + pos;
            const size_t have = (size_t)std::min<uint64_t>(avail(), comp_left);
            fdec->set_input(base, base + have, have == comp_left);
            uint8_t* o = hist.data() + hp;
            const int rc = fdec->run(&o, hist.data() + hist.size(), hist.data());
            const size_t used = (size_t)(fdec->input_pos() - base);
            pos += used;
            comp_left -= used;
            hp = (size_t)(o - hist.data());
            if (rc == fnpz_fast::Inflate::kCorrupt) return -1;
            if (rc == fnpz_fast::Inflate::kEnd) {
                fend = true;
                pos += (size_t)comp_left;                          // the member's last (partial) byte
                comp_left = 0;
            }
        }
        const int64_t n = std::min<int64_t>(cap, (int64_t)(hp - hd));
        if (n > 0) {
            std::memcpy(dst, hist.data() + hd, (size_t)n);
            hd += (size_t)n;
            crc = fnpz_fast::crc32((uint32_t)crc, dst, (size_t)n);
        }
        if (fend && hd == hp) zend = true;
        return n;
    }

    // Pull up to cap uncompressed bytes of the current member into dst. Returns the count
    // (crc updated); sets zend at the member's end; -1 on a corrupt stream.
    int64_t produce(uint8_t* dst, int64_t cap) {
        if (zend || cap <= 0) return 0;
        if (fast) return produce_fast(dst, cap);
        if (method == 0) {
            const int64_t n = (int64_t)std::min<uint64_t>({(uint64_t)cap, (uint64_t)avail(), raw_left});
            std::memcpy(dst, in.data() + pos, (size_t)n);
            pos += (size_t)n;
            raw_left -= (uint64_t)n;
            crc = crc32(crc, dst, (uInt)n);
            if (raw_left == 0) zend = true;
            return n;
        }
        zs.next_in = in.data() + pos;
        zs.avail_in = (uInt)std::min<size_t>(avail(), kChunk);
        zs.next_out = dst;
        zs.avail_out = (uInt)std::min<int64_t>(cap, kChunk);
        const uInt in0 = zs.avail_in, out0 = zs.avail_out;
        const int rc = inflate(&zs, Z_NO_FLUSH);
        pos += in0 - zs.avail_in;
        const int64_t n = out0 - zs.avail_out;
        crc = crc32(crc, dst, (uInt)n);
        if (rc == Z_STREAM_END) zend = true;
        else if (rc != Z_OK && rc != Z_BUF_ERROR) return -1;
        return n;
    }
};

namespace {

int sfail(fnpz_stream* s, int code, const char* fmt, const char* a) {
    s->err = code;
    return fail(code, fmt, a);
}

// local file header at s->in[s->pos]: 1 = parsed, 0 = need input, < 0 = -status
int stream_local_header(fnpz_stream* s) {
    const uint8_t* h = s->in.data() + s->pos;
    if (s->avail() < 30) return 0;
    const uint16_t nlen = rd16(h + 26), xlen = rd16(h + 28);
    if (s->avail() < 30u + nlen + xlen) return 0;
    s->flags = rd16(h + 6);
    s->method = rd16(h + 8);
    s->crc_want = rd32(h + 14);
    uint64_t csize = rd32(h + 18), usize = rd32(h + 22);
    s->name.assign(reinterpret_cast<const char*>(h + 30), nlen);
    s->zip64 = false;
    const uint8_t* x = h + 30 + nlen;
    const uint8_t* xe = x + xlen;
    while (x + 4 <= xe) {
        const uint16_t id = rd16(x), sz = rd16(x + 2);
        if (id == 0x0001) {                       // ZIP64 extended information
            s->zip64 = true;
            const uint8_t* v = x + 4;
            if (usize == 0xFFFFFFFFu && v + 8 <= x + 4 + sz) usize = rd64(v), v += 8;
            if (csize == 0xFFFFFFFFu && v + 8 <= x + 4 + sz) csize = rd64(v);
        }
        x += 4 + sz;
    }
    if (s->method != 0 && s->method != 8) return -sfail(s, FNPZ_EFORMAT, "%s: compression method unsupported", s->name.c_str());
    if (s->method == 0 && (s->flags & 8)) return -sfail(s, FNPZ_EFORMAT, "%s: stored member with a data descriptor", s->name.c_str());
    s->pos += 30u + nlen + xlen;
    s->raw_left = csize;
    s->fast = s->method == 8 && !(s->flags & 8);             // compressed size known: the codec's decoder
    if (s->fast) {
        s->fdec.reset(new fnpz_fast::Inflate(nullptr, 0));
        s->fend = false;
        s->comp_left = csize;
        if (s->hist.size() < fnpz_stream::kHistCap) s->hist.resize(fnpz_stream::kHistCap);
        s->hp = s->hd = 0;
    } else if (s->method == 8) {
        const int rc = s->zinit ? inflateReset(&s->zs) : inflateInit2(&s->zs, -MAX_WBITS);
        if (rc != Z_OK) return -sfail(s, FNPZ_ECORRUPT, "%s: inflate init failed", s->name.c_str());
        s->zinit = true;
    }
    s->zend = false;
    s->crc = crc32(0L, Z_NULL, 0);
    s->pend.clear();
    s->pend_pos = 0;
    (void)usize;
    return 1;
}

// .npy preamble + dict at the front of s->pend: 1 = parsed into *e, 0 = need more, < 0 = -status
int stream_npy_header(fnpz_stream* s, fnpz_entry* e) {
    const std::vector<uint8_t>& p = s->pend;
    if (p.size() < 10) return 0;
    if (std::memcmp(p.data(), "\x93NUMPY", 6) != 0) return -sfail(s, FNPZ_EFORMAT, "%s: not a .npy member", s->name.c_str());
    size_t hoff, hlen;
    if (p[6] == 1) {
        hoff = 10;
        hlen = rd16(p.data() + 8);
    } else if (p[6] == 2 || p[6] == 3) {
        if (p.size() < 12) return 0;
        hoff = 12;
        hlen = rd32(p.data() + 8);
    } else {
        return -sfail(s, FNPZ_EFORMAT, "%s: .npy version unsupported", s->name.c_str());
    }
    if (hoff + hlen > kMaxNpyHeader) return -sfail(s, FNPZ_EFORMAT, "%s: .npy header too long", s->name.c_str());
    if (p.size() < hoff + hlen) return 0;
    std::memset(e, 0, sizeof(*e));
    std::string nm = s->name;
    if (nm.size() >= 4 && nm.compare(nm.size() - 4, 4, ".npy") == 0) nm.resize(nm.size() - 4);
    if (nm.size() >= sizeof(e->name)) return -sfail(s, FNPZ_EFORMAT, "%s: member name too long", s->name.c_str());
    std::memcpy(e->name, nm.data(), nm.size());
    const std::string dict(reinterpret_cast<const char*>(p.data() + hoff), hlen);
    if (!parse_npy_dict(dict, e)) return -sfail(s, FNPZ_EFORMAT, "%s: unsupported .npy header", s->name.c_str());
    int64_t count = 1;
    for (int d = 0; d < e->ndim; ++d) count *= e->shape[d];
    e->nbytes = count * descr_itemsize(e->descr);
    e->npy_header = (int64_t)(hoff + hlen);
    e->method = s->method;
    e->crc32 = s->crc_want;
    s->pend_pos = hoff + hlen;
    s->left = e->nbytes;
    return 1;
}

}  // namespace

extern "C" {

int fnpz_abi_version(void) { return FNPZ_ABI_VERSION; }

int fnpz_inflate_raw(const uint8_t* in, int64_t in_len, uint8_t* out, int64_t out_len, int64_t window, int* stream_end) {
    return fnpz_internal::guard("fnpz_inflate_raw", [&]() -> int {
        g_err[0] = 0;
        if (in_len < 0 || out_len < 0 || window < 0 || (in_len > 0 && !in) || (out_len > 0 && !out))
            return fail(FNPZ_EINVAL, "fnpz_inflate_raw: bad arguments");
        std::unique_ptr<fnpz_fast::Inflate> dec(new fnpz_fast::Inflate(in, (size_t)in_len));
        uint8_t* o = out;
        uint8_t* const end = out + out_len;
        int rc = fnpz_fast::Inflate::kFull;
        while (rc == fnpz_fast::Inflate::kFull && o < end) {
            uint8_t* w = window > 0 ? std::min(end, o + window) : end;
            rc = dec->run(&o, w, out);
            if (rc == fnpz_fast::Inflate::kFull && o != w) break;
        }
        if (rc == fnpz_fast::Inflate::kFull && o == end) rc = dec->run(&o, end, out);   // the final block's end, if here
        if (stream_end) *stream_end = rc == fnpz_fast::Inflate::kEnd;
        if (rc == fnpz_fast::Inflate::kCorrupt)
            return fail(FNPZ_ECORRUPT, "fnpz_inflate_raw: invalid deflate stream (inflate.h:%d) after %lld bytes",
                        dec->error_line(), (long long)(o - out));
        if (o != end) return fail(FNPZ_ECORRUPT, "fnpz_inflate_raw: stream ended after %lld of %lld bytes", (long long)(o - out),
                                  (long long)out_len);
        return FNPZ_OK;
    });
}

void fnpz_parallel_config(int64_t min_member, int64_t min_chunk, int64_t* parallel, int64_t* fallback) {
    if (min_member > 0) g_par_min = min_member;
    if (min_chunk > 0) g_par_chunk = min_chunk;
    if (parallel) *parallel = g_par_ok.load();
    if (fallback) *fallback = g_par_fallback.load();
}

uint32_t fnpz_crc32(uint32_t crc, const uint8_t* data, int64_t len) {
    return len > 0 ? fnpz_fast::crc32(crc, data, (size_t)len) : crc;
}
const char* fnpz_last_error(void) { return g_err; }

int fnpz_open(const uint8_t* archive, int64_t len, fnpz_entry* entries, int max_entries, int* n_entries) {
    return fnpz_internal::guard("fnpz_open", [&]() -> int {
        g_err[0] = 0;
        if (!archive || len < 0 || !n_entries || (max_entries > 0 && !entries)) return fail(FNPZ_EINVAL, "fnpz_open: bad arguments");
        std::vector<CdEntry> cd;
        int rc = read_central(archive, len, cd);
        if (rc) return rc;
        *n_entries = (int)cd.size();
        if ((int)cd.size() > max_entries) return fail(FNPZ_ENOSPC, "fnpz_open: archive has %d members, room for %d", (int)cd.size(), max_entries);
        for (size_t i = 0; i < cd.size(); ++i)
            if ((rc = resolve_entry(archive, len, cd[i], &entries[i]))) return rc;
        return FNPZ_OK;
    });
}

int fnpz_read(const uint8_t* archive, int64_t len, const fnpz_entry* entries, int n, void* const* dsts, int threads) {
    return fnpz_internal::guard("fnpz_read", [&]() -> int {
        g_err[0] = 0;
        if (!archive || n < 0 || (n > 0 && (!entries || !dsts))) return fail(FNPZ_EINVAL, "fnpz_read: bad arguments");
        for (int i = 0; i < n; ++i) {
            if (entries[i].data_offset + entries[i].comp_size > len) return fail(FNPZ_EINVAL, "fnpz_read: entry %d out of range", i);
            if (entries[i].nbytes > 0 && !dsts[i]) return fail(FNPZ_EINVAL, "fnpz_read: dsts[%d] is NULL", i);
        }
        // tasks: one per member, or one per block of members that carry a block index
        struct Task { int member, block; };
        std::vector<Task> tasks;
        for (int i = 0; i < n; ++i) {
            if (entries[i].method == 8 && entries[i].index_count > 0)
                for (int b = 0; b < entries[i].index_count; ++b) tasks.push_back({i, b});
            else
                tasks.push_back({i, -1});
        }
        // a thread per MiB of compressed input at most: starting threads costs more than inflating a
        // small model's members (mnist-sized archives decode 1.8x faster on the calling thread alone)
        int64_t comp_total = 0;
        for (int i = 0; i < n; ++i) comp_total += entries[i].comp_size;
        const int64_t unit = std::max<int64_t>(1, std::min<int64_t>(1 << 20, g_par_chunk.load()));
        threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, comp_total / unit));
        std::vector<int> rcs(tasks.size(), FNPZ_OK);
        std::vector<uLong> bcrc(tasks.size(), 0);
        std::vector<std::string> errs(tasks.size());
        parallel_for((int)tasks.size(), threads, [&](int t) {
            const fnpz_entry& e = entries[tasks[t].member];
            void* dst = dsts[tasks[t].member];
            char msg[300] = "";
            if (tasks[t].block < 0) {
                // threads the other tasks leave idle decode this member's stream in parallel
                rcs[t] = decode_one(archive, e, dst, msg, sizeof(msg), std::max(1, threads / (int)tasks.size()));
            } else {
                const uint8_t* ix = archive + e.index_offset;
                const uint64_t B = rd64(ix + 8);
                const int b = tasks[t].block;
                const uint64_t c0 = rd64(ix + 16 + 8ull * b), c1 = rd64(ix + 16 + 8ull * (b + 1));
                const uint64_t r0 = B * (uint64_t)b, r1 = std::min<uint64_t>(r0 + B, (uint64_t)e.uncomp_size);
                if (c1 < c0 || c1 > (uint64_t)e.comp_size || r0 >= r1) {
                    rcs[t] = FNPZ_ECORRUPT;
                    snprintf(msg, sizeof(msg), "%s: bad block index", e.name);
                } else {
                    // block 0 starts with the .npy header; each block is its own deflate history
                    const uint64_t h0 = r0 < (uint64_t)e.npy_header ? (uint64_t)e.npy_header - r0 : 0;
                    if (r0 + h0 > r1) {
                        rcs[t] = FNPZ_ECORRUPT;
                        snprintf(msg, sizeof(msg), "%s: bad block index", e.name);
                    } else {
                        std::vector<uint8_t> hdr((size_t)h0);
                        uint8_t* out = static_cast<uint8_t*>(dst) + (r0 + h0 - (uint64_t)e.npy_header);
                        uint32_t crc = 0;
                        int line = 0;
                        if (inflate_split(archive + e.data_offset + c0, (int64_t)(c1 - c0), hdr.data(), (int64_t)h0, out,
                                          (int64_t)(r1 - r0 - h0), &crc, &line)) {
                            rcs[t] = FNPZ_ECORRUPT;
                            snprintf(msg, sizeof(msg), "%s: corrupt block %d (inflate.h:%d)", e.name, b, line);
                        }
                        bcrc[t] = crc;
                    }
                }
            }
            errs[t] = msg;
        });
        for (size_t t = 0; t < tasks.size(); ++t)
            if (rcs[t]) return fail(rcs[t], "%s", errs[t].c_str());
        // combine the block CRCs of indexed members, in order
        for (size_t t = 0; t < tasks.size();) {
            const int i = tasks[t].member;
            if (tasks[t].block < 0) {
                ++t;
                continue;
            }
            const fnpz_entry& e = entries[i];
            const uint64_t B = rd64(archive + e.index_offset + 8);
            uLong crc = 0;
            for (int b = 0; b < e.index_count; ++b, ++t) {
                const uint64_t r0 = B * (uint64_t)b, r1 = std::min<uint64_t>(r0 + B, (uint64_t)e.uncomp_size);
                crc = b == 0 ? bcrc[t] : crc32_combine(crc, bcrc[t], (z_off_t)(r1 - r0));
            }
            if ((uint32_t)crc != e.crc32) return fail(FNPZ_ECORRUPT, "%s: CRC-32 mismatch", e.name);
        }
        return FNPZ_OK;
    });
}

int64_t fnpz_write_bound(int n, const int64_t* header_lens, const int64_t* nbytes, const int32_t* name_lens) {
    int64_t total = 22 + 56 + 20;
    for (int i = 0; i < n; ++i) {
        const int64_t raw = header_lens[i] + nbytes[i];
        // deflate's worst case: fixed codes (Z_FIXED never falls back to stored blocks) expand by up to
        // 1/8 + block headers; the stored worst case (5 bytes per 16 KiB) is below that; plus per-block
        // flush markers and the zip records
        total += raw + raw / 8 + raw / 64 + (raw / 65536 + 2) * 72 + 2 * (30 + 46 + name_lens[i] + 4 + 20 + 28) + 64;
    }
    return total;
}

int fnpz_write(int n, const char* const* names, const uint8_t* const* headers, const int64_t* header_lens,
               const void* const* datas, const int64_t* nbytes, int level, int strategy, int threads, int64_t block,
               uint8_t* out, int64_t out_cap, int64_t* out_len) {
    return fnpz_internal::guard("fnpz_write", [&]() -> int {
        g_err[0] = 0;
        if (n < 0 || !out || !out_len || (n > 0 && (!names || !headers || !header_lens || !datas || !nbytes)))
            return fail(FNPZ_EINVAL, "fnpz_write: bad arguments");
        if (level < 0 || level > 9) return fail(FNPZ_EINVAL, "fnpz_write: level must be 0..9");
        if (strategy != FNPZ_STRATEGY_AUTO && (strategy < Z_DEFAULT_STRATEGY || strategy > Z_FIXED))
            return fail(FNPZ_EINVAL, "fnpz_write: strategy must be FNPZ_STRATEGY_AUTO or a zlib strategy 0..4");
        if (block <= 0) block = 4 << 20;
        block = std::min<int64_t>(std::max<int64_t>(block, 64 << 10), 1 << 30);
        std::vector<MemberSrc> src((size_t)n);
        std::vector<Block> blocks;
        std::vector<int64_t> mblock((size_t)n);
        for (int i = 0; i < n; ++i) {
            src[i] = MemberSrc{headers[i], header_lens[i], static_cast<const uint8_t*>(datas[i]), nbytes[i]};
            const int64_t total = header_lens[i] + nbytes[i];
            const int64_t B = std::max<int64_t>(block, (total + kMaxIndexBlocks - 1) / kMaxIndexBlocks);
            mblock[i] = B;
            for (int64_t b = 0; b < total || b == 0; b += B) {
                Block blk;
                blk.member = i;
                blk.begin = b;
                blk.len = std::min(B, total - b);
                blk.last = b + B >= total;
                blocks.push_back(std::move(blk));
                if (total == 0) break;
            }
        }
        parallel_for((int)blocks.size(), threads,
                     [&](int j) { deflate_block(src[blocks[j].member], blocks[j], level, strategy); });
        for (auto& b : blocks)
            if (b.rc != Z_OK) return fail(FNPZ_ECORRUPT, "fnpz_write: deflate failed on member %d", b.member);

        uint8_t* p = out;
        uint8_t* const lim = out + out_cap;
        std::vector<uint64_t> offs((size_t)n), comps((size_t)n);
        std::vector<uint32_t> crcs((size_t)n);
        size_t bi = 0;
        for (int i = 0; i < n; ++i) {
            const size_t nl = std::strlen(names[i]) + 4;
            uint64_t comp = 0;
            uLong crc = 0;
            size_t bj = bi;
            for (; bj < blocks.size() && blocks[bj].member == i; ++bj) {
                comp += blocks[bj].out.size();
                crc = bj == bi ? blocks[bj].crc : crc32_combine(crc, blocks[bj].crc, (z_off_t)blocks[bj].len);
            }
            const uint64_t raw = (uint64_t)(header_lens[i] + nbytes[i]);
            const int nblk = (int)(bj - bi);
            const int xl = 20 + 4 + 16 + 8 * (nblk + 1);
            if (p + 30 + nl + xl + comp > lim) return fail(FNPZ_ENOSPC, "fnpz_write: output buffer too small");
            offs[i] = (uint64_t)(p - out);
            comps[i] = comp;
            crcs[i] = (uint32_t)crc;
            wr32(p, kLocalSig);
            wr16(p + 4, 45);
            wr16(p + 6, 0);
            wr16(p + 8, 8);
            wr16(p + 10, 0);        // DOS time 00:00
            wr16(p + 12, 0x21);     // DOS date 1980-01-01
            wr32(p + 14, (uint32_t)crc);
            wr32(p + 18, 0xFFFFFFFFu);
            wr32(p + 22, 0xFFFFFFFFu);
            wr16(p + 26, (uint16_t)nl);
            wr16(p + 28, (uint16_t)xl);
            std::memcpy(p + 30, names[i], nl - 4);
            std::memcpy(p + 30 + nl - 4, ".npy", 4);
            uint8_t* x = p + 30 + nl;
            wr16(x, 1);
            wr16(x + 2, 16);
            wr64(x + 4, raw);
            wr64(x + 12, comp);
            x += 20;
            wr16(x, kIndexId);
            wr16(x + 2, (uint16_t)(16 + 8 * (nblk + 1)));
            wr32(x + 4, (uint32_t)nblk);
            wr32(x + 8, 0);
            wr64(x + 12, (uint64_t)mblock[i]);
            uint64_t off = 0;
            for (int b = 0; b <= nblk; ++b) {
                wr64(x + 20 + 8 * b, off);
                if (b < nblk) off += blocks[bi + b].out.size();
            }
            p = x + 20 + 8 * (nblk + 1);
            for (; bi < bj; ++bi) {
                std::memcpy(p, blocks[bi].out.data(), blocks[bi].out.size());
                p += blocks[bi].out.size();
                std::vector<uint8_t>().swap(blocks[bi].out);
            }
        }
        const uint64_t cd_off = (uint64_t)(p - out);
        for (int i = 0; i < n; ++i) {
            const size_t nl = std::strlen(names[i]) + 4;
            if (p + 46 + nl + 28 > lim) return fail(FNPZ_ENOSPC, "fnpz_write: output buffer too small");
            const uint64_t raw = (uint64_t)(header_lens[i] + nbytes[i]);
            wr32(p, kCentralSig);
            wr16(p + 4, 45);
            wr16(p + 6, 45);
            wr16(p + 8, 0);
            wr16(p + 10, 8);
            wr16(p + 12, 0);
            wr16(p + 14, 0x21);
            wr32(p + 16, crcs[i]);
            wr32(p + 20, 0xFFFFFFFFu);
            wr32(p + 24, 0xFFFFFFFFu);
            wr16(p + 28, (uint16_t)nl);
            wr16(p + 30, 28);
            wr16(p + 32, 0);
            wr16(p + 34, 0);
            wr16(p + 36, 0);
            wr32(p + 38, 0x01800000u);   // -rw------- (what zipfile writes for numpy)
            wr32(p + 42, 0xFFFFFFFFu);
            std::memcpy(p + 46, names[i], nl - 4);
            std::memcpy(p + 46 + nl - 4, ".npy", 4);
            uint8_t* x = p + 46 + nl;
            wr16(x, 1);
            wr16(x + 2, 24);
            wr64(x + 4, raw);
            wr64(x + 12, comps[i]);
            wr64(x + 20, offs[i]);
            p = x + 28;
        }
        const uint64_t cd_size = (uint64_t)(p - out) - cd_off;
        if (p + 56 + 20 + 22 > lim) return fail(FNPZ_ENOSPC, "fnpz_write: output buffer too small");
        const uint64_t z64 = (uint64_t)(p - out);
        wr32(p, kZ64EocdSig);
        wr64(p + 4, 44);
        wr16(p + 12, 45);
        wr16(p + 14, 45);
        wr32(p + 16, 0);
        wr32(p + 20, 0);
        wr64(p + 24, (uint64_t)n);
        wr64(p + 32, (uint64_t)n);
        wr64(p + 40, cd_size);
        wr64(p + 48, cd_off);
        p += 56;
        wr32(p, kZ64LocSig);
        wr32(p + 4, 0);
        wr64(p + 8, z64);
        wr32(p + 16, 1);
        p += 20;
        wr32(p, kEocdSig);
        wr16(p + 4, 0);
        wr16(p + 6, 0);
        wr16(p + 8, (uint16_t)std::min(n, 0xFFFF));
        wr16(p + 10, (uint16_t)std::min(n, 0xFFFF));
        wr32(p + 12, (uint32_t)std::min<uint64_t>(cd_size, 0xFFFFFFFFu));
        wr32(p + 16, (uint32_t)std::min<uint64_t>(cd_off, 0xFFFFFFFFu));
        wr16(p + 20, 0);
        p += 22;
        *out_len = (int64_t)(p - out);
        return FNPZ_OK;
    });
}

int fnpz_stream_open(fnpz_stream** s) {
    return fnpz_internal::guard("fnpz_stream_open", [&]() -> int {
        if (!s) return fail(FNPZ_EINVAL, "fnpz_stream_open: bad arguments");
        *s = new fnpz_stream();
        return FNPZ_OK;
    });
}

void fnpz_stream_close(fnpz_stream* s) { delete s; }

int fnpz_stream_feed(fnpz_stream* s, const uint8_t* data, int64_t len) {
    return fnpz_internal::guard("fnpz_stream_feed", [&]() -> int {
        if (!s || len < 0 || (len > 0 && !data)) return fail(FNPZ_EINVAL, "fnpz_stream_feed: bad arguments");
        if (s->pos > 0 && s->pos >= s->in.size() / 2) {      // drop consumed input
            s->in.erase(s->in.begin(), s->in.begin() + (std::ptrdiff_t)s->pos);
            s->pos = 0;
        }
        s->in.insert(s->in.end(), data, data + len);
        return FNPZ_OK;
    });
}

int fnpz_stream_next(fnpz_stream* s, uint8_t* out, int64_t out_cap, int* event, fnpz_entry* entry, int64_t* out_len) {
    return fnpz_internal::guard("fnpz_stream_next", [&]() -> int {
        if (!s || !event || !out_len || (out_cap > 0 && !out)) return fail(FNPZ_EINVAL, "fnpz_stream_next: bad arguments");
        *out_len = 0;
        if (s->err) return fail(s->err, "fnpz_stream_next: the stream already failed");
        for (;;) {
            switch (s->st) {
            case fnpz_stream::HDR: {
                if (s->avail() < 4) return *event = FNPZ_EV_NEED_INPUT, FNPZ_OK;
                const uint32_t sig = rd32(s->in.data() + s->pos);
                if (sig == kCentralSig || sig == kEocdSig || sig == kZ64EocdSig || sig == kZ64LocSig) {
                    s->st = fnpz_stream::END;
                    continue;
                }
                if (sig != kLocalSig) return sfail(s, FNPZ_EFORMAT, "%s", "not a zip local file header");
                const int rc = stream_local_header(s);
                if (rc < 0) return -rc;
                if (rc == 0) return *event = FNPZ_EV_NEED_INPUT, FNPZ_OK;
                s->st = fnpz_stream::NPY;
                continue;
            }
            case fnpz_stream::NPY: {
                if (!entry) return fail(FNPZ_EINVAL, "fnpz_stream_next: a member header needs an entry");
                const int rc = stream_npy_header(s, entry);
                if (rc < 0) return -rc;
                if (rc == 1) {
                    s->st = fnpz_stream::DATA;
                    return *event = FNPZ_EV_MEMBER, FNPZ_OK;
                }
                if (s->zend) return sfail(s, FNPZ_ECORRUPT, "%s: truncated .npy header", s->name.c_str());
                const size_t old = s->pend.size();
                s->pend.resize(old + 4096);
                const size_t pos0 = s->pos;
                const int64_t n = s->produce(s->pend.data() + old, 4096);
                if (n < 0) return sfail(s, FNPZ_ECORRUPT, "%s: corrupt deflate stream", s->name.c_str());
                s->pend.resize(old + (size_t)n);
                if (n == 0 && s->pos == pos0 && !s->zend) return *event = FNPZ_EV_NEED_INPUT, FNPZ_OK;
                continue;
            }
            case fnpz_stream::DATA: {
                if (s->pend_pos < s->pend.size()) {                // payload inflated with the header
                    const int64_t have = (int64_t)(s->pend.size() - s->pend_pos);
                    if (have > s->left) return sfail(s, FNPZ_EFORMAT, "%s: more data than its .npy header declares", s->name.c_str());
                    const int64_t n = std::min(have, out_cap);
                    if (n == 0) return fail(FNPZ_EINVAL, "fnpz_stream_next: payload pending and no output window");
                    std::memcpy(out, s->pend.data() + s->pend_pos, (size_t)n);
                    s->pend_pos += (size_t)n;
                    s->left -= n;
                    *out_len = n;
                    return *event = FNPZ_EV_DATA, FNPZ_OK;
                }
                const size_t pos0 = s->pos;
                if (s->left > 0) {
                    if (out_cap <= 0) return fail(FNPZ_EINVAL, "fnpz_stream_next: payload pending and no output window");
                    if (s->zend) return sfail(s, FNPZ_ECORRUPT, "%s: member shorter than its .npy header declares", s->name.c_str());
                    const int64_t n = s->produce(out, std::min(out_cap, s->left));
                    if (n < 0) return sfail(s, FNPZ_ECORRUPT, "%s: corrupt deflate stream", s->name.c_str());
                    if (n > 0) {
                        s->left -= n;
                        *out_len = n;
                        return *event = FNPZ_EV_DATA, FNPZ_OK;
                    }
                    if (s->pos == pos0 && !s->zend) return *event = FNPZ_EV_NEED_INPUT, FNPZ_OK;
                    continue;
                }
                if (!s->zend) {                                    // payload complete: the stream must end here
                    uint8_t extra;
                    const int64_t n = s->produce(&extra, 1);
                    if (n < 0) return sfail(s, FNPZ_ECORRUPT, "%s: corrupt deflate stream", s->name.c_str());
                    if (n > 0) return sfail(s, FNPZ_EFORMAT, "%s: more data than its .npy header declares", s->name.c_str());
                    if (!s->zend) {
                        if (s->pos == pos0) return *event = FNPZ_EV_NEED_INPUT, FNPZ_OK;
                        continue;
                    }
                }
                if (s->flags & 8) {
                    s->st = fnpz_stream::DESC;
                    continue;
                }
                if ((uint32_t)s->crc != s->crc_want) return sfail(s, FNPZ_ECORRUPT, "%s: CRC-32 mismatch", s->name.c_str());
                s->st = fnpz_stream::HDR;
                return *event = FNPZ_EV_MEMBER_END, FNPZ_OK;
            }
            case fnpz_stream::DESC: {
                if (s->avail() < 4) return *event = FNPZ_EV_NEED_INPUT, FNPZ_OK;
                const bool has_sig = rd32(s->in.data() + s->pos) == kDescSig;
                const size_t size = (has_sig ? 4 : 0) + 4 + (s->zip64 ? 16 : 8);
                if (s->avail() < size) return *event = FNPZ_EV_NEED_INPUT, FNPZ_OK;
                const uint32_t crc = rd32(s->in.data() + s->pos + (has_sig ? 4 : 0));
                s->pos += size;
                if ((uint32_t)s->crc != crc) return sfail(s, FNPZ_ECORRUPT, "%s: CRC-32 mismatch", s->name.c_str());
                s->st = fnpz_stream::HDR;
                return *event = FNPZ_EV_MEMBER_END, FNPZ_OK;
            }
            case fnpz_stream::END:
                return *event = FNPZ_EV_END, FNPZ_OK;
            }
        }
    });
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// host staging: gather copy on a persistent worker pool
// ---------------------------------------------------------------------------------------
namespace {

// Workers created once and parked on a condition variable; run() hands them one job at a time
// (callers are serialised) and the calling thread works on it too. A worker joins a job only
// while it is posted (under the lock), so run() returns once every joined worker has left it.
class CopyPool {
   public:
    // One pool per process: a child forked while the parent's workers existed gets a fresh pool
    // (the parent's threads do not exist in it, and its mutexes may have been copied locked). Pools
    // are never destroyed: their parked workers end with the process.
    static CopyPool& get() {
        static std::mutex m;
        static CopyPool* pool = nullptr;
        static pid_t owner = 0;
        std::lock_guard<std::mutex> lk(m);
        if (!pool || owner != getpid()) {
            pool = new CopyPool();
            owner = getpid();
        }
        return *pool;
    }
    void run(int threads, int n, const std::function<void(int)>& f) {
        std::lock_guard<std::mutex> call(call_mu_);
        std::atomic<int> next{0};
        Job job{&f, n, &next};
        {
            std::lock_guard<std::mutex> lk(mu_);
            try {
                while ((int)workers_.size() < threads - 1) workers_.emplace_back([this] { work(); });
            } catch (...) {
                // no more threads: the parked ones and the caller copy
            }
            job_ = &job;
            ++gen_;
        }
        cv_.notify_all();
        for (int i; (i = next.fetch_add(1)) < n;) f(i);
        std::unique_lock<std::mutex> lk(mu_);
        job_ = nullptr;                          // late wakers see no job
        idle_.wait(lk, [this] { return active_ == 0; });
    }

   private:
    struct Job {
        const std::function<void(int)>* f;
        int n;
        std::atomic<int>* next;
    };
    void work() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            Job* j = job_;
            if (!j) continue;
            ++active_;
            lk.unlock();
            for (int i; (i = j->next->fetch_add(1)) < j->n;) (*j->f)(i);
            lk.lock();
            if (--active_ == 0) idle_.notify_all();
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, idle_;
    std::vector<std::thread> workers_;
    Job* job_ = nullptr;
    uint64_t gen_ = 0;
    int active_ = 0;
    bool stop_ = false;   // never set: the pool lives as long as the process
};

}  // namespace

// Asynchronous gathers (fnpz_gather_start / fnpz_gather_wait): a caller that packs many small
// updates one after the other (staging arenas) hands each update's copies to one background thread
// and goes on with the next update; the thread takes every queued job at once and copies them on the
// CopyPool. Jobs complete in submission order, so a ticket is done once the completed count reaches
// it. One queue per process (fork-safe like CopyPool).
//
// Latency: a round of a small model queues a few jobs tens of microseconds apart and then waits for
// the last one right away, so a thread that parks between jobs (a futex wake-up on each side costs
// ~10-20 us) would cost more than the copies. The worker therefore spins for kSpinUs after a job
// before parking, and a waiter spins as long for its ticket before blocking; a batch under
// kThreadBytes per thread is copied by the worker alone (waking pool threads costs more).
class GatherQueue {
   public:
    struct Piece {
        uint8_t* d;
        const uint8_t* s;
        int64_t len;
    };
    static constexpr int64_t kSpinUs = 200;
    static constexpr int64_t kThreadBytes = 512 << 10;
    static GatherQueue& get() {
        static std::mutex m;
        static GatherQueue* q = nullptr;
        static pid_t owner = 0;
        std::lock_guard<std::mutex> lk(m);
        if (!q || owner != getpid()) {
            q = new GatherQueue();
            owner = getpid();
        }
        return *q;
    }
    int64_t submit(std::vector<Piece>&& pieces, int threads) {
        std::lock_guard<std::mutex> lk(mu_);
        if (!started_) {
            std::thread([this] { work(); }).detach();
            started_ = true;
        }
        const int64_t t = ++issued_;
        for (auto& p : pieces) pending_.push_back(p);
        threads_ = std::max(threads_, threads);
        last_.store(t, std::memory_order_release);
        cv_.notify_one();
        return t;
    }
    void wait(int64_t t) {
        if (spin_until([&] { return done_.load(std::memory_order_acquire) >= t; })) return;
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return done_.load(std::memory_order_acquire) >= t; });
    }

   private:
    template <class F>
    static bool spin_until(F ready) {
        const auto end = std::chrono::steady_clock::now() + std::chrono::microseconds(kSpinUs);
        for (int i = 0;; ++i) {
            if (ready()) return true;
            if ((i & 63) == 63 && std::chrono::steady_clock::now() > end) return false;
            __builtin_ia32_pause();
        }
    }
    void work() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            if (last_.load(std::memory_order_relaxed) <= done_.load(std::memory_order_relaxed)) {
                lk.unlock();                                 // idle: spin a while before parking
                spin_until([&] { return last_.load(std::memory_order_acquire) > done_.load(std::memory_order_relaxed); });
                lk.lock();
            }
            cv_.wait(lk, [&] { return last_.load(std::memory_order_relaxed) > done_.load(std::memory_order_relaxed); });
            std::vector<Piece> batch;
            batch.swap(pending_);
            const int64_t upto = last_.load(std::memory_order_relaxed);
            const int threads = threads_;
            threads_ = 1;
            lk.unlock();
            int64_t total = 0;
            for (auto& p : batch) total += p.len;
            const int np = (int)batch.size();
            auto copy = [&](int k) { std::memcpy(batch[k].d, batch[k].s, (size_t)batch[k].len); };
            const int t = (int)std::min<int64_t>(threads, std::max<int64_t>(1, total / kThreadBytes));
            if (t <= 1 || np <= 1)
                for (int k = 0; k < np; ++k) copy(k);
            else
                CopyPool::get().run(std::min(t, np), np, copy);
            lk.lock();
            done_.store(upto, std::memory_order_release);
            done_cv_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<Piece> pending_;
    int64_t issued_ = 0;
    std::atomic<int64_t> last_{0}, done_{0};
    int threads_ = 1;
    bool started_ = false;
};

// Every destination segment inside the caller's buffer [lo, lo + len): checked before anything is
// copied or queued, so an accounting slip above (a full arena, a wrong offset) is a status, not a
// write past a pinned block.
static int check_window(const char* who, int n, void* const* dsts, const int64_t* nbytes, const void* lo, int64_t len) {
    if (n > 0 && (!lo || len < 0)) return fail(FNPZ_EINVAL, "%s: no destination window", who);
    const uintptr_t w0 = reinterpret_cast<uintptr_t>(lo);
    for (int i = 0; i < n; ++i) {
        if (nbytes[i] == 0) continue;
        const uintptr_t d = reinterpret_cast<uintptr_t>(dsts[i]);
        if (d < w0 || d - w0 > (uint64_t)len || (uint64_t)nbytes[i] > (uint64_t)len - (d - w0))
            return fail(FNPZ_ENOSPC, "%s: segment %d (%lld bytes at offset %lld) outside the %lld-byte destination buffer",
                        who, i, (long long)nbytes[i], (long long)((int64_t)d - (int64_t)w0), (long long)len);
    }
    return FNPZ_OK;
}

static int64_t gather_start(int n, void* const* dsts, const void* const* srcs, const int64_t* nbytes, int threads,
                            const void* dst_lo, int64_t dst_len) {
    if (n < 0 || (n > 0 && (!dsts || !srcs || !nbytes)) || threads < 1)
        return -fail(FNPZ_EINVAL, "fnpz_gather_start: bad arguments");
    for (int i = 0; i < n; ++i)
        if (nbytes[i] < 0 || (nbytes[i] > 0 && (!dsts[i] || !srcs[i])))
            return -fail(FNPZ_EINVAL, "fnpz_gather_start: segment %d", i);
    if (int rc = check_window("fnpz_gather_start", n, dsts, nbytes, dst_lo, dst_len)) return -rc;
    std::vector<GatherQueue::Piece> pieces;
    for (int i = 0; i < n; ++i) {
        // 64 KiB pieces: a small update (one tensor dominating, e.g. mnist's 200 KB first layer) still
        // spreads over several threads
        for (int64_t o = 0; o < nbytes[i]; o += 1 << 16)
            pieces.push_back({static_cast<uint8_t*>(dsts[i]) + o, static_cast<const uint8_t*>(srcs[i]) + o,
                              std::min<int64_t>(1 << 16, nbytes[i] - o)});
    }
    return GatherQueue::get().submit(std::move(pieces), threads);
}

extern "C" int64_t fnpz_gather_start(int n, void* const* dsts, const void* const* srcs, const int64_t* nbytes,
                                     int threads, const void* dst_lo, int64_t dst_len) {
    int64_t ticket = 0;
    const int rc = fnpz_internal::guard("fnpz_gather_start", [&]() -> int {
        ticket = gather_start(n, dsts, srcs, nbytes, threads, dst_lo, dst_len);
        return ticket < 0 ? (int)-ticket : FNPZ_OK;
    });
    return rc ? -(int64_t)rc : ticket;
}

extern "C" int fnpz_gather_wait(int64_t ticket) {
    return fnpz_internal::guard("fnpz_gather_wait", [&]() -> int {
        if (ticket <= 0) return fail(FNPZ_EINVAL, "fnpz_gather_wait: bad ticket %lld", (long long)ticket);
        GatherQueue::get().wait(ticket);
        return FNPZ_OK;
    });
}

extern "C" int fnpz_gather(int n, void* const* dsts, const void* const* srcs, const int64_t* nbytes, int threads,
                           const void* dst_lo, int64_t dst_len) {
    return fnpz_internal::guard("fnpz_gather", [&]() -> int {
        if (n < 0 || (n > 0 && (!dsts || !srcs || !nbytes)) || threads < 1)
            return fail(FNPZ_EINVAL, "fnpz_gather: bad arguments");
        int64_t total = 0;
        for (int i = 0; i < n; ++i) {
            if (nbytes[i] < 0 || (nbytes[i] > 0 && (!dsts[i] || !srcs[i]))) return fail(FNPZ_EINVAL, "fnpz_gather: segment %d", i);
            total += nbytes[i];
        }
        if (int rc = check_window("fnpz_gather", n, dsts, nbytes, dst_lo, dst_len)) return rc;
        if (total == 0) return FNPZ_OK;
        struct Piece {
            uint8_t* d;
            const uint8_t* s;
            int64_t len;
        };
        const int64_t piece = std::max<int64_t>(1 << 20, (total + 2 * threads - 1) / (2 * threads));
        std::vector<Piece> pieces;
        for (int i = 0; i < n; ++i)
            for (int64_t o = 0; o < nbytes[i]; o += piece)
                pieces.push_back({static_cast<uint8_t*>(dsts[i]) + o, static_cast<const uint8_t*>(srcs[i]) + o,
                                  std::min(piece, nbytes[i] - o)});
        const int np = (int)pieces.size();
        auto copy = [&](int k) { std::memcpy(pieces[k].d, pieces[k].s, (size_t)pieces[k].len); };
        const int t = std::min(threads, np);
        if (t <= 1) {
            for (int k = 0; k < np; ++k) copy(k);
            return FNPZ_OK;
        }
        CopyPool::get().run(t, np, copy);
        return FNPZ_OK;
    });
}
