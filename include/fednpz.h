/*
 * fednpz.h — C ABI of libfednpz.so, the native .npz wire codec (host side, C++ + zlib).
 *
 * FEDn moves every model as an `np.savez_compressed` archive (a ZIP of deflated .npy
 * files): numpyhelper.Helper.save / load (fedn/utils/helpers/plugins/numpyhelper.py:
 * 144-189), model_as_bytesIO / load_model_from_bytes / serialize_model_to_BytesIO
 * (fedn/network/combiner/modelservice.py:57-75, 110-146). Decoding a 100 M-param update
 * takes ~2.8 s and encoding the aggregate ~17 s there, more than the
 * aggregation itself. This codec reads an archive in memory and inflates every .npy
 * payload straight into caller-provided (e.g. pinned) buffers, entries in parallel, and
 * writes archives with a block-parallel deflate (independent blocks joined by sync
 * flushes form one valid deflate stream; CRC-32s are combined). Archives it writes are
 * ordinary ZIP64 npz files that np.load reads; decoded arrays are byte-identical.
 *
 * All functions return 0 on success or a positive FNPZ_E* status; fnpz_last_error()
 * holds a thread-local message.
 */
#ifndef FEDNPZ_H
#define FEDNPZ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FNPZ_ABI_VERSION 7
#define FNPZ_MAX_DIMS 64   /* numpy 2's NPY_MAXDIMS (ABI 6; 16 before) */

/* Every entry point returns a status; no C++ exception leaves the library. FNPZ_ENOMEM (ABI 6):
 * memory or a worker thread could not be had inside the call — nothing was returned, and the
 * library stays usable (fnpz_last_error() says which). */
enum fnpz_status { FNPZ_OK = 0, FNPZ_EFORMAT = 1, FNPZ_ECORRUPT = 2, FNPZ_EINVAL = 3, FNPZ_ENOSPC = 4, FNPZ_EFALLBACK = 5,
                   FNPZ_ENOMEM = 6 };

/* One archive member holding a .npy array. */
typedef struct {
    char name[256];           /* member name without the ".npy" suffix (numpy: "0", "1", ...) */
    char descr[32];           /* numpy dtype string, e.g. "<f4" */
    int32_t fortran_order;
    int32_t ndim;
    int64_t shape[FNPZ_MAX_DIMS];
    int64_t nbytes;           /* payload bytes after the .npy header */
    int64_t npy_header;       /* bytes of the .npy preamble + header dict */
    int64_t data_offset;      /* offset of the member's (compressed) data in the archive */
    int64_t comp_size;
    int64_t uncomp_size;      /* npy_header + nbytes */
    uint32_t crc32;
    int32_t method;           /* 0 stored, 8 deflated */
    int64_t index_offset;     /* archive offset of this codec's block index (0 if absent) */
    int32_t index_count;      /* independently inflatable blocks (0 if absent) */
    int32_t reserved;
} fnpz_entry;

int fnpz_abi_version(void);
const char* fnpz_last_error(void);

/* Parse the central directory and every member's .npy header (only the header bytes are
 * inflated). Writes up to max_entries entries in archive order; *n_entries = count (also
 * set when FNPZ_ENOSPC reports that max_entries was too small). */
int fnpz_open(const uint8_t* archive, int64_t len, fnpz_entry* entries, int max_entries, int* n_entries);

/* Inflate the payload of entries[i] into dsts[i] (entries[i].nbytes bytes each), checking
 * each member's CRC-32. Members are decoded by up to `threads` threads; members written by
 * fnpz_write carry a block index and are additionally split across threads by block. */
int fnpz_read(const uint8_t* archive, int64_t len, const fnpz_entry* entries, int n, void* const* dsts, int threads);

/* Upper bound of the archive size fnpz_write produces for these members. */
int64_t fnpz_write_bound(int n, const int64_t* header_lens, const int64_t* nbytes, const int32_t* name_lens);

/* Write an npz archive: member i is names[i] + ".npy" = headers[i] (a complete .npy
 * preamble + header dict, e.g. from numpy.lib.format.write_array_header_1_0) followed by
 * datas[i] (nbytes[i] bytes). level: zlib level (numpy uses 6; 0 stores); strategy: a zlib
 * strategy (Z_DEFAULT_STRATEGY 0 ... Z_FIXED 4) or FNPZ_STRATEGY_AUTO (ABI 5): run-length matching
 * (Z_RLE) per block — as small or smaller and several times faster on model weights — with the
 * default strategy at level 1 kept instead where it is smaller on a block that shrinks below 60 %;
 * threads: deflate workers; block: bytes per independently deflated block (0 = 4 MiB).
 * *out_len = bytes written. Any deflate stream np.load reads: the arrays are what was written. */
#define FNPZ_STRATEGY_AUTO (-1)
int fnpz_write(int n, const char* const* names, const uint8_t* const* headers, const int64_t* header_lens,
               const void* const* datas, const int64_t* nbytes, int level, int strategy, int threads, int64_t block,
               uint8_t* out, int64_t out_cap, int64_t* out_len);

/* numpy-identical writer (ABI 6): the exact bytes np.savez_compressed writes for these members —
 * numpyhelper.Helper.save (fedn/utils/helpers/plugins/numpyhelper.py:144-169, np.savez_compressed at
 * :162). Member i is names[i] + ".npy" = headers[i] (the .npy preamble numpy writes for the array:
 * numpy.lib.format._write_array_header) followed by datas[i] (nbytes[i] bytes in numpy's write order:
 * C order, or F order for a Fortran-contiguous array), deflated the way zipfile does it — zlib level
 * 6, raw (wbits -15), memLevel 8, default strategy, the header in one deflate() call and the payload
 * in calls of seg_bytes[i] bytes (numpy's 16 MiB // itemsize elements; NULL or <= 0: one call) — and
 * wrapped in zipfile's headers (ZIP64 local extra on every member, 1980-01-01 timestamps, ZIP64
 * central / end records only past zipfile's limits). Members deflate on up to `threads` threads.
 * The output bound is fnpz_write_bound's. *out_len = bytes written. */
int fnpz_savez(int n, const char* const* names, const uint8_t* const* headers, const int64_t* header_lens,
               const void* const* datas, const int64_t* nbytes, const int64_t* seg_bytes, int threads,
               uint8_t* out, int64_t out_cap, int64_t* out_len);

/* fnpz_savez's single-stream parallel deflate (fedn_amd/csrc/pdeflate.h): a member of at least
 * min_member bytes (default 32 MiB), or of at least 4 chunks and more than 1/threads of the archive,
 * is deflated on every thread in chunks of `chunk` bytes (default 4 MiB) by a reimplementation of
 * zlib 1.2.11's level-6 parse and trees.c whose output is zlib's, byte for byte; an input it does not model falls back to zlib itself. Values <= 0 keep a setting.
 * *parallel / *fallback (may be NULL): members that went parallel / fell back so far. */
void fnpz_savez_config(int64_t min_member, int64_t chunk, int64_t* parallel, int64_t* fallback);

/* Which libz fnpz_savez's big members may bypass (ABI 7). pdeflate.h reproduces zlib 1.2.11's
 * level-6 stream only; a big member takes it while the process's libz reports a modelled version,
 * equals the libz Python's zlib runs (zlib.ZLIB_RUNTIME_VERSION: numpy's archive comes from it) and
 * passes a self-test (one 1.5 MiB member through both, byte for byte), checked once, at the first
 * big member. Otherwise EVERY member goes through the process's libz, so an archive never mixes two
 * deflaters. fnpz_savez_zlib_expect records Python's runtime version (NULL keeps it) and, for tests,
 * force_zlib = 1 acts as a failed check (0 clears it, < 0 keeps it); the check is then redone.
 * fnpz_savez_zlib_status returns 1 when big members may take pdeflate.h, else 0, and copies the
 * reason into reason[0, cap). */
void fnpz_savez_zlib_expect(const char* runtime_version, int force_zlib);
int fnpz_savez_zlib_status(char* reason, int64_t cap);

/* Phase times (s) of fnpz_savez's last big member (ABI 7): out[0..8) = input copy, parse, sync,
 * window schedule + tail replay, block plan, encode, CRC, archive assembly, and out[8] the last
 * call's total. Returns how many were written (9 at most; with out NULL, how many there are). */
int fnpz_savez_stats(double* out, int n);

/* zipfile's ZIP64_LIMIT ((1 << 31) - 1) and ZIP_FILECOUNT_LIMIT ((1 << 16) - 1) as fnpz_savez applies
 * them (sizes / offsets past the first: ZIP64 fields and version 45; more members than the second,
 * or a central directory past the first: ZIP64 end records). Values <= 0 restore those defaults.
 * For tests: with smaller limits, and CPython's zipfile patched to the same, the ZIP64 branches are
 * compared with np.savez_compressed at kilobyte sizes. */
void fnpz_savez_zip_limits(int64_t zip64_limit, int64_t filecount_limit);

/* That deflate on its own (tests): in[0, len) fed as deflate(Z_NO_FLUSH) calls ending at ends[0 ..
 * nends) (ends[nends - 1] == len) and then Z_FINISH, raw (wbits -15), level 6, memLevel 8. FNPZ_OK
 * with the stream in out, or FNPZ_EFALLBACK (fnpz_last_error says why) where the caller must use
 * zlib. After FNPZ_OK, fnpz_last_error() describes the run (chunks, fix-ups, blocks). */
int fnpz_deflate_exact(const uint8_t* in, int64_t len, const int64_t* ends, int nends, int threads, int64_t chunk,
                       uint8_t* out, int64_t out_cap, int64_t* out_len);

/* Test hook: 1 if in[] holds a plausible dynamic-Huffman block header at input bit `bit` (the
 * parallel decoder's candidate filter: block type, code counts and a complete precode). */
int fnpz_probe_dynamic_header(const uint8_t* in, int64_t len, int64_t bit);

/* Streaming reader — an archive decoded while it arrives (ModelService.Upload chunks,
 * fedn/network/combiner/modelservice.py:198-221), members taken from their local headers in
 * archive order. Feed input with fnpz_stream_feed (copied), then call fnpz_stream_next until
 * it reports FNPZ_EV_NEED_INPUT:
 *   FNPZ_EV_MEMBER      *entry = the next member (name without ".npy", descr, fortran_order,
 *                       shape, nbytes); its payload follows as FNPZ_EV_DATA events
 *   FNPZ_EV_DATA        *out_len (> 0) payload bytes were inflated into out[0..out_cap); pass a
 *                       window of at most the member's remaining bytes
 *   FNPZ_EV_MEMBER_END  the member's payload is complete and its CRC-32 matched
 *   FNPZ_EV_END         the central directory was reached: every member has been delivered
 * An error status is sticky: the stream stays failed. */
typedef struct fnpz_stream fnpz_stream;
enum fnpz_event { FNPZ_EV_NEED_INPUT = 0, FNPZ_EV_MEMBER = 1, FNPZ_EV_DATA = 2, FNPZ_EV_MEMBER_END = 3, FNPZ_EV_END = 4 };

int fnpz_stream_open(fnpz_stream** stream);
void fnpz_stream_close(fnpz_stream* stream);
int fnpz_stream_feed(fnpz_stream* stream, const uint8_t* data, int64_t len);
int fnpz_stream_next(fnpz_stream* stream, uint8_t* out, int64_t out_cap, int* event, fnpz_entry* entry,
                     int64_t* out_len);

/* Raw DEFLATE (RFC 1951) decode of in[0, in_len) into out[0, out_len), in windows of `window`
 * bytes (0: one window; the decoder resumes at any output position) — the decoder fnpz_read
 * inflates whole members and blocks with (fedn_amd/csrc/inflate.h; ABI 5). FNPZ_OK once out is
 * full (*stream_end = 1 if the stream's final block ended there); FNPZ_ECORRUPT on an invalid or
 * truncated stream, or one that ends before out is full. */
int fnpz_inflate_raw(const uint8_t* in, int64_t in_len, uint8_t* out, int64_t out_len, int64_t window, int* stream_end);

/* Parallel decode of ONE large deflate stream (round 4, fnpz_read): a member of at least
 * min_member compressed bytes (default 16 MiB) is cut into chunks of at least min_chunk bytes
 * (default 4 MiB) decoded by the threads the other members leave idle — chunk starts found as
 * block headers, back-references into the unknown history carried as markers, every chunk
 * verified to end exactly where the next begins, the member's CRC-32 checked; anything that does
 * not hold falls back to the sequential decode. Values <= 0 keep the current setting.
 * *parallel / *fallback (may be NULL): decodes that went parallel / fell back so far. */
void fnpz_parallel_config(int64_t min_member, int64_t min_chunk, int64_t* parallel, int64_t* fallback);

/* CRC-32 of the zip format with zlib's convention (crc32(0, ...) starts; pass the previous value to
 * continue), folded with carry-less multiplies where the CPU has them (ABI 5). */
uint32_t fnpz_crc32(uint32_t crc, const uint8_t* data, int64_t len);

/* Host staging (beside the wire format; the aggregators' pack of a decoded update into its pinned
 * staging buffer, fedn_amd/layout.py): dsts[i][0, nbytes[i]) = srcs[i][0, nbytes[i]) for i < n,
 * cut into pieces of at least 1 MiB that up to `threads` threads copy (the calling thread and a
 * pool created once per process: no thread start-up per call). Regions must not overlap.
 * [dst_lo, dst_lo + dst_len) is the destination buffer the caller allocated (a pinned slot or
 * arena): every destination segment must lie inside it, else nothing is copied and FNPZ_ENOSPC is
 * returned (ABI 4) — a caller whose own accounting slipped gets an error, not heap corruption. */
int fnpz_gather(int n, void* const* dsts, const void* const* srcs, const int64_t* nbytes, int threads,
                const void* dst_lo, int64_t dst_len);

/* The same copies, asynchronously: queued to one background thread (which copies every queued job
 * at once on up to `threads` threads) and returned at once. Returns a ticket > 0, or -status
 * (-FNPZ_ENOSPC: a segment outside [dst_lo, dst_lo + dst_len); nothing queued).
 * fnpz_gather_wait(ticket) blocks until that job — and every job submitted before it — is done.
 * The caller keeps the sources and destinations alive until then. */
int64_t fnpz_gather_start(int n, void* const* dsts, const void* const* srcs, const int64_t* nbytes, int threads,
                          const void* dst_lo, int64_t dst_len);
int fnpz_gather_wait(int64_t ticket);

#ifdef __cplusplus
}
#endif

#endif /* FEDNPZ_H */
