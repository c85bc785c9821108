/*
 * fedagg_probe.h — measurement and tuning entry points of `libfedagg_probe.so`.
 *
 * NOT part of the drop-in boundary: the product library `libfedagg.so` exports only
 * include/fedagg.h, built with the measured-best launch settings as compile-time constants
 * (no mutable or process-global state). `libfedagg_probe.so` is the same source compiled with
 * -DFEDAGG_PROBES: it exports everything fedagg.h declares PLUS the knobs and probe kernels
 * below, which tools/ (microbench, PMC probes, A/B runs) and the division tests use to measure
 * alternatives. Knob settings are process-global (atomics) within the probe library only.
 */
#ifndef FEDAGG_PROBE_H
#define FEDAGG_PROBE_H

#include "fedagg.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Measurement helpers (not part of the reference interface): achievable-peak
 * reference kernels for the roofline section of bench.py.
 *   fa_stream_copy  dst[i] = src[i], 16 B per lane
 *   fa_stream_read  reads `bytes` and writes one 16-B word per workgroup to `sink`
 *                   (sink must hold >= 16 * fa_stream_read_blocks(bytes) bytes)
 */
int fa_stream_copy(void* dst, const void* src, int64_t bytes, void* stream);
/* out[i] = sum_k bufs[k][i] (fp32, K <= 64) with exactly the traversal of the FedAvg fold
 * kernel but one add per element: the access-pattern ceiling of fa_fedavg_fold.        */
int fa_stream_sum(float* out, const float* const* bufs, int K, int64_t P, void* stream);

/* Launch-geometry knobs of the fp32 FedAvg kernel (process-global; measurement and
 * tuning only, results are identical for every setting):
 *   FA_TUNE_STRIPS  16-B strips per lane (1 | 2 | 4 | 8 | 16)
 *   FA_TUNE_UNROLL  clients loaded before folding (1 | 2 | 4 | 8 | 16)
 *   (instantiated pairs: see launch_fedavg_vec; other pairs fall back to 1 x 8)
 *   FA_TUNE_NT      non-temporal loads of the client buffers (0 | 1)
 *   FA_TUNE_FASTDIV fp32 t/N via the exact RN64(1/N) product (1, default) or IEEE
 *                   division (0); both are correctly rounded
 *   FA_TUNE_LANETAB pipelined kernel (unroll 0) reads the client table from registers
 *                   via v_readlane (1) or by scalar loads (0)
 *   FA_TUNE_GRID    pipelined kernel: 0 = one 16-KiB-per-client tile per workgroup,
 *                   n = persistent grid of n workgroups per CU sweeping tiles        */
enum fa_tune_knob { FA_TUNE_STRIPS = 0, FA_TUNE_UNROLL = 1, FA_TUNE_NT = 2, FA_TUNE_FASTDIV = 3, FA_TUNE_LANETAB = 4,
                    FA_TUNE_GRID = 5, FA_TUNE_READ = 6 /* fa_stream_read loads per lane: 4 | 8 | 16 */,
                    FA_TUNE_BLOCK = 7 /* pipelined kernel workgroup size 256 | 512 | 1024 */,
                    FA_TUNE_SUM_NOSTORE = 8 /* fa_stream_sum probe: 1 = skip the store (reads + adds only) */,
                    FA_TUNE_NT_STORE = 9 /* aggregate stores: 0 plain, 1 non-temporal, 2 write-through (sc1) */,
                    FA_TUNE_FASTDIV64 = 10 /* fp64 t/N via RN64(1/N) + two exact Markstein corrections (1,
                                              default) or IEEE division (0); both correctly rounded */,
                    FA_TUNE_TILEMAP = 11 /* pipelined kernel: workgroup -> tile order, 0 identity or runs of
                                            R = 2 | 4 | 8 | 16 | 32 consecutive tiles per XCD */,
                    FA_TUNE_OPT_NT = 12 /* FedOpt client loads non-temporal (1, product) or cached (0) */,
                    FA_TUNE_OPT_NOSTORE = 13 /* FedOpt FIRST|FINAL launch: 1 = skip the stores (reads + math) */,
                    FA_TUNE_OPT_STORE = 14 /* FedOpt FIRST|FINAL, strip map (OPT_COAL 0): stores 0 plain, 1 nt, 2 sc1 */,
                    FA_TUNE_OPT_COAL = 15 /* FedOpt FIRST|FINAL element map: 2 = the product's (k_fedopt_c, 4
                                             coalesced pairs per lane, nt stores), 1 = 2 pairs per lane,
                                             0 = the r01 per-lane 4-element strip map */,
                    FA_TUNE_NARROW = 16 /* bf16 -> f32 FedAvg: 1 = the product's 8-B client strips / 16-B
                                           aggregate strips (4 elements, 8 strips per lane: every wave store
                                           one contiguous 1 KiB), 0 = r01's 16-B client strips (8 elements,
                                           4 per lane) */,
                    FA_TUNE_LDS = 17 /* occupancy probe: KiB of (unused) dynamic LDS per workgroup of the fold
                                        and FedOpt kernels, 0..64 */,
                    FA_TUNE_WPE = 18 /* occupancy probe: fp32 fold / FedOpt FIRST|FINAL kernels compiled for at
                                        least W waves per SIMD (0 = compiler's choice, 5, 6, 8) */,
                    FA_TUNE_OPT_MV = 19 /* layout probe, FedOpt FIRST|FINAL steady state: 1 = fp64 m and v
                                           interleaved per 512-element wave tile in ONE buffer passed as
                                           m_in / m_out (2P doubles each; P % 2048 == 0) */,
                    FA_TUNE_AUTO_GEOM = 20 /* 1 (default) = with the default geometry knobs, the product's
                                              size-dependent choice (4-strip pipelined kernel only for client
                                              buffers >= 160 MiB, else 1 strip x 4/8 clients ahead); 0 = the
                                              knobs as set, at every size */,
                    FA_TUNE_OPT_MIX = 21 /* FedOpt FIRST|FINAL, access-pattern probe: 1 = k_fedopt_c's exact loads
                                            and stores with one add per value instead of the arithmetic
                                            (results are NOT the reference's; a ragged last 2048-element
                                            tile is skipped) */,
                    FA_TUNE_OPT_BURST = 22 /* FedOpt FIRST|FINAL, burst-store probe (fp64 m out): G = 1, 2 or 4
                                              wave tiles per wave with k_fedopt_mix's loads, the new v / out / m
                                              of all G held in registers and stored together after the last
                                              tile's reads (0 = off; a ragged last group is skipped) */,
                    FA_TUNE_OPT_G = 23 /* FedOpt FINAL launches over an fp64 model with fp64 state out: the
                                          product arithmetic with G = 1, 2 or 4 wave tiles per wave and their
                                          v / out / m stored after the last tile's reads (0 = off) */,
                    FA_TUNE_OPT_WIN_PERIOD = 24 /* FedOpt FIRST|FINAL, clock-windowed store probe (fp64 m out):
                                                k_fedopt_mix's pattern with every store issued only while the
                                                100 MHz reference clock mod value < OPT_WIN_W
                                                (period in 10-ns ticks, 64 .. 2^24; 0 = off) */,
                    FA_TUNE_OPT_WIN_W = 25 /* the store window in 10-ns ticks */,
                    FA_TUNE_OPT_WIN_MODE = 26 /* 0: gate the stores only; 1: also start a tile's reads outside
                                                 the window; 2: also every client batch's reads */,
                    FA_TUNE_AVG_WIN_PERIOD = 27 /* FedAvg fp32 k_fedavg_pipe (the headline instantiation): its
                                                   store window — 0 = the product's own (avg_store_window),
                                                   -1 = none, > 0 = this period with AVG_WIN_W / _MODE */,
                    FA_TUNE_AVG_WIN_W = 28,
                    FA_TUNE_AVG_WIN_MODE = 29,
                    FA_TUNE_OPT_WIN_PROD = 30 /* 1: OPT_WIN_PERIOD / _W apply to the product step (k_fedopt_cw,
                                                 bit-identical) instead of the pattern probe; OPT_WIN_PERIOD 0 =
                                                 the product's own window (opt_store_window), -1 = none */,
                    FA_TUNE_OPT_QUAD = 31 /* FedOpt over bf16 updates, fp64 old, fp64 pg (configs[4]'s waves):
                                             1 = k_fedopt_cq, lane L owning 4-element quads at lane stride 4
                                             (dwordx2 client loads) instead of the product's pairs */ };
int fa_tune(int knob, int value);
int64_t fa_stream_read_blocks(int64_t bytes);
int fa_stream_read(const void* src, int64_t bytes, void* sink, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_PROBE_H */
