// fedagg.hip — gfx950 (MI355X) kernels + C ABI for FEDn's combiner-side aggregation.
//
// The hot path is an elementwise, HBM-bound recurrence over K client buffers:
//   FedAvg  (numpyhelper.py:32, fedavg.py:47-71):   x <- x + (n_k*(y_k - x))/N_k
//   FedOpt  (fedopt.py:74-118):  pg <- running mean of (y_k - old), then one
//           Adam/Yogi/AdaGrad server step (fedopt.py:151-258) over (old, m, v).
// Every output element depends only on the same element of the inputs, and the
// client order is fixed by FEDn's FIFO queue, so parallelism is across elements:
// one lane owns a 16-byte strip of elements, keeps the running aggregate in
// registers for all K clients (no LDS round trip: nothing is shared between
// lanes), issues the K strip loads U at a time so every wave has U x 1 KiB in
// flight, and stores once. Bit-exact parity with numpy requires replaying the
// op order with IEEE rounding at every step: this file is compiled with
// -ffp-contract=off and relies on hipcc's correctly rounded f32/f64 `/` and
// f64 sqrt (checked against the golden fixtures).
//
// Client tables (pointer, n_k, N_k) travel in the kernarg segment (<= 64 clients
// per launch, ~1.5 KiB): they are read by scalar loads, need no H2D copy and keep
// launches graph-capturable. K > 64 is chunked by the host code below; the chunks
// continue from the stored aggregate, which replays the same recurrence exactly.

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <atomic>
#include <cstring>
#include <type_traits>
#include <vector>

#include "../../include/fedagg.h"
#ifdef FEDAGG_PROBES
#include "../../include/fedagg_probe.h"
#endif

namespace {

// ----------------------------------------------------------------------------
// error plumbing
// ----------------------------------------------------------------------------
thread_local char g_err[512] = "";
// the kernel family the calling thread's last fold / FedOpt launch used (fa_last_kernel): a diagnostic
// like g_err, so a benchmark names the kernel that ran, not one it infers
thread_local const char* g_kernel = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FA_EHIP, "%s: %s", what, hipGetErrorString(e));
    return FA_OK;
}

constexpr int kMaxK = 64;     // clients per launch (kernarg table)
constexpr int kBlock = 256;   // 4 waves
constexpr int kUnroll = 8;    // client strips in flight per lane

size_t dt_size(int dt) {
    switch (dt) {
        case FA_F32: return 4;
        case FA_F64: return 8;
        case FA_BF16: return 2;
        case FA_F16: return 2;
        case FA_I32: return 4;
        case FA_I64: return 8;
        default: return 0;
    }
}

// ----------------------------------------------------------------------------
// element types and exact conversions
// ----------------------------------------------------------------------------
struct bf16 { uint16_t bits; };
struct f16 { uint16_t bits; };

__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float(static_cast<uint32_t>(b) << 16); }
__device__ __forceinline__ float f16_to_f32(uint16_t b) {
    __half h;
    __builtin_memcpy(&h, &b, 2);
    return __half2float(h);
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
    __half h = __float2half_rn(f);
    uint16_t b;
    __builtin_memcpy(&b, &h, 2);
    return b;
}

// ----------------------------------------------------------------------------
// compute policies: the arithmetic numpy performs for each dtype
// ----------------------------------------------------------------------------
struct CF32 {            // float32 ufunc loops
    using V = float;     // register type
    using S = float;     // scalar (n, N) type
    using T = float;     // storage type (FedOpt's pseudo-gradient workspace)
    __device__ static __forceinline__ V fold(V x, V y, S n, S N, double r) {
        V t[1] = {x}, yy[1] = {y};
        fold_strip<1>(t, yy, n, N, r);
        return t[0];
    }
    // One client step over E elements: x <- x + (n*(y-x))/N.
    // t/N is correctly rounded. N is the same for every element of a client step, so
    // the host supplies r = RN64(1/N) and the quotient is RN32(RN64(t * r)): its
    // relative error is < 2^-52, while t/N (t, N binary32, N's odd part < 2^24) is
    // never closer than 2^-49 (relative) to a binary32 rounding midpoint in the normal
    // range, so the final rounding lands where IEEE division does (DESIGN.md has the
    // argument; tests/test_gpu_divide.py checks every binary32 t exhaustively).
    // r == 0 (host: N == 0, |N| >= 2^28, or fa_tune) selects IEEE division; lanes with
    // 0 < |t| < 2^-98 (a subnormal quotient is possible) redo it with IEEE division.
    template <int E>
    __device__ static __forceinline__ void fold_strip(V (&x)[E], const V (&y)[E], S n, S N, double r) {
        V t[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            t[e] = y[e] - x[e];
            t[e] = n * t[e];
        }
        if (r != 0.0) {
            V q[E];
            bool small = false;   // |t| < 2^-98, zeros included: one compare per element
#pragma unroll
            for (int e = 0; e < E; ++e) {
                q[e] = (float)((double)t[e] * r);
                small |= __builtin_fabsf(t[e]) < 0x1p-98f;
            }
            if (__builtin_expect(small, 0)) {
                // zero lanes already hold the right signed zero (t*r); only nonzero tiny t divide
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (__builtin_fabsf(t[e]) < 0x1p-98f && t[e] != 0.0f) q[e] = t[e] / N;
            }
#pragma unroll
            for (int e = 0; e < E; ++e) x[e] = x[e] + q[e];
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e) x[e] = x[e] + t[e] / N;
        }
    }
};
struct CF64 {            // float64 ufunc loops
    using V = double;
    using S = double;
    using T = double;
    // RN64(t/N) without a division when the host supplies r = RN64(1/N) (r == 0: IEEE
    // division). q0 = RN(t*r) is within 1.5 ulp of z = t/N; one Markstein step
    // q1 = RN(q0 + RN(t - q0*N)*r) makes it faithful (the error left is ~2^-52 of q0's);
    // for a faithful q the remainder t - q*N is exact (FMA), and q2 = RN(q1 + (t - q1*N)*r)
    // lands within |z - q1|*|N*r - 1| < 2^-53.x ulp of z, which is closer than z can be to a
    // rounding midpoint without being one (|z - mid| >= ulp/(2*N') with N' < 2^53 N's odd
    // significand; z is never exactly a midpoint), so q2 = RN(z). DESIGN.md §3.2b has the
    // argument. The bounds |t| in [2^-600, 2^600] (host: |N| in [2^-60, 2^60]) keep every
    // intermediate and remainder normal; other lanes (0, tiny, huge, inf, NaN) divide.
    __device__ static __forceinline__ V div(V t, S N, double r) {
        if (r != 0.0) {
            const double a = __builtin_fabs(t);
            if (a >= 0x1p-600 && a <= 0x1p600) {
                double q = t * r;
                double e = __builtin_fma(-q, N, t);
                q = __builtin_fma(e, r, q);
                e = __builtin_fma(-q, N, t);
                return __builtin_fma(e, r, q);
            }
            if (a == 0.0) return t * r;   // signed zero: sign(t) * sign(N), as t / N
        }
        return t / N;
    }
    __device__ static __forceinline__ V fold(V x, V y, S n, S N, double r) {
        V t = y - x;
        t = n * t;
        t = div(t, N, r);
        return x + t;
    }
};
struct CF16 {            // numpy half loops: op in float, round to half after every op
    using V = float;     // holds a value exactly representable in f16
    using S = float;     // n, N pre-rounded to f16 on the host
    using T = f16;
    __device__ static __forceinline__ V rh(float a) { return f16_to_f32(f32_to_f16(a)); }
    __device__ static __forceinline__ V fold(V x, V y, S n, S N, double) {
        V t = rh(y - x);
        t = rh(n * t);
        t = rh(t / N);
        return rh(x + t);
    }
};

// Server-function aggregation rules, the two the reference ships as
// examples of user `aggregate` / `incremental_aggregate` code (hooks.py:109-143):
//
// CWSUM — examples/server-functions/server_functions.py:58-67
//     weighted_sum[i] += client_parameters[i] * num_examples
//   the product is taken in the update dtype Y (python scalar w is weak: cast to Y), the sum
//   in promote(acc, Y), the result stored back in the accumulator dtype X (in-place +=).
template <typename Y, typename X>
struct CWSUM {
    static constexpr bool kF32 = std::is_same<Y, float>::value && std::is_same<X, float>::value;
    using V = typename std::conditional<kF32, float, double>::type;
    using S = double;
    __device__ static __forceinline__ V fold(V x, V y, S w, S, double) {
        V s;
        if constexpr (std::is_same<Y, float>::value) {
            const float p = (float)y * (float)w;     // y holds an exact f32 value
            s = x + (V)p;
        } else {
            s = x + y * w;                           // f64 product, f64 sum
        }
        if constexpr (std::is_same<X, float>::value && std::is_same<V, double>::value)
            return (double)(float)s;                 // += into an f32 accumulator rounds every step
        else
            return s;
    }
};

// CRUN — examples/server-functions/sf_incremental_aggregation.py:36-37
//     g = (g * (T - n) + m * n) / T       (T = running total including this client)
//   g and m share the dtype T_; every python scalar is cast to it (numpy weak scalars) and each
//   operation rounds in it: RN(RN(RN(g*a) + RN(m*b)) / T). The client table carries
//   b = n in n[], T in N[] and a = T - n in r[].
template <typename T_>
struct CRUN {
    using V = T_;
    using S = double;
    __device__ static __forceinline__ V fold(V x, V y, S b, S T, double a) {
        const V u = x * (V)a;
        const V w = y * (V)b;
        const V s = u + w;
        return s / (V)T;
    }
};

template <class CP> struct is_nostore : std::false_type {};
#ifdef FEDAGG_PROBES
struct CADD {            // measurement only: x <- x + y (same traversal as the fold, minimal VALU)
    using V = float;
    using S = float;
    __device__ static __forceinline__ V fold(V x, V y, S, S, double) { return x + y; }
};
struct CADDNW : CADD {};  // measurement only: CADD whose store is skipped (never-true data test)
template <> struct is_nostore<CADDNW> : std::true_type {};
#endif

// element-wise client step for policies without a strip-level shortcut
template <class CP, int E>
__device__ __forceinline__ void fold_strip(typename CP::V (&x)[E], const typename CP::V (&y)[E], typename CP::S n,
                                           typename CP::S N, double r) {
    if constexpr (std::is_same<CP, CF32>::value) {
        CP::template fold_strip<E>(x, y, n, N, r);
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = CP::fold(x[e], y[e], n, N, r);
    }
}

// load one element of storage type T, widened to the compute register type V
template <typename T, typename V> __device__ __forceinline__ V widen(T v) { return static_cast<V>(v); }
template <> __device__ __forceinline__ float widen<bf16, float>(bf16 v) { return bf16_to_f32(v.bits); }
template <> __device__ __forceinline__ double widen<bf16, double>(bf16 v) { return (double)bf16_to_f32(v.bits); }
template <> __device__ __forceinline__ float widen<f16, float>(f16 v) { return f16_to_f32(v.bits); }

template <typename T, typename V> __device__ __forceinline__ T narrow(V v) { return static_cast<T>(v); }
template <> __device__ __forceinline__ f16 narrow<f16, float>(float v) { return f16{f32_to_f16(v)}; }

// ----------------------------------------------------------------------------
// 16-byte strip loads/stores (E elements of T). NT = non-temporal (read-once data)
// ----------------------------------------------------------------------------
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <typename T, int E, bool NT>
__device__ __forceinline__ void strip_load(const T* __restrict__ p, T (&r)[E]) {
    constexpr int bytes = E * (int)sizeof(T);
    if constexpr (bytes % 16 == 0) {
        const u32x4* q = reinterpret_cast<const u32x4*>(p);
#pragma unroll
        for (int j = 0; j < bytes / 16; ++j) {
            u32x4 w = NT ? __builtin_nontemporal_load(q + j) : q[j];
            __builtin_memcpy(reinterpret_cast<char*>(r) + 16 * j, &w, 16);
        }
    } else if constexpr (bytes == 8) {          // one dwordx2 (8-B aligned: the caller's contract)
        const u32x2* q = reinterpret_cast<const u32x2*>(p);
        u32x2 w = NT ? __builtin_nontemporal_load(q) : *q;
        __builtin_memcpy(reinterpret_cast<char*>(r), &w, 8);
    } else if constexpr (bytes == 4) {          // one dword (4-B aligned)
        const unsigned int* q = reinterpret_cast<const unsigned int*>(p);
        unsigned int w = NT ? __builtin_nontemporal_load(q) : *q;
        __builtin_memcpy(reinterpret_cast<char*>(r), &w, 4);
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) r[e] = p[e];
    }
}

// SM (store mode): 0 plain (write-back in L2), 1 non-temporal, 2 write-through (`sc1`,
// MI355X_MICROARCH.md "stores of each flavour": the line leaves L2 as the store issues)
template <typename T, int E, int SM = 0>
__device__ __forceinline__ void strip_store(T* __restrict__ p, const T (&r)[E]) {
    constexpr int bytes = E * (int)sizeof(T);
    if constexpr (bytes == 8 && SM == 0) {
        u32x2 w;
        __builtin_memcpy(&w, reinterpret_cast<const char*>(r), 8);
        *reinterpret_cast<u32x2*>(p) = w;
    } else if constexpr (bytes == 8 && SM == 1) {
        u32x2 w;
        __builtin_memcpy(&w, reinterpret_cast<const char*>(r), 8);
        __builtin_nontemporal_store(w, reinterpret_cast<u32x2*>(p));
    } else if constexpr (bytes % 16 == 0) {
        u32x4* q = reinterpret_cast<u32x4*>(p);
#pragma unroll
        for (int j = 0; j < bytes / 16; ++j) {
            u32x4 w;
            __builtin_memcpy(&w, reinterpret_cast<const char*>(r) + 16 * j, 16);
            if constexpr (SM == 1) __builtin_nontemporal_store(w, q + j);
            else if constexpr (SM == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(q + j), "v"(w) : "memory");
            else q[j] = w;
        }
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) p[e] = r[e];
    }
}

// ----------------------------------------------------------------------------
// FedAvg fold kernel
// ----------------------------------------------------------------------------
template <typename S>
struct ClientTable {
    const void* ptr[kMaxK];
    S n[kMaxK];
    S N[kMaxK];
    double r[kMaxK];   // RN64(1/N) for CF32's division shortcut, 0 = use IEEE division
};

// Start one strip's running value. INIT: x := updates[0] (the `model = model_next`
// alias, fedavg.py:65-66); else x := agg (continuing a chunked / streamed fold).
// INT_FIRST: integer updates; the first fold runs in integer arithmetic (numpy int
// subtract + multiply wrap), then true_divide to f64 (numpyhelper.py:32 on int arrays).
// Returns the first client index still to fold.
template <typename Y, typename X, class CP, int E, bool INIT, bool INT_FIRST, bool NT>
__device__ __forceinline__ int strip_start(typename CP::V (&x)[E], const X* __restrict__ agg,
                                           const ClientTable<typename CP::S>& tab, int64_t i0, int rem) {
    using V = typename CP::V;
    if constexpr (INIT) {
        const Y* y0p = static_cast<const Y*>(tab.ptr[0]) + i0;
        Y y0[E];
        if (rem == E) strip_load<Y, E, NT>(y0p, y0);
        else {
#pragma unroll
            for (int e = 0; e < E; ++e) y0[e] = e < rem ? y0p[e] : Y{};
        }
        if constexpr (INT_FIRST) {
            const Y* y1p = static_cast<const Y*>(tab.ptr[1]) + i0;   // K >= 2 guaranteed by the host
            using U = typename std::make_unsigned<Y>::type;
            const U n1 = (U)(int64_t)tab.n[1];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const Y y1 = e < rem ? y1p[e] : Y{};
                U t = (U)y1 - (U)y0[e];   // wrapping subtract
                t = n1 * t;               // wrapping multiply
                x[e] = (double)y0[e] + (double)(Y)t / (double)tab.N[1];
            }
            return 2;
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e) x[e] = widen<Y, V>(y0[e]);
            return 1;
        }
    } else {
        X xa[E];
        if (rem == E) strip_load<X, E, false>(agg + i0, xa);
        else {
#pragma unroll
            for (int e = 0; e < E; ++e) xa[e] = e < rem ? agg[i0 + e] : X{};
        }
#pragma unroll
        for (int e = 0; e < E; ++e) x[e] = widen<X, V>(xa[e]);
        return 0;
    }
}

// The grid's last block: its strips may be ragged or past the end of the buffers.
template <typename Y, typename X, class CP, int E, int S, bool INIT, bool INT_FIRST, int BLK = kBlock>
__device__ __forceinline__ void k_fedavg_tail(X* __restrict__ agg, const ClientTable<typename CP::S>& tab, const int K,
                                           const int64_t P, const int64_t strip0) {
    using V = typename CP::V;
    for (int s = 0; s < S; ++s) {
        const int64_t i0 = (strip0 + s * BLK) * E;
        if (i0 >= P) break;
        const int rem = (P - i0) < E ? (int)(P - i0) : E;
        V x[E];
        int k = strip_start<Y, X, CP, E, INIT, INT_FIRST, false>(x, agg, tab, i0, rem);
        for (; k < K; ++k) {
            const Y* yp = static_cast<const Y*>(tab.ptr[k]) + i0;
            const typename CP::S n = tab.n[k], N = tab.N[k];
            const double r = tab.r[k];
            for (int e = 0; e < rem; ++e) x[e] = CP::fold(x[e], widen<Y, V>(yp[e]), n, N, r);
        }
        for (int e = 0; e < rem; ++e) agg[i0 + e] = narrow<X, V>(x[e]);
    }
}

// Destinations a piece is pushed to besides its own buffer (the peers' model buffers, IPC-mapped
// or in-process): fa_push and the fused fold + push (fa_fedavg_fold_push).
constexpr int kPushMax = 16;
struct PushTable {
    u32x4* dst[kPushMax];
};

// k_fedavg with the all-gather fused in (fa_fedavg_fold_push; sharded.P2PAllGather engine "fused"):
// every finished strip is stored to this rank's own copy of the model AND to each peer's copy — the
// same vector stores a copy kernel would issue, straight from the registers that hold the result, so
// a round needs no second pass over the piece and no second launch. fp32 updates and aggregate,
// 16-B aligned buffers, one strip per lane; the fold arithmetic and order are k_fedavg's.
template <int U, bool INIT>
__global__ void __launch_bounds__(kBlock)
k_fedavg_push(float* __restrict__ agg, const ClientTable<CF32::S> tab, const int K, const int64_t P, PushTable t,
              const int nd) {
    using V = CF32::V;
    constexpr int E = 4;
    const int64_t strip = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t i0 = strip * E;
    if (i0 + E <= P) {
        V x[E];
        int k = strip_start<float, float, CF32, E, INIT, false, false>(x, agg, tab, i0, E);
        for (; k + U <= K; k += U) {
            float y[U][E];
#pragma unroll
            for (int u = 0; u < U; ++u) strip_load<float, E, false>(static_cast<const float*>(tab.ptr[k + u]) + i0, y[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                V yv[E];
#pragma unroll
                for (int e = 0; e < E; ++e) yv[e] = widen<float, V>(y[u][e]);
                fold_strip<CF32, E>(x, yv, tab.n[k + u], tab.N[k + u], tab.r[k + u]);
            }
        }
        for (; k < K; ++k) {
            float y[E];
            strip_load<float, E, false>(static_cast<const float*>(tab.ptr[k]) + i0, y);
            V yv[E];
#pragma unroll
            for (int e = 0; e < E; ++e) yv[e] = widen<float, V>(y[e]);
            fold_strip<CF32, E>(x, yv, tab.n[k], tab.N[k], tab.r[k]);
        }
        float xo[E];
#pragma unroll
        for (int e = 0; e < E; ++e) xo[e] = narrow<float, V>(x[e]);
        u32x4 w;
        __builtin_memcpy(&w, xo, 16);
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(agg + i0));
        for (int d = 0; d < nd; ++d) __builtin_nontemporal_store(w, t.dst[d] + strip);
    } else if (i0 < P) {                                       // the ragged last strip
        const int rem = (int)(P - i0);
        V x[E];
        int k = strip_start<float, float, CF32, E, INIT, false, false>(x, agg, tab, i0, rem);
        for (; k < K; ++k) {
            const float* yp = static_cast<const float*>(tab.ptr[k]) + i0;
            for (int e = 0; e < rem; ++e) x[e] = CF32::fold(x[e], widen<float, V>(yp[e]), tab.n[k], tab.N[k], tab.r[k]);
        }
        for (int e = 0; e < rem; ++e) {
            const float v = narrow<float, V>(x[e]);
            agg[i0 + e] = v;
            for (int d = 0; d < nd; ++d) reinterpret_cast<float*>(t.dst[d])[i0 + e] = v;
        }
    }
}

// A system-scope release on every XCD after a grid that stored into other GPUs' memory
// (k_fedavg_push, k_push): the stores still held in an XCD's L2 are written back before anything
// later on the stream (the fence the ranks exchange). A release inside every wave of a large grid
// would write the L2s back hundreds of thousands of times, so a separate grid of kReleaseBlocks
// single-wave workgroups releases instead — but HIP does not promise which XCDs a grid's workgroups
// land on, so each workgroup reads the XCD it runs on (HW_REG_XCC_ID) and ORs it into the caller's
// release record (FA_REL_*, include/fedagg.h). The launch's last workgroup to arrive (an acq_rel
// arrival counter: it sees every other workgroup's bit) compares the number of distinct XCDs covered
// with the device's XCD count and counts a miss; the record is read by the caller at its next synchronisation
// (sharded.P2PAllGather.check_release), which fails the session on any miss. The mask and the
// arrival counter are reset by that last workgroup, so the next launch on the stream starts clean.
constexpr int kReleaseBlocks = 64;
constexpr unsigned kXccIdReg = (3u << 11) | 20u;   // s_getreg operand: HW_REG_XCC_ID, offset 0, 4 bits

__global__ void __launch_bounds__(64) k_release(unsigned* __restrict__ rec, unsigned expect) {
    if (threadIdx.x != 0) return;
    __threadfence_system();
    if (rec == nullptr) return;
    const unsigned xcc = __builtin_amdgcn_s_getreg(kXccIdReg) & 15u;
    __hip_atomic_fetch_or(rec + FA_REL_MASK, 1u << xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned before = __hip_atomic_fetch_add(rec + FA_REL_ARRIVED, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (before + 1 != gridDim.x) return;
    const unsigned seen = __hip_atomic_exchange(rec + FA_REL_MASK, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(rec + FA_REL_ARRIVED, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_or(rec + FA_REL_SEEN, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(rec + FA_REL_LAUNCHES, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(rec + FA_REL_EXPECT, expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // distinct XCDs seen vs the device's count (a partition mode may number its XCDs by their
    // physical index rather than 0 .. n - 1: the mask is reported, the count is what is checked)
    if (__builtin_popcount(seen) < __builtin_popcount(expect))
        __hip_atomic_fetch_add(rec + FA_REL_MISSES, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// XCDs of the current device (1 in a partition mode that exposes one XCD per device)
int device_xccs(int dev, int* n) {
    int v = 0;
    hipError_t e = hipDeviceGetAttribute(&v, hipDeviceAttributeNumberOfXccs, dev);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(FA_EHIP, "hipDeviceGetAttribute(NumberOfXccs, %d): %s", dev, hipGetErrorString(e));
    }
    if (v < 1 || v > 16) return fail(FA_EHIP, "device %d reports %d XCDs", dev, v);
    *n = v;
    return FA_OK;
}

int launch_release(hipStream_t st, unsigned* rec) {
    unsigned expect = 0;
    if (rec) {
        int dev = 0, nx = 0;
        (void)hipGetDevice(&dev);
        const int rc = device_xccs(dev, &nx);
        if (rc) return rc;
        expect = (nx >= 32) ? ~0u : ((1u << nx) - 1u);
    }
    hipLaunchKernelGGL(k_release, dim3(kReleaseBlocks), dim3(64), 0, st, rec, expect);
    return check_launch("release after peer stores");
}

// One lane owns S strips of E elements (strip s at lane + s*kBlock within the block's
// span, so every wave instruction stays a contiguous 1 KiB). U clients' strips are
// loaded before any of them is folded, so a lane keeps U*S 16-B loads in flight.
template <typename Y, typename X, class CP, int E, int S, int U, bool INIT, bool INT_FIRST, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedavg(X* __restrict__ agg, const ClientTable<typename CP::S> tab, const int K, const int64_t P) {
    using V = typename CP::V;
    using Sc = typename CP::S;
    const int64_t strip0 = (int64_t)blockIdx.x * (kBlock * S) + threadIdx.x;
    if ((strip0 + (int64_t)(S - 1) * kBlock) * E + E <= P) {
        V x[S][E];
        int k = 0;
#pragma unroll
        for (int s = 0; s < S; ++s)
            k = strip_start<Y, X, CP, E, INIT, INT_FIRST, NT>(x[s], agg, tab, (strip0 + s * kBlock) * E, E);
        for (; k + U <= K; k += U) {
            Y y[U][S][E];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const Y* yp = static_cast<const Y*>(tab.ptr[k + u]);
#pragma unroll
                for (int s = 0; s < S; ++s) strip_load<Y, E, NT>(yp + (strip0 + s * kBlock) * E, y[u][s]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const Sc n = tab.n[k + u], N = tab.N[k + u];
                const double r = tab.r[k + u];
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    V yv[E];
#pragma unroll
                    for (int e = 0; e < E; ++e) yv[e] = widen<Y, V>(y[u][s][e]);
                    fold_strip<CP, E>(x[s], yv, n, N, r);
                }
            }
        }
        for (; k < K; ++k) {
            const Y* yp = static_cast<const Y*>(tab.ptr[k]);
            Y y[S][E];
#pragma unroll
            for (int s = 0; s < S; ++s) strip_load<Y, E, NT>(yp + (strip0 + s * kBlock) * E, y[s]);
            const Sc n = tab.n[k], N = tab.N[k];
            const double r = tab.r[k];
#pragma unroll
            for (int s = 0; s < S; ++s) {
                V yv[E];
#pragma unroll
                for (int e = 0; e < E; ++e) yv[e] = widen<Y, V>(y[s][e]);
                fold_strip<CP, E>(x[s], yv, n, N, r);
            }
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
            X xo[E];
#pragma unroll
            for (int e = 0; e < E; ++e) xo[e] = narrow<X, V>(x[s][e]);
            strip_store<X, E>(agg + (strip0 + s * kBlock) * E, xo);
        }
    } else {
        k_fedavg_tail<Y, X, CP, E, S, INIT, INT_FIRST>(agg, tab, K, P, strip0);
    }
}

// Software-pipelined variant: while client k's S strips are folded, client k+1's are
// already in flight (two register buffers, explicit ping-pong), so a lane never waits
// for a whole batch to drain before issuing the next.
// Client-table access from registers: lane j of every wave holds client j's pointer,
// n, N and r (K <= 64 = wave size), and a client step reads them with v_readlane
// (uniform index -> SGPR) instead of a scalar-memory load + lgkmcnt wait.
template <class CP>
struct LaneTable {
    uint64_t p;
    typename CP::S n, N;
    double r;
    __device__ __forceinline__ explicit LaneTable(const ClientTable<typename CP::S>& tab) {
        const int lane = threadIdx.x & 63;
        p = reinterpret_cast<uint64_t>(tab.ptr[lane]);
        n = tab.n[lane];
        N = tab.N[lane];
        r = tab.r[lane];
    }
    template <typename T>
    __device__ __forceinline__ static T rl(T v, int k) {
        static_assert(sizeof(T) == 4 || sizeof(T) == 8, "readlane of 4/8-byte values");
        if constexpr (sizeof(T) == 4) {
            int i;
            __builtin_memcpy(&i, &v, 4);
            i = __builtin_amdgcn_readlane(i, k);
            __builtin_memcpy(&v, &i, 4);
            return v;
        } else {
            int i[2];
            __builtin_memcpy(i, &v, 8);
            i[0] = __builtin_amdgcn_readlane(i[0], k);
            i[1] = __builtin_amdgcn_readlane(i[1], k);
            __builtin_memcpy(&v, i, 8);
            return v;
        }
    }
};

// Chip-wide store windows (probe kernels: fa_tune OPT_WIN_* / AVG_WIN_*). Every wave reads the GPU's
// 100 MHz reference clock (s_memrealtime: one counter for all XCDs) and stores only while
// clock mod period < win_w, reads (optionally) only outside that window: the DRAM then sees
// read-only stretches and write bursts instead of writes interleaved everywhere, with no grid
// barrier. A wait gives up after 2^18 polls, far past one period, should the clock stand still.
// (the clock's low 32 bits: one irregular period every 43 s where they wrap; the remainder by a
// power-of-two period is a mask, otherwise a multiply-high by floor(2^32 / period) and one correction)
[[maybe_unused]] __device__ __forceinline__ bool in_write_window(uint32_t period, uint32_t win_w) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
    uint32_t r;
    if ((period & (period - 1)) == 0) {
        r = t & (period - 1);
    } else {
        const uint32_t recip = 0xFFFFFFFFu / period;   // uniform: the compiler keeps it out of the poll loop
        r = t - __umulhi(t, recip) * period;
        if (r >= period) r -= period;
    }
    return r < win_w;
}
// (a wait gives up after 2^18 polls, far past one period, should the clock ever stand still)
[[maybe_unused]] __device__ __forceinline__ void wait_write_window(uint32_t period, uint32_t win_w) {
    for (int n = 0; n < (1 << 18) && !in_write_window(period, win_w); ++n) __builtin_amdgcn_s_sleep(1);
}
[[maybe_unused]] __device__ __forceinline__ void wait_read_window(uint32_t period, uint32_t win_w) {
    for (int n = 0; n < (1 << 18) && in_write_window(period, win_w); ++n) __builtin_amdgcn_s_sleep(1);
}


// Workgroup -> tile order for the one-tile-per-workgroup grid (fa_tune FA_TUNE_TILEMAP).
// Workgroups are dealt round-robin to the 8 XCDs, so with MAP 0 consecutive tiles run on
// different XCDs. MAP = R > 0 gives each XCD runs of R consecutive tiles (groups of 8R tiles,
// XCD x taking tiles [xR, xR + R) of each group): a bijection on the first whole groups and
// the identity on the rest. (One contiguous eighth of the model per XCD measured 0.5-4 %
// slower than identity: profiles/r01_tilemap.log.)
template <int MAP>
__device__ __forceinline__ int64_t map_tile(int64_t t, int64_t ntiles) {
    if constexpr (MAP > 0) {
        const int64_t g = ntiles / (8 * MAP);
        if (t < 8 * MAP * g) {
            const int64_t j = t / 8;
            t = (j / MAP) * (8 * MAP) + (t % 8) * MAP + (j % MAP);
        }
    }
    return t;
}

template <typename Y, typename X, class CP, int E, int S, bool INIT, bool INT_FIRST, bool NT, bool LT, int BLK, int NTS,
          int MAP, bool WIN = false>
__device__ __forceinline__ void fedavg_pipe_body(X* __restrict__ agg, const ClientTable<typename CP::S>& tab, const int K,
                                                 const int64_t P, const uint32_t period = 0, const uint32_t win_w = 0,
                                                 const int win_mode = 0) {
    using V = typename CP::V;
    const LaneTable<CP> lt(tab);
    const int64_t ntiles = ((P + E - 1) / E + (int64_t)BLK * S - 1) / ((int64_t)BLK * S);
    // one tile per block (gridDim == ntiles), or a persistent grid sweeping tiles in grid
    // order so the tiles read concurrently from one client buffer are adjacent
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t tile = map_tile<MAP>(t, ntiles);
        const int64_t strip0 = tile * (BLK * S) + threadIdx.x;
        if ((strip0 + (int64_t)(S - 1) * BLK) * E + E > P) {
            k_fedavg_tail<Y, X, CP, E, S, INIT, INT_FIRST, BLK>(agg, tab, K, P, strip0);
            continue;
        }
        if constexpr (WIN) {
            if (win_mode >= 1) wait_read_window(period, win_w);
        }
        V x[S][E];
        int k = 0;
#pragma unroll
        for (int s = 0; s < S; ++s)
            k = strip_start<Y, X, CP, E, INIT, INT_FIRST, NT>(x[s], agg, tab, (strip0 + s * BLK) * E, E);
        auto load = [&](int kk, Y (&y)[S][E]) {
            const Y* yp = LT ? reinterpret_cast<const Y*>(LaneTable<CP>::rl(lt.p, kk)) : static_cast<const Y*>(tab.ptr[kk]);
#pragma unroll
            for (int s = 0; s < S; ++s) strip_load<Y, E, NT>(yp + (strip0 + s * BLK) * E, y[s]);
        };
        auto fold = [&](int kk, const Y (&y)[S][E]) {
            const typename CP::S n = LT ? LaneTable<CP>::rl(lt.n, kk) : tab.n[kk];
            const typename CP::S N = LT ? LaneTable<CP>::rl(lt.N, kk) : tab.N[kk];
            const double r = LT ? LaneTable<CP>::rl(lt.r, kk) : tab.r[kk];
#pragma unroll
            for (int s = 0; s < S; ++s) {
                V yv[E];
#pragma unroll
                for (int e = 0; e < E; ++e) yv[e] = widen<Y, V>(y[s][e]);
                fold_strip<CP, E>(x[s], yv, n, N, r);
            }
        };
        Y a[S][E], b[S][E];
        if (k < K) load(k, a);
        while (k + 1 < K) {
            if constexpr (WIN) {
                if (win_mode >= 2) wait_read_window(period, win_w);
            }
            load(k + 1, b);
            fold(k, a);
            if (k + 2 < K) load(k + 2, a);
            fold(k + 1, b);
            k += 2;
        }
        if (k < K) fold(k, a);
        if constexpr (WIN) wait_write_window(period, win_w);
#pragma unroll
        for (int s = 0; s < S; ++s) {
            X xo[E];
#pragma unroll
            for (int e = 0; e < E; ++e) xo[e] = narrow<X, V>(x[s][e]);
            if constexpr (is_nostore<CP>::value) {
                if (__float_as_uint(x[s][0]) != 0xFFFFFFFFu) continue;   // keeps loads + adds live
            }
            strip_store<X, E, NTS>(agg + (strip0 + s * BLK) * E, xo);
        }
    }
}

template <typename Y, typename X, class CP, int E, int S, bool INIT, bool INT_FIRST, bool NT, bool LT, int BLK = kBlock,
          int NTS = 0, int MAP = 0>
__global__ void __launch_bounds__(BLK)
k_fedavg_pipe(X* __restrict__ agg, const ClientTable<typename CP::S> tab, const int K, const int64_t P) {
    fedavg_pipe_body<Y, X, CP, E, S, INIT, INT_FIRST, NT, LT, BLK, NTS, MAP>(agg, tab, K, P);
}

// The same fold with every wave's stores inside a chip-wide window of the GPU's 100 MHz clock
// (avg_store_window): bit-identical, the stores bunched into common bursts.
template <typename Y, typename X, class CP, int E, int S, bool INIT, bool INT_FIRST, bool NT, bool LT, int BLK, int NTS,
          int MAP>
__global__ void __launch_bounds__(BLK)
k_fedavg_pipe_win(X* __restrict__ agg, const ClientTable<typename CP::S> tab, const int K, const int64_t P,
                  const uint32_t period, const uint32_t win_w, const int win_mode) {
    fedavg_pipe_body<Y, X, CP, E, S, INIT, INT_FIRST, NT, LT, BLK, NTS, MAP, true>(agg, tab, K, P, period, win_w, win_mode);
}

#ifdef FEDAGG_PROBES
// occupancy probe (FA_TUNE_WPE): the same body compiled for at least W waves per SIMD
template <typename Y, typename X, class CP, int E, int S, bool INIT, bool INT_FIRST, bool NT, bool LT, int BLK, int NTS,
          int MAP, int W>
__global__ void __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(W)))
k_fedavg_pipe_w(X* __restrict__ agg, const ClientTable<typename CP::S> tab, const int K, const int64_t P) {
    fedavg_pipe_body<Y, X, CP, E, S, INIT, INT_FIRST, NT, LT, BLK, NTS, MAP>(agg, tab, K, P);
}
#endif

// ----------------------------------------------------------------------------
// FedOpt kernel: pseudo-gradient fold + server step, fused
// ----------------------------------------------------------------------------
struct OptScalars {
    // python-float constants exactly as fedopt.py computes them
    double lr, b1, b2, tau, tau2, c1, c2, nc2;   // c1 = 1-b1, c2 = 1-b2, nc2 = -(1-b2)
    float b1f, c1f, c2f;                         // the same cast to f32 (numpy weak-scalar rule)
    float b1h, c1h, c2h;                         // ... and to f16 (held in f32): float16 state / pg
    int opt;
};

struct OptBuffers {
    const void* old;
    void* pg;
    const void* m_in;
    void* m_out;
    const void* v_in;
    void* v_out;
    void* out;
    int m_in_f64;    // 0: f32, 1: f64, -1: None
    int m_out_f64;
    // storage dtype of v and the new model (fa_fedopt_step_ex): 0 = f64 (the reference's), 1 = f32
    // (the fp32-state mode: same f64 arithmetic, rounded once to f32 on store, widened exactly on load)
    int v_in_f32;
    int v_out_f32;
    int out_f32;
};

// multiply an array element held as PG by a python float constant (numpy weak scalar)
template <class PG> __device__ __forceinline__ double mul_pg(double a, double c, float cf, float ch);
template <> __device__ __forceinline__ double mul_pg<CF32>(double a, double, float cf, float) { return (double)((float)a * cf); }
template <> __device__ __forceinline__ double mul_pg<CF64>(double a, double c, float, float) { return a * c; }
template <> __device__ __forceinline__ double mul_pg<CF16>(double a, double, float, float ch) {
    return (double)CF16::rh((float)a * ch);
}

// numpyhelper.subtract(next, old) = next*1.0 + old*(-1.0) (numpyhelper.py:44-56) and power(pg, 2)
// (:94-104) in the pseudo-gradient's dtype: float16 rounds every op to half, as numpy's half loops
template <class PG> __device__ __forceinline__ typename PG::V pg_sub(typename PG::V y, typename PG::V o) { return y - o; }
template <> __device__ __forceinline__ float pg_sub<CF16>(float y, float o) { return CF16::rh(y - o); }
template <class PG> __device__ __forceinline__ typename PG::V pg_sq(typename PG::V v) { return (typename PG::V)(v * v); }
template <> __device__ __forceinline__ float pg_sq<CF16>(float v) { return CF16::rh(v * v); }

__device__ __forceinline__ double np_sign(double d) {
    // numpy sign: 1 / -1 / 0 (for +-0), NaN propagates
    return d > 0.0 ? 1.0 : (d < 0.0 ? -1.0 : (d == 0.0 ? 0.0 : d));
}

// The server state of one strip: m_in (as exact f64 values; f32 state is widened exactly) and
// v_in (or tau**2 when v is None, fedopt.py:170-171). rem < E: ragged strip.
template <int E, bool SNT = false>
__device__ __forceinline__ void opt_load_state(const OptBuffers& b, const OptScalars& s, int64_t i0, int rem,
                                               double (&mi)[E], double (&v)[E]) {
    const bool full = rem == E;
    if (b.m_in_f64 == 0) {
        float mf[E];
        const float* mp = static_cast<const float*>(b.m_in) + i0;
        if (full) strip_load<float, E, SNT>(mp, mf);
        else
            for (int e = 0; e < E; ++e) mf[e] = e < rem ? mp[e] : 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) mi[e] = (double)mf[e];
    } else if (b.m_in_f64 == 1) {
        const double* mp = static_cast<const double*>(b.m_in) + i0;
        if (full) strip_load<double, E, SNT>(mp, mi);
        else
            for (int e = 0; e < E; ++e) mi[e] = e < rem ? mp[e] : 0.0;
    } else if (b.m_in_f64 == 2) {                // float16 m (a float16 session's first rounds)
        f16 mh[E];
        const f16* mp = static_cast<const f16*>(b.m_in) + i0;
        if (full) strip_load<f16, E, SNT>(mp, mh);
        else
            for (int e = 0; e < E; ++e) mh[e] = e < rem ? mp[e] : f16{0};
#pragma unroll
        for (int e = 0; e < E; ++e) mi[e] = (double)f16_to_f32(mh[e].bits);
    }
    if (b.v_in && b.v_in_f32) {
        float vf[E];
        const float* vp = static_cast<const float*>(b.v_in) + i0;
        if (full) strip_load<float, E, SNT>(vp, vf);
        else
            for (int e = 0; e < E; ++e) vf[e] = e < rem ? vp[e] : 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = (double)vf[e];
    } else if (b.v_in) {
        const double* vp = static_cast<const double*>(b.v_in) + i0;
        if (full) strip_load<double, E, SNT>(vp, v);
        else
            for (int e = 0; e < E; ++e) v[e] = e < rem ? vp[e] : 0.0;
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = s.tau2;
    }
}

// The server step for one strip of E elements (fedopt.py:151-258), from the folded
// pseudo-gradient pg, the widened old model ov (OLD -> V is exact or the same conversion
// numpy's `old * 1.0` makes, so (double)ov == old as numpy sees it) and the state loaded by
// opt_load_state (mi, v; v is updated in place). rem < E: ragged strip.
template <class PG, int E, bool NOST = false, int OSM = 0>
__device__ __forceinline__ void opt_apply(const OptBuffers& b, const OptScalars& s, const typename PG::V (&pg)[E],
                                          const typename PG::V (&ov)[E], const double (&mi)[E], double (&v)[E],
                                          int64_t i0, int rem) {
    using V = typename PG::V;
    constexpr bool PG32 = std::is_same<PG, CF32>::value;
    const bool full = rem == E;
    // ---- m (fedopt.py:173-176 and the two twins)
    constexpr bool PG64 = std::is_same<PG, CF64>::value;
    double m[E];
    if (b.m_in_f64 < 0) {
#pragma unroll
        for (int e = 0; e < E; ++e) m[e] = mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
    } else {
        // m*beta1 in m's dtype, pg*(1-beta1) in pg's dtype, their sum in the promoted dtype
        // (f16 < f32 < f64); each operand is exact in its dtype, so the float sum rounds once
        if (b.m_in_f64 == 1) {                     // f64 m: an f64 sum
#pragma unroll
            for (int e = 0; e < E; ++e) m[e] = mi[e] * s.b1 + mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
        } else if (b.m_in_f64 == 0) {              // f32 m (mi is an exact f32)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float a = (float)mi[e] * s.b1f;
                const double pm = mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
                if constexpr (PG64) m[e] = (double)a + pm;          // f32 + f64
                else m[e] = (double)(a + (float)pm);                // f32 + f32 (or f16) in f32
            }
        } else {                                   // f16 m (a float16 session's first rounds)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float a = CF16::rh((float)mi[e] * s.b1h);
                const double pm = mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
                if constexpr (PG64) m[e] = (double)a + pm;
                else if constexpr (PG32) m[e] = (double)(a + (float)pm);
                else m[e] = (double)CF16::rh(a + (float)pm);
            }
        }
    }
    // ---- v (fedopt.py:178-179 / 214-217 / 251-252)
    double o[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const V pv = pg[e];
        const double p = (double)pg_sq<PG>(pv);   // power(pg, 2) in the pg dtype
        if (s.opt == FA_ADAM) {
            v[e] = v[e] * s.b2 + mul_pg<PG>(p, s.c2, s.c2f, s.c2h);
        } else if (s.opt == FA_YOGI) {
            const double sg = np_sign(v[e] - p);
            v[e] = v[e] + (sg * p) * s.nc2;
        } else {
            v[e] = v[e] + p;
        }
        const double sv = __builtin_sqrt(v[e]) + s.tau;
        const double t = m[e] / sv;
        o[e] = (double)ov[e] + t * s.lr;
    }
    // ---- stores
    if constexpr (NOST) {   // probe build: stores skipped behind a never-true data test (reads + math live)
        if (__double_as_longlong(o[0]) != 0x7FF4DEADBEEF0001LL) return;
    }
    if (full) {
        if (b.v_out_f32) {
            float vf[E];
#pragma unroll
            for (int e = 0; e < E; ++e) vf[e] = (float)v[e];
            strip_store<float, E, OSM>(static_cast<float*>(b.v_out) + i0, vf);
        } else {
            strip_store<double, E, OSM>(static_cast<double*>(b.v_out) + i0, v);
        }
        if (b.out_f32) {
            float of[E];
#pragma unroll
            for (int e = 0; e < E; ++e) of[e] = (float)o[e];
            strip_store<float, E, OSM>(static_cast<float*>(b.out) + i0, of);
        } else {
            strip_store<double, E, OSM>(static_cast<double*>(b.out) + i0, o);
        }
        if (b.m_out_f64 == 1) strip_store<double, E, OSM>(static_cast<double*>(b.m_out) + i0, m);
        else if (b.m_out_f64 == 0) {
            float mf[E];
#pragma unroll
            for (int e = 0; e < E; ++e) mf[e] = (float)m[e];
            strip_store<float, E, OSM>(static_cast<float*>(b.m_out) + i0, mf);
        } else {                                  // f16 m: every value is already a half
            f16 mh[E];
#pragma unroll
            for (int e = 0; e < E; ++e) mh[e] = f16{f32_to_f16((float)m[e])};
            strip_store<f16, E, 0>(static_cast<f16*>(b.m_out) + i0, mh);
        }
    } else {
        for (int e = 0; e < rem; ++e) {
            if (b.v_out_f32) static_cast<float*>(b.v_out)[i0 + e] = (float)v[e];
            else static_cast<double*>(b.v_out)[i0 + e] = v[e];
            if (b.out_f32) static_cast<float*>(b.out)[i0 + e] = (float)o[e];
            else static_cast<double*>(b.out)[i0 + e] = o[e];
            if (b.m_out_f64 == 1) static_cast<double*>(b.m_out)[i0 + e] = m[e];
            else if (b.m_out_f64 == 0) static_cast<float*>(b.m_out)[i0 + e] = (float)m[e];
            else static_cast<f16*>(b.m_out)[i0 + e] = f16{f32_to_f16((float)m[e])};
        }
    }
}

template <class PG, int E, bool NOST = false, int OSM = 0>
__device__ __forceinline__ void opt_final(const OptBuffers& b, const OptScalars& s, const typename PG::V (&pg)[E],
                                          const typename PG::V (&ov)[E], int64_t i0, int rem) {
    double mi[E], v[E];
    opt_load_state<E>(b, s, i0, rem, mi, v);
    opt_apply<PG, E, NOST, OSM>(b, s, pg, ov, mi, v, i0, rem);
}

// One lane's strip of E elements at i0 < P, clients batched kUnroll/2 at a time. (A
// k_fedavg_pipe-style traversal — 2 or 4 strips per lane, next client in flight — measured
// within noise of this one on configs[3]: profiles/r01_fedopt_ab.log)
template <typename Y, typename OLD, class PG, int E, bool FIRST, bool FINAL, bool NT, bool NOST = false, int OSM = 0>
__device__ __forceinline__ void fedopt_strip(const OptBuffers& b, const OptScalars& s,
                                             const ClientTable<typename PG::S>& tab, const int K, const int64_t P,
                                             const int64_t i0) {
    using V = typename PG::V;   // float or double
    const int rem = (P - i0) < E ? (int)(P - i0) : E;
    const bool full = rem == E;

    OLD old[E];
    const OLD* oldp = static_cast<const OLD*>(b.old) + i0;
    if (full) strip_load<OLD, E, false>(oldp, old);
    else {
#pragma unroll
        for (int e = 0; e < E; ++e) old[e] = e < rem ? oldp[e] : OLD{};
    }
    V ov[E];
#pragma unroll
    for (int e = 0; e < E; ++e) ov[e] = widen<OLD, V>(old[e]);

    // ---- pseudo-gradient: pg = y0 - old ; pg = pg + (n*((y_k - old) - pg))/N (fedopt.py:89-94)
    V pg[E];
    int k = 0;
    if constexpr (FIRST) {
        Y y[E];
        const Y* yp = static_cast<const Y*>(tab.ptr[0]) + i0;
        if (full) strip_load<Y, E, NT>(yp, y);
        else {
#pragma unroll
            for (int e = 0; e < E; ++e) y[e] = e < rem ? yp[e] : Y{};
        }
#pragma unroll
        for (int e = 0; e < E; ++e) pg[e] = pg_sub<PG>(widen<Y, V>(y[e]), ov[e]);
        k = 1;
    } else {
        using T = typename PG::T;                 // the workspace holds pg in its own dtype
        const T* pgp = static_cast<const T*>(b.pg) + i0;
        if (full) {
            T t[E];
            strip_load<T, E, false>(pgp, t);
#pragma unroll
            for (int e = 0; e < E; ++e) pg[e] = widen<T, V>(t[e]);
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e) pg[e] = e < rem ? widen<T, V>(pgp[e]) : V{};
        }
    }
    if (full) {
        for (; k + kUnroll / 2 <= K; k += kUnroll / 2) {
            Y y[kUnroll / 2][E];
#pragma unroll
            for (int u = 0; u < kUnroll / 2; ++u)
                strip_load<Y, E, NT>(static_cast<const Y*>(tab.ptr[k + u]) + i0, y[u]);
#pragma unroll
            for (int u = 0; u < kUnroll / 2; ++u) {
                const typename PG::S n = tab.n[k + u], N = tab.N[k + u];
                const double r = tab.r[k + u];
                V d[E];
#pragma unroll
                for (int e = 0; e < E; ++e) d[e] = pg_sub<PG>(widen<Y, V>(y[u][e]), ov[e]);   // subtract(next, old)
                fold_strip<PG, E>(pg, d, n, N, r);
            }
        }
    }
    for (; k < K; ++k) {
        const Y* yp = static_cast<const Y*>(tab.ptr[k]) + i0;
        const typename PG::S n = tab.n[k], N = tab.N[k];
        const double r = tab.r[k];
#pragma unroll
        for (int e = 0; e < E; ++e)
            if (e < rem) pg[e] = PG::fold(pg[e], pg_sub<PG>(widen<Y, V>(yp[e]), ov[e]), n, N, r);
    }

    if constexpr (!FINAL) {
        using T = typename PG::T;
        T* pgp = static_cast<T*>(b.pg) + i0;
        T t[E];
#pragma unroll
        for (int e = 0; e < E; ++e) t[e] = narrow<T, V>(pg[e]);
        if (full) strip_store<T, E>(pgp, t);
        else
            for (int e = 0; e < rem; ++e) pgp[e] = t[e];
        return;
    } else {
        opt_final<PG, E, NOST, OSM>(b, s, pg, ov, i0, rem);
    }
}

// The same lane work with a wave-coalesced element map: lane L of a wave tile of 128*NH elements
// owns the pairs {2L, 2L+1} + 128 j, j < NH, so every 8-byte stream (old, m, v, pg, out) moves one
// contiguous 1 KiB per wave instruction (full 128-B lines, no half-line stores) and the client loads
// are contiguous 512-B dwordx2 wave instructions. Whole wave tiles only.
// H (probe builds only, FA_TUNE_OPT_QUAD): elements per lane per strip — 2 (the product: pairs) or 4
// (quads at lane stride 4: 2-byte client loads become dwordx2, 8-byte streams two dwordx4 per strip).
template <typename Y, typename OLD, class PG, bool FIRST, bool FINAL, bool NT, int OSM = 0, int NH = 2,
          int U = kUnroll / 2, bool WIN = false, int H = 2>
__device__ __forceinline__ void fedopt_strip_split(const OptBuffers& b, const OptScalars& s,
                                                   const ClientTable<typename PG::S>& tab, const int K,
                                                   const int64_t i0, const uint32_t period = 0,
                                                   const uint32_t win_w = 0) {
    using V = typename PG::V;
    constexpr int E = H * NH;
    auto half = [](auto& a, int h) -> auto& {
        using T = std::remove_reference_t<decltype(a[0])>;
        return *reinterpret_cast<T(*)[H]>(&a[h * H]);
    };
    auto at = [i0](int h) { return i0 + (int64_t)h * 64 * H; };
    OLD old[E];
#pragma unroll
    for (int h = 0; h < NH; ++h) strip_load<OLD, H, false>(static_cast<const OLD*>(b.old) + at(h), half(old, h));
    V ov[E];
#pragma unroll
    for (int e = 0; e < E; ++e) ov[e] = widen<OLD, V>(old[e]);
    V pg[E];
    int k = 0;
    if constexpr (FIRST) {
        Y y[E];
        const Y* yp = static_cast<const Y*>(tab.ptr[0]);
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), half(y, h));
#pragma unroll
        for (int e = 0; e < E; ++e) pg[e] = pg_sub<PG>(widen<Y, V>(y[e]), ov[e]);
        k = 1;
    } else {
        using T = typename PG::T;                 // the workspace holds pg in its own dtype
        T t[E];
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<T, H, false>(static_cast<const T*>(b.pg) + at(h), half(t, h));
#pragma unroll
        for (int e = 0; e < E; ++e) pg[e] = widen<T, V>(t[e]);
    }
    for (; k + U <= K; k += U) {
        Y y[U][E];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const Y* yp = static_cast<const Y*>(tab.ptr[k + u]);
#pragma unroll
            for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), half(y[u], h));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            V d[E];
#pragma unroll
            for (int e = 0; e < E; ++e) d[e] = pg_sub<PG>(widen<Y, V>(y[u][e]), ov[e]);
            fold_strip<PG, E>(pg, d, tab.n[k + u], tab.N[k + u], tab.r[k + u]);
        }
    }
    for (; k < K; ++k) {
        const Y* yp = static_cast<const Y*>(tab.ptr[k]);
        Y y[E];
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), half(y, h));
        V d[E];
#pragma unroll
        for (int e = 0; e < E; ++e) d[e] = pg_sub<PG>(widen<Y, V>(y[e]), ov[e]);
        fold_strip<PG, E>(pg, d, tab.n[k], tab.N[k], tab.r[k]);
    }
    if constexpr (!FINAL) {
        using T = typename PG::T;
        T t[E];
#pragma unroll
        for (int e = 0; e < E; ++e) t[e] = narrow<T, V>(pg[e]);
        if constexpr (WIN) wait_write_window(period, win_w);
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_store<T, H>(static_cast<T*>(b.pg) + at(h), half(t, h));
    } else {
        double mi[E], vv[E];
#pragma unroll
        for (int h = 0; h < NH; ++h) opt_load_state<H>(b, s, at(h), H, half(mi, h), half(vv, h));
        if constexpr (WIN) wait_write_window(period, win_w);   // the state loads land meanwhile
#pragma unroll
        for (int h = 0; h < NH; ++h)
            opt_apply<PG, H, false, OSM>(b, s, half(pg, h), half(ov, h), half(mi, h), half(vv, h), at(h), H);
    }
}

template <typename Y, typename OLD, class PG, bool FIRST, bool FINAL, bool NT, int OSM, int NH, int U, bool MV = false,
          bool WIN = false>
__device__ __forceinline__ void fedopt_c_body(const OptBuffers& b, const OptScalars& s, const ClientTable<typename PG::S>& tab,
                                              const int K, const int64_t P, const uint32_t period = 0,
                                              const uint32_t win_w = 0) {
    constexpr int64_t T = 128 * NH;                                     // elements per wave tile
    const int64_t base = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * T;
    const int lane = threadIdx.x & 63;
    if constexpr (MV) {
        // layout probe (FA_TUNE_OPT_MV): fp64 m and v interleaved per wave tile in one buffer
        // ([m of tile w | v of tile w] at 2wT), read from m_in and written to m_out; whole tiles only
        if (base + T > P) return;
        OptBuffers bb = b;
        bb.m_in = static_cast<const double*>(b.m_in) + base;
        bb.v_in = static_cast<const double*>(b.m_in) + base + T;
        bb.m_out = static_cast<double*>(b.m_out) + base;
        bb.v_out = static_cast<double*>(b.m_out) + base + T;
        fedopt_strip_split<Y, OLD, PG, FIRST, FINAL, NT, OSM, NH, U>(bb, s, tab, K, base + 2 * lane);
        return;
    }
    if (base + T <= P) {
        fedopt_strip_split<Y, OLD, PG, FIRST, FINAL, NT, OSM, NH, U, WIN>(b, s, tab, K, base + 2 * lane, period, win_w);
    } else {                                      // the ragged last tile: the per-lane strip map
#pragma unroll
        for (int j = 0; j < NH / 2; ++j) {
            const int64_t i0 = base + j * 256 + 4 * lane;
            if (i0 < P) fedopt_strip<Y, OLD, PG, 4, FIRST, FINAL, NT, false, OSM>(b, s, tab, K, P, i0);
        }
    }
}

#ifdef FEDAGG_PROBES
// burst-store probe of the product step (FA_TUNE_OPT_G = G): k_fedopt_c's FINAL phase
// with every wave taking G consecutive 512-element tiles and storing the new v / out / m of all G
// after the last tile's reads (k_fedopt_mixg measured the access pattern alone). The arithmetic is
// opt_apply's, duplicated here (opt_compute_p) so that the product kernels' code stays as measured.
template <class PG, int E>
__device__ __forceinline__ void opt_compute_p(const OptBuffers& b, const OptScalars& s, const typename PG::V (&pg)[E],
                                              const typename PG::V (&ov)[E], const double (&mi)[E], double (&v)[E],
                                              double (&m)[E], double (&o)[E]) {
    using V = typename PG::V;
    constexpr bool PG32 = std::is_same<PG, CF32>::value;
    // ---- m (fedopt.py:173-176 and the two twins)
    constexpr bool PG64 = std::is_same<PG, CF64>::value;
    if (b.m_in_f64 < 0) {
#pragma unroll
        for (int e = 0; e < E; ++e) m[e] = mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
    } else {
        // m*beta1 in m's dtype, pg*(1-beta1) in pg's dtype, their sum in the promoted dtype
        // (f16 < f32 < f64); each operand is exact in its dtype, so the float sum rounds once
        if (b.m_in_f64 == 1) {                     // f64 m: an f64 sum
#pragma unroll
            for (int e = 0; e < E; ++e) m[e] = mi[e] * s.b1 + mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
        } else if (b.m_in_f64 == 0) {              // f32 m (mi is an exact f32)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float a = (float)mi[e] * s.b1f;
                const double pm = mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
                if constexpr (PG64) m[e] = (double)a + pm;          // f32 + f64
                else m[e] = (double)(a + (float)pm);                // f32 + f32 (or f16) in f32
            }
        } else {                                   // f16 m (a float16 session's first rounds)
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const float a = CF16::rh((float)mi[e] * s.b1h);
                const double pm = mul_pg<PG>((double)pg[e], s.c1, s.c1f, s.c1h);
                if constexpr (PG64) m[e] = (double)a + pm;
                else if constexpr (PG32) m[e] = (double)(a + (float)pm);
                else m[e] = (double)CF16::rh(a + (float)pm);
            }
        }
    }
    // ---- v (fedopt.py:178-179 / 214-217 / 251-252)
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const V pv = pg[e];
        const double p = (double)pg_sq<PG>(pv);   // power(pg, 2) in the pg dtype
        if (s.opt == FA_ADAM) {
            v[e] = v[e] * s.b2 + mul_pg<PG>(p, s.c2, s.c2f, s.c2h);
        } else if (s.opt == FA_YOGI) {
            const double sg = np_sign(v[e] - p);
            v[e] = v[e] + (sg * p) * s.nc2;
        } else {
            v[e] = v[e] + p;
        }
        const double sv = __builtin_sqrt(v[e]) + s.tau;
        const double t = m[e] / sv;
        o[e] = (double)ov[e] + t * s.lr;
    }
}

template <typename Y, typename OLD, class PG, bool FIRST, bool NT, int G, bool WIN = false>
__device__ __forceinline__ void fedopt_cg_body(const OptBuffers& b, const OptScalars& s, const ClientTable<typename PG::S>& tab,
                                               const int K, const int64_t P, const uint32_t period = 0,
                                               const uint32_t win_w = 0) {
    using V = typename PG::V;
    constexpr int NH = 4, H = 2, E = H * NH, U = kUnroll / 2;
    constexpr int64_t T = 128 * NH;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if ((wave + 1) * G * T > P) {                 // a partial group: the product kernel's per-tile path
        for (int g = 0; g < G; ++g) {
            const int64_t base = (wave * G + g) * T;
            if (base >= P) break;
            if (base + T <= P) fedopt_strip_split<Y, OLD, PG, FIRST, true, NT, 1, NH, U>(b, s, tab, K, base + 2 * lane);
            else
                for (int j = 0; j < NH / 2; ++j) {
                    const int64_t i0 = base + j * 256 + 4 * lane;
                    if (i0 < P) fedopt_strip<Y, OLD, PG, 4, FIRST, true, NT, false, 1>(b, s, tab, K, P, i0);
                }
        }
        return;
    }
    double mo[G][E], vo[G][E], oo[G][E];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t i0 = (wave * G + g) * T + 2 * lane;
        auto half = [](auto& a, int h) -> auto& {
            using TT = std::remove_reference_t<decltype(a[0])>;
            return *reinterpret_cast<TT(*)[H]>(&a[h * H]);
        };
        auto at = [i0](int h) { return i0 + (int64_t)h * 128; };
        OLD old[E];
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<OLD, H, false>(static_cast<const OLD*>(b.old) + at(h), half(old, h));
        V ov[E];
#pragma unroll
        for (int e = 0; e < E; ++e) ov[e] = widen<OLD, V>(old[e]);
        V pg[E];
        int k = 0;
        if constexpr (FIRST) {
            Y y[E];
            const Y* yp = static_cast<const Y*>(tab.ptr[0]);
#pragma unroll
            for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), half(y, h));
#pragma unroll
            for (int e = 0; e < E; ++e) pg[e] = pg_sub<PG>(widen<Y, V>(y[e]), ov[e]);
            k = 1;
        } else {
            using TT = typename PG::T;
            TT t[E];
#pragma unroll
            for (int h = 0; h < NH; ++h) strip_load<TT, H, false>(static_cast<const TT*>(b.pg) + at(h), half(t, h));
#pragma unroll
            for (int e = 0; e < E; ++e) pg[e] = widen<TT, V>(t[e]);
        }
        for (; k + U <= K; k += U) {
            Y y[U][E];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const Y* yp = static_cast<const Y*>(tab.ptr[k + u]);
#pragma unroll
                for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), half(y[u], h));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                V d[E];
#pragma unroll
                for (int e = 0; e < E; ++e) d[e] = pg_sub<PG>(widen<Y, V>(y[u][e]), ov[e]);
                fold_strip<PG, E>(pg, d, tab.n[k + u], tab.N[k + u], tab.r[k + u]);
            }
        }
        for (; k < K; ++k) {
            const Y* yp = static_cast<const Y*>(tab.ptr[k]);
            Y y[E];
#pragma unroll
            for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), half(y, h));
            V d[E];
#pragma unroll
            for (int e = 0; e < E; ++e) d[e] = pg_sub<PG>(widen<Y, V>(y[e]), ov[e]);
            fold_strip<PG, E>(pg, d, tab.n[k], tab.N[k], tab.r[k]);
        }
        double mi[E];
#pragma unroll
        for (int h = 0; h < NH; ++h) opt_load_state<H>(b, s, at(h), H, half(mi, h), half(vo[g], h));
#pragma unroll
        for (int h = 0; h < NH; ++h)
            opt_compute_p<PG, H>(b, s, half(pg, h), half(ov, h), half(mi, h), half(vo[g], h), half(mo[g], h), half(oo[g], h));
    }
    if constexpr (WIN) wait_write_window(period, win_w);      // everything computed: only the stores wait
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t i0 = (wave * G + g) * T + 2 * lane;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const int64_t o = i0 + (int64_t)h * 128;
            double* vp = &vo[g][h * H];
            double* op = &oo[g][h * H];
            double* mp = &mo[g][h * H];
            // fp64 state and model (the steady state of configs[3]; other dtypes refused at launch)
            strip_store<double, H, 1>(static_cast<double*>(b.v_out) + o, *reinterpret_cast<double(*)[H]>(vp));
            strip_store<double, H, 1>(static_cast<double*>(b.out) + o, *reinterpret_cast<double(*)[H]>(op));
            strip_store<double, H, 1>(static_cast<double*>(b.m_out) + o, *reinterpret_cast<double(*)[H]>(mp));
        }
    }
}

template <typename Y, typename OLD, class PG, bool FIRST, bool NT, int G>
__global__ void __launch_bounds__(kBlock)
k_fedopt_cg(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P) {
    fedopt_cg_body<Y, OLD, PG, FIRST, NT, G>(b, s, tab, K, P);
}

// the windowed product step compiled for at least W waves per SIMD (FA_TUNE_WPE with a window): the
// waves idling for their window need other waves resident to keep the reads flowing
template <typename Y, typename OLD, class PG, bool NT, int W>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W)))
k_fedopt_cw_w(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P,
              const uint32_t period, const uint32_t win_w) {
    fedopt_c_body<Y, OLD, PG, true, true, NT, 1, 4, kUnroll / 2, false, true>(b, s, tab, K, P, period, win_w);
}

// the windowed step on 256-element wave tiles (2 pairs per lane; OPT_WIN_PROD = 3): fewer registers
// held per wave, so more waves resident to keep reading while others wait for their window
template <typename Y, typename OLD, class PG, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_cw2(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P,
             const uint32_t period, const uint32_t win_w) {
    fedopt_c_body<Y, OLD, PG, true, true, NT, 1, 2, kUnroll / 2, false, true>(b, s, tab, K, P, period, win_w);
}

// store-window probe on the compute-then-store order (OPT_WIN_PROD = 2): one tile per wave, its
// v / out / m computed first and stored inside the window (k_fedopt_cw waits before opt_apply, so
// its fp64 square roots and divisions run inside the window)
template <typename Y, typename OLD, class PG, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_cgw(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P,
             const uint32_t period, const uint32_t win_w) {
    fedopt_cg_body<Y, OLD, PG, true, NT, 1, true>(b, s, tab, K, P, period, win_w);
}
#endif

template <typename Y, typename OLD, class PG, bool FIRST, bool FINAL, bool NT, int OSM = 0, int NH = 2,
          int U = kUnroll / 2>
__global__ void __launch_bounds__(kBlock)
k_fedopt_c(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P) {
    fedopt_c_body<Y, OLD, PG, FIRST, FINAL, NT, OSM, NH, U>(b, s, tab, K, P);
}

// The same single-launch step (all K clients, FIRST | FINAL) with every wave's v / out / m stores
// issued inside a chip-wide window of the GPU's 100 MHz reference clock (clock mod period < win_w;
// opt_window() sizes both from the launch's bytes per round of resident waves). Reads continue
// throughout; the stores of all waves bunch into common bursts instead of interleaving with 36
// read streams everywhere — fewer DRAM read/write turnarounds (profiles/r05_fedopt_window.log).
// Arithmetic and element map are k_fedopt_c's: bit-identical results.
template <typename Y, typename OLD, class PG, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_cw(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P,
            const uint32_t period, const uint32_t win_w) {
    fedopt_c_body<Y, OLD, PG, true, true, NT, 1, 4, kUnroll / 2, false, true>(b, s, tab, K, P, period, win_w);
}

#ifdef FEDAGG_PROBES
// store-window probe on a wave of a multi-launch round (staging.FedOptPipeline: the first or a middle
// launch, pg written back to the workspace; fa_tune OPT_WIN_PERIOD > 0 with OPT_WIN_PROD = 1):
// k_fedopt_c's bits. Null for the product: 8 bf16 updates over fp64 pg, 250 M params, every period
// 400-2500 ticks slower than no window (first +7...+76 %, middle +1...+34 %;
// profiles/r05_wave_window.log) — the 20-25 % write share of the FedAvg bf16 K = 8 case.
template <typename Y, typename OLD, class PG, bool FIRST, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_cwp(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P,
             const uint32_t period, const uint32_t win_w) {
    fedopt_c_body<Y, OLD, PG, FIRST, false, NT, 1, 4, kUnroll / 2, false, true>(b, s, tab, K, P, period, win_w);
}
#endif

#ifdef FEDAGG_PROBES
// element-map probe (FA_TUNE_OPT_QUAD): k_fedopt_c's 512-element wave tiles with lane L owning the
// quads {4L .. 4L+3} + 256 j, j < 2, instead of the pairs {2L, 2L+1} + 128 j, j < 4. Same elements
// per lane, same arithmetic per element: bit-identical. 2-byte client loads widen from one dword to
// one dwordx2 per strip; the 8-byte streams (old, pg, m, v, out) take two dwordx4 per strip.
template <typename Y, typename OLD, class PG, bool FIRST, bool FINAL, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_cq(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P) {
    const int64_t base = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 512;
    const int lane = threadIdx.x & 63;
    if (base + 512 <= P) {
        fedopt_strip_split<Y, OLD, PG, FIRST, FINAL, NT, 1, 2, kUnroll / 2, false, 4>(b, s, tab, K, base + 4 * lane);
    } else {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t i0 = base + j * 256 + 4 * lane;
            if (i0 < P) fedopt_strip<Y, OLD, PG, 4, FIRST, FINAL, NT, false, 1>(b, s, tab, K, P, i0);
        }
    }
}

template <typename Y, typename OLD, class PG, bool FIRST, bool FINAL, bool NT, int OSM, int NH, int U, int W>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W)))
k_fedopt_c_w(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P) {
    fedopt_c_body<Y, OLD, PG, FIRST, FINAL, NT, OSM, NH, U>(b, s, tab, K, P);
}

template <typename Y, typename OLD, class PG, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_c_mv(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P) {
    fedopt_c_body<Y, OLD, PG, true, true, NT, 1, 4, kUnroll / 2, true>(b, s, tab, K, P);
}

// access-pattern probe (FA_TUNE_OPT_MIX): exactly k_fedopt_c's loads and stores for a FIRST|FINAL
// launch — the element map (4 pairs per lane), clients loaded 4 at a time then the K % 4 remainder,
// the state after the fold, non-temporal stores of v / out / m — with the arithmetic cut to one
// add per value: the ceiling of the kernel's HBM traffic pattern alone. Whole wave tiles only.
template <typename Y, typename OLD, typename S, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_mix(const OptBuffers b, const ClientTable<S> tab, const int K, const int64_t P) {
    constexpr int NH = 4, H = 2, E = 2 * NH, U = kUnroll / 2;
    constexpr int64_t T = 128 * NH;
    const int64_t base = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * T;
    if (base + T > P) return;
    const int64_t i0 = base + 2 * (threadIdx.x & 63);
    auto at = [i0](int h) { return i0 + (int64_t)h * 128; };
    double acc[E];
    {
        OLD old[E];
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<OLD, H, false>(static_cast<const OLD*>(b.old) + at(h), *reinterpret_cast<OLD(*)[H]>(&old[h * H]));
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = (double)widen<OLD, double>(old[e]);
    }
    auto add_client = [&](int k, Y (&y)[E]) {
        const Y* yp = static_cast<const Y*>(tab.ptr[k]);
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), *reinterpret_cast<Y(*)[H]>(&y[h * H]));
    };
    int k = 0;
    {
        Y y[E];
        add_client(0, y);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[e]);
        k = 1;
    }
    for (; k + U <= K; k += U) {
        Y y[U][E];
#pragma unroll
        for (int u = 0; u < U; ++u) add_client(k + u, y[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[u][e]);
    }
    for (; k < K; ++k) {
        Y y[E];
        add_client(k, y);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[e]);
    }
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        double mi[H] = {}, vv[H] = {};
        opt_load_state<H>(b, OptScalars{}, at(h), H, mi, vv);
        double m[H], v[H], o[H];
#pragma unroll
        for (int e = 0; e < H; ++e) {
            m[e] = mi[e] + acc[h * H + e];
            v[e] = vv[e] + acc[h * H + e];
            o[e] = acc[h * H + e];
        }
        strip_store<double, H, 1>(static_cast<double*>(b.v_out) + at(h), v);
        strip_store<double, H, 1>(static_cast<double*>(b.out) + at(h), o);
        if (b.m_out_f64) strip_store<double, H, 1>(static_cast<double*>(b.m_out) + at(h), m);
        else {
            float mf[H];
#pragma unroll
            for (int e = 0; e < H; ++e) mf[e] = (float)m[e];
            strip_store<float, H, 1>(static_cast<float*>(b.m_out) + at(h), mf);
        }
    }
}
#endif

#ifdef FEDAGG_PROBES
// burst-store probe (FA_TUNE_OPT_BURST = G): k_fedopt_mix's access pattern, but each
// wave takes G consecutive wave tiles and holds the new v / out / m of all G in registers (LDS
// staging of several tiles would leave one workgroup per CU), storing them together after the
// reads of the last one — the writes leave the wave in one burst of 3 x G KiB-lines per stream
// instead of interleaved with every tile's reads. Whole groups of G tiles only.
template <typename Y, typename OLD, typename S, bool NT, int G>
__global__ void __launch_bounds__(kBlock)
k_fedopt_mixg(const OptBuffers b, const ClientTable<S> tab, const int K, const int64_t P) {
    constexpr int NH = 4, H = 2, E = 2 * NH, U = kUnroll / 2;
    constexpr int64_t T = 128 * NH;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if ((wave + 1) * G * T > P) return;
    double vo[G][E], oo[G][E], mo[G][E];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t i0 = (wave * G + g) * T + 2 * (threadIdx.x & 63);
        auto at = [i0](int h) { return i0 + (int64_t)h * 128; };
        double acc[E];
        {
            OLD old[E];
#pragma unroll
            for (int h = 0; h < NH; ++h)
                strip_load<OLD, H, false>(static_cast<const OLD*>(b.old) + at(h), *reinterpret_cast<OLD(*)[H]>(&old[h * H]));
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] = (double)widen<OLD, double>(old[e]);
        }
        auto add_client = [&](int k, Y (&y)[E]) {
            const Y* yp = static_cast<const Y*>(tab.ptr[k]);
#pragma unroll
            for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), *reinterpret_cast<Y(*)[H]>(&y[h * H]));
        };
        int k = 0;
        for (; k + U <= K; k += U) {
            Y y[U][E];
#pragma unroll
            for (int u = 0; u < U; ++u) add_client(k + u, y[u]);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[u][e]);
        }
        for (; k < K; ++k) {
            Y y[E];
            add_client(k, y);
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[e]);
        }
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            double mi[H] = {}, vv[H] = {};
            opt_load_state<H>(b, OptScalars{}, at(h), H, mi, vv);
#pragma unroll
            for (int e = 0; e < H; ++e) {
                mo[g][h * H + e] = mi[e] + acc[h * H + e];
                vo[g][h * H + e] = vv[e] + acc[h * H + e];
                oo[g][h * H + e] = acc[h * H + e];
            }
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t i0 = (wave * G + g) * T + 2 * (threadIdx.x & 63);
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            const int64_t o = i0 + (int64_t)h * 128;
            strip_store<double, H, 1>(static_cast<double*>(b.v_out) + o, *reinterpret_cast<double(*)[H]>(&vo[g][h * H]));
            strip_store<double, H, 1>(static_cast<double*>(b.out) + o, *reinterpret_cast<double(*)[H]>(&oo[g][h * H]));
            strip_store<double, H, 1>(static_cast<double*>(b.m_out) + o, *reinterpret_cast<double(*)[H]>(&mo[g][h * H]));
        }
    }
}
#endif

#ifdef FEDAGG_PROBES
// clock-windowed store probe (FA_TUNE_OPT_WIN_*): k_fedopt_mix's access pattern with the whole chip's
// stores confined to a common time window. Every wave reads the GPU's 100 MHz reference clock
// (s_memrealtime, one counter for all XCDs) and issues its v / out / m stores only while
// clock mod period < win_w, and (mode >= 1) starts a tile's reads, or (mode 2) each client batch's
// reads, only outside that window — so the DRAM sees read-only stretches and write bursts instead of
// 36 streams with 14 % writes interleaved everywhere, without a grid barrier. Waits are bounded by
// one period; results are k_fedopt_mix's.
template <typename Y, typename OLD, typename S, bool NT>
__global__ void __launch_bounds__(kBlock)
k_fedopt_mixw(const OptBuffers b, const ClientTable<S> tab, const int K, const int64_t P, const uint32_t period,
              const uint32_t win_w, const int mode) {
    constexpr int NH = 4, H = 2, E = 2 * NH, U = kUnroll / 2;
    constexpr int64_t T = 128 * NH;
    const int64_t base = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * T;
    if (base + T > P) return;
    const int64_t i0 = base + 2 * (threadIdx.x & 63);
    auto at = [i0](int h) { return i0 + (int64_t)h * 128; };
    if (mode >= 1) wait_read_window(period, win_w);
    double acc[E];
    {
        OLD old[E];
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<OLD, H, false>(static_cast<const OLD*>(b.old) + at(h), *reinterpret_cast<OLD(*)[H]>(&old[h * H]));
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = (double)widen<OLD, double>(old[e]);
    }
    auto add_client = [&](int k, Y (&y)[E]) {
        const Y* yp = static_cast<const Y*>(tab.ptr[k]);
#pragma unroll
        for (int h = 0; h < NH; ++h) strip_load<Y, H, NT>(yp + at(h), *reinterpret_cast<Y(*)[H]>(&y[h * H]));
    };
    int k = 0;
    {
        Y y[E];
        add_client(0, y);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[e]);
        k = 1;
    }
    for (; k + U <= K; k += U) {
        if (mode >= 2) wait_read_window(period, win_w);
        Y y[U][E];
#pragma unroll
        for (int u = 0; u < U; ++u) add_client(k + u, y[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[u][e]);
    }
    for (; k < K; ++k) {
        Y y[E];
        add_client(k, y);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += (double)widen<Y, double>(y[e]);
    }
    double mo[E], vo[E];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        double mi[H] = {}, vv[H] = {};
        opt_load_state<H>(b, OptScalars{}, at(h), H, mi, vv);
#pragma unroll
        for (int e = 0; e < H; ++e) {
            mo[h * H + e] = mi[e] + acc[h * H + e];
            vo[h * H + e] = vv[e] + acc[h * H + e];
        }
    }
    wait_write_window(period, win_w);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        strip_store<double, H, 1>(static_cast<double*>(b.v_out) + at(h), *reinterpret_cast<double(*)[H]>(&vo[h * H]));
        strip_store<double, H, 1>(static_cast<double*>(b.out) + at(h), *reinterpret_cast<double(*)[H]>(&acc[h * H]));
        strip_store<double, H, 1>(static_cast<double*>(b.m_out) + at(h), *reinterpret_cast<double(*)[H]>(&mo[h * H]));
    }
}
#endif

template <typename Y, typename OLD, class PG, int E, bool FIRST, bool FINAL, bool NT, bool NOST = false, int OSM = 0>
__global__ void __launch_bounds__(kBlock)
k_fedopt(const OptBuffers b, const OptScalars s, const ClientTable<typename PG::S> tab, const int K, const int64_t P) {
    const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * E;
    if (i0 < P) fedopt_strip<Y, OLD, PG, E, FIRST, FINAL, NT, NOST, OSM>(b, s, tab, K, P, i0);
}

// ----------------------------------------------------------------------------
// numpyhelper primitives (numpyhelper.py:34-142) as elementwise kernels, numpy rounding:
// every product/quotient in its operand's dtype (python floats are weak scalars), the
// final combination in the promoted dtype.
// ----------------------------------------------------------------------------
template <typename T> __device__ __forceinline__ T as_t(double v) { return (T)v; }

// numpyhelper.add / subtract on float16 arrays: x*a + y*b with the python scalars cast to half and
// every op computed in float and rounded to half (numpy's half loops)
__global__ void __launch_bounds__(kBlock) k_axpby_half(f16* __restrict__ out, const f16* __restrict__ x,
                                                       const f16* __restrict__ y, float ah, float bh, int64_t P) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P; i += (int64_t)gridDim.x * kBlock) {
        const float xa = CF16::rh(f16_to_f32(x[i].bits) * ah);
        const float yb = CF16::rh(f16_to_f32(y[i].bits) * bh);
        out[i] = f16{f32_to_f16(xa + yb)};
    }
}

template <typename TX, typename TY, typename TO>
__global__ void __launch_bounds__(kBlock)
k_elementwise(int op, TO* __restrict__ out, const TX* __restrict__ x, const TY* __restrict__ y, double a, double b,
              int64_t P) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P; i += (int64_t)gridDim.x * kBlock) {
        TO r;
        switch (op) {
            case FA_EW_AXPBY: {                                   // x*a + y*b   (numpyhelper.add)
                const TX xa = x[i] * as_t<TX>(a);
                const TY yb = y[i] * as_t<TY>(b);
                r = (TO)xa + (TO)yb;
                break;
            }
            case FA_EW_MUL:                                       // numpyhelper.multiply
                r = y ? (TO)x[i] * (TO)y[i] : (TO)(x[i] * as_t<TX>(a));
                break;
            case FA_EW_DIV:                                       // numpyhelper.divide
                r = y ? (TO)x[i] / (TO)y[i] : (TO)(x[i] / as_t<TX>(a));
                break;
            case FA_EW_SQRT:                                      // numpyhelper.sqrt
                r = (TO)__builtin_sqrt((double)x[i]);
                if constexpr (std::is_same<TX, float>::value) r = (TO)__builtin_sqrtf(x[i]);
                break;
            case FA_EW_SQUARE:                                    // numpyhelper.power(m, 2)
                r = (TO)(x[i] * x[i]);
                break;
            case FA_EW_SIGN: {                                    // numpyhelper.sign
                const TX v = x[i];
                r = v > (TX)0 ? (TO)1 : (v < (TX)0 ? (TO)-1 : (v == (TX)0 ? (TO)0 : (TO)v));
                break;
            }
            case FA_EW_POW:                                       // numpyhelper.power(m, a), float a
                if constexpr (std::is_same<TX, float>::value) r = (TO)(float)::pow((double)x[i], a);
                else r = (TO)::pow((double)x[i], a);
                break;
            default:                                              // FA_EW_FILL: np.ones(shape) * a
                r = (TO)(1.0 * a);
                break;
        }
        out[i] = r;
    }
}

// numpyhelper.power on an integer array with a non-negative python int exponent: numpy's
// exponentiation by squaring in the array's integer type (wrapping products).
template <typename T>
__global__ void __launch_bounds__(kBlock) k_ipow(T* __restrict__ out, const T* __restrict__ x, uint64_t e, int64_t P) {
    // products in uint64 (no signed overflow, no promotion of 8/16-bit operands to int): x**e mod
    // 2**64 taken mod 2**bits(T) is numpy's wrapped result in T
    using U = typename std::make_unsigned<T>::type;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P; i += (int64_t)gridDim.x * kBlock) {
        uint64_t base = (uint64_t)(U)x[i], r = 1;
        for (uint64_t k = e; k; k >>= 1) {
            if (k & 1) r *= base;
            base *= base;
        }
        out[i] = (T)(U)r;
    }
}

// numpyhelper.increment_average (numpyhelper.py:32) on integer arrays folded with a python-float
// num_examples: numpy subtracts in the integer dtype (wrapping), multiplies the difference by the
// float n in float64, divides by N in float64 and adds x in float64 — each op rounded once.
// Any integer width: the difference is taken in the same-width unsigned type (no signed overflow)
// and wrapped back to T.
template <typename T>
__global__ void __launch_bounds__(kBlock) k_ifold(double* __restrict__ out, const T* __restrict__ x,
                                                  const T* __restrict__ y, double n, double N, int64_t P) {
    using U = typename std::make_unsigned<T>::type;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P; i += (int64_t)gridDim.x * kBlock) {
        const T d = (T)(U)((U)y[i] - (U)x[i]);
        double t = (double)d * n;
        t = t / N;
        out[i] = (double)x[i] + t;
    }
}

// The same fold with a python-INT num_examples (numpy's weak int scalar takes the array's dtype):
// difference AND product wrap in T (computed in a >= 32-bit unsigned type, so no signed overflow
// and no int promotion surprises for 8/16-bit T), then true_divide by N in float64 and add x.
template <typename T>
__global__ void __launch_bounds__(kBlock) k_nfold(double* __restrict__ out, const T* __restrict__ x,
                                                  const T* __restrict__ y, T n, double N, int64_t P) {
    using U = typename std::make_unsigned<T>::type;
    using W = typename std::conditional<(sizeof(T) < 8), uint32_t, uint64_t>::type;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P; i += (int64_t)gridDim.x * kBlock) {
        const W d = (W)(U)((W)(U)y[i] - (W)(U)x[i]);
        const T p = (T)(U)(d * (W)(U)n);
        out[i] = (double)x[i] + (double)p / N;
    }
}

// numpyhelper.norm (numpyhelper.py:106-117): np.linalg.norm(x, 1) of one tensor, accumulated in f64
// with a fixed (deterministic) order. Vector: sum |x|, grid-stride partials per block then one
// block sums the partials. Matrix (rows x cols, C order): column sums of |x| (one lane per
// column, rows in order), then the max over columns (NaN propagates, as numpy's max).
constexpr int kNormBlocks = 1024;
template <typename T>
__global__ void __launch_bounds__(kBlock) k_abssum_partial(const T* __restrict__ x, int64_t P, double* __restrict__ work) {
    __shared__ double red[kBlock];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P; i += (int64_t)gridDim.x * kBlock)
        acc += __builtin_fabs((double)x[i]);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) work[blockIdx.x] = red[0];
}
template <typename T>
__global__ void __launch_bounds__(kBlock) k_colabssum(const T* __restrict__ x, int64_t rows, int64_t cols,
                                                      double* __restrict__ work) {
    for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < cols; c += (int64_t)gridDim.x * kBlock) {
        double acc = 0.0;
        for (int64_t r = 0; r < rows; ++r) acc += __builtin_fabs((double)x[r * cols + c]);
        work[c] = acc;
    }
}
__global__ void __launch_bounds__(kBlock) k_final_reduce(const double* __restrict__ work, int64_t n, int is_max,
                                                         double* __restrict__ out) {
    __shared__ double red[kBlock];
    double acc = is_max ? -__builtin_inf() : 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kBlock) {
        const double v = work[i];
        acc = is_max ? (acc != acc ? acc : (v != v || v > acc ? v : acc)) : acc + v;   // NaN wins, as numpy max
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            const double a = red[threadIdx.x], b = red[threadIdx.x + w];
            red[threadIdx.x] = is_max ? (a != a ? a : (b != b || b > a ? b : a)) : a + b;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = (n == 0 && is_max) ? 0.0 : red[0];
}

// ----------------------------------------------------------------------------
// broadcast + widening conversion (fa_cast): numpy's implicit operand preparation when a
// client update differs from the running model in dtype or broadcastable shape. Only the
// per-tensor path (fedn_amd/mixed.py) uses it; the uniform-round kernels above never do.
// ----------------------------------------------------------------------------
constexpr int kCastMaxDim = 8;
struct CastGeom {
    int64_t shape[kCastMaxDim];    // out shape (C order)
    int64_t stride[kCastMaxDim];   // element strides of `in` per out dimension (0 = broadcast)
    int ndim;
};

template <> __device__ __forceinline__ double widen<f16, double>(f16 v) { return (double)f16_to_f32(v.bits); }

template <typename TI, typename TO, bool BC>
__global__ void __launch_bounds__(kBlock)
k_cast(TO* __restrict__ out, const TI* __restrict__ in, const CastGeom g, const int64_t P) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < P; i += (int64_t)gridDim.x * kBlock) {
        int64_t j = i;
        if constexpr (BC) {
            int64_t rem = i;
            j = 0;
            for (int d = g.ndim - 1; d >= 0; --d) {
                const int64_t q = rem / g.shape[d];
                j += (rem - q * g.shape[d]) * g.stride[d];
                rem = q;
            }
        }
        if constexpr (std::is_same<TO, f16>::value && std::is_integral<TI>::value)
            out[i] = f16{f32_to_f16((float)in[j])};          // int8 / uint8 only: exact in half
        else if constexpr (std::is_same<TO, f16>::value && std::is_same<TI, float>::value)
            out[i] = f16{f32_to_f16(in[j])};                 // narrowing: round to nearest even (astype)
        else if constexpr (std::is_same<TO, float>::value && std::is_same<TI, double>::value)
            out[i] = (float)in[j];                           // narrowing: round to nearest even (astype)
        else
            out[i] = widen<TI, TO>(in[j]);
    }
}

// ----------------------------------------------------------------------------
// k_push: one folded piece to every peer's copy of the model (fa_push; sharded.P2PAllGather's
// "kernel" engine). Each lane loads a 16-B word of the piece ONCE and stores it to every
// destination: the piece crosses each peer's own xGMI link once, all links at once, and local HBM
// is read once instead of once per DMA copy. The stores are plain vector stores (non-temporal:
// nothing here is read back by this GPU); k_release after the grid makes them visible to the peers
// before the stream's next operation (the fence the ranks exchange).
// ----------------------------------------------------------------------------
constexpr int kPushWords = 4;                    // 16-B words per lane per iteration (64 B in flight)

__global__ void __launch_bounds__(kBlock) k_push(PushTable t, int nd, const u32x4* __restrict__ src, int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * kBlock * kPushWords;
    for (int64_t base = (int64_t)blockIdx.x * kBlock * kPushWords + threadIdx.x; base < n16; base += stride) {
        u32x4 v[kPushWords];
#pragma unroll
        for (int j = 0; j < kPushWords; ++j) {
            const int64_t i = base + (int64_t)j * kBlock;
            if (i < n16) v[j] = __builtin_nontemporal_load(src + i);
        }
        for (int d = 0; d < nd; ++d) {
            u32x4* __restrict__ o = t.dst[d];
#pragma unroll
            for (int j = 0; j < kPushWords; ++j) {
                const int64_t i = base + (int64_t)j * kBlock;
                if (i < n16) __builtin_nontemporal_store(v[j], o + i);
            }
        }
    }
}

// the < 16 B tail of a piece whose length is not a multiple of 16 (one lane per byte)
__global__ void k_push_tail(PushTable t, int nd, const uint8_t* __restrict__ src, int64_t off, int rem) {
    const int b = threadIdx.x;
    if (b < rem)
        for (int d = 0; d < nd; ++d) reinterpret_cast<uint8_t*>(t.dst[d])[off + b] = src[off + b];
}

#ifdef FEDAGG_PROBES
// ----------------------------------------------------------------------------
// measurement kernels (libfedagg_probe.so only)
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_stream_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, int64_t n16) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n16) dst[i] = __builtin_nontemporal_load(src + i);
}

constexpr int kReadPerLane = 16;
template <int RPL>
__global__ void __launch_bounds__(kBlock) k_stream_read(const u32x4* __restrict__ src, int64_t n16, u32x4* __restrict__ sink) {
    const int64_t base = (int64_t)blockIdx.x * kBlock * RPL + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
        const int64_t i = base + (int64_t)j * kBlock;
        if (i < n16) acc ^= __builtin_nontemporal_load(src + i);
    }
    // one 16-B word per block keeps the loads alive; the bandwidth probe needs no exact reduction
    __shared__ u32x4 red[kBlock];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        u32x4 r = red[0];
        for (int t = 1; t < kBlock; ++t) r ^= red[t];
        sink[blockIdx.x] = r;
    }
}
#endif  // FEDAGG_PROBES

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Launch configuration. The product library (libfedagg.so) is built with the measured-best
// settings as compile-time constants: nothing in it is mutable or process-global. The probe
// build (-DFEDAGG_PROBES -> libfedagg_probe.so, tools/ and the division tests only) adds the
// fa_tune knobs that produced those measurements (profiles/r01_microbench.md).
#ifdef FEDAGG_PROBES
struct FedAvgCfg {
    std::atomic<int> strips{4}, unroll{0}, lanetab{0}, grid_per_cu{0}, read_per_lane{16}, block_log{8},
        sum_nostore{0}, nt_store{1}, nt{0}, tilemap{0}, fastdiv{1}, fastdiv64{1}, opt_nt{1}, opt_nostore{0}, opt_store{0}, opt_coal{2}, narrow{1}, lds_kib{0}, wpe{0}, opt_mv{0}, auto_geom{1}, opt_mix{0}, opt_burst{0}, opt_g{0}, opt_win_period{0}, opt_win_w{0}, opt_win_mode{0}, avg_win_period{0}, avg_win_w{0}, avg_win_mode{0}, opt_win_prod{0}, opt_quad{0};
};
FedAvgCfg g_cfg;
int cfg_fastdiv() { return g_cfg.fastdiv.load(std::memory_order_relaxed); }
int cfg_fastdiv64() { return g_cfg.fastdiv64.load(std::memory_order_relaxed); }
int cfg_grid_per_cu() { return g_cfg.grid_per_cu.load(std::memory_order_relaxed); }
#else
constexpr int cfg_fastdiv() { return 1; }     // fp32 t/N via the exact RN64(1/N) product
constexpr int cfg_fastdiv64() { return 1; }   // fp64 t/N via RN64(1/N) + two exact corrections (§3.2b)
constexpr int cfg_grid_per_cu() { return 0; } // one 16-KiB-per-client tile per workgroup
#endif

template <typename S>
void fill_table(ClientTable<S>& t, const void* const* ptrs, const double* n, const double* N, int k0, int cnt) {
    for (int j = 0; j < cnt; ++j) {
        t.ptr[j] = ptrs[k0 + j];
        t.n[j] = (S)n[k0 + j];
        t.N[j] = (S)N[k0 + j];
        if constexpr (std::is_same<S, double>::value) {
            // CF64's division shortcut: r = RN64(1/N) for 2^-60 <= |N| <= 2^60 (CWSUM ignores r,
            // CRUN overwrites it)
            const double Nd = N[k0 + j], a = std::fabs(Nd);
            t.r[j] = (cfg_fastdiv64() && a >= 0x1p-60 && a <= 0x1p60) ? 1.0 / Nd : 0.0;
        } else {
            // reciprocal for CF32's division shortcut: only for N that keep every normal-range
            // quotient normal (|N| < 2^28) and only when enabled
            const float Nf = (float)N[k0 + j];
            t.r[j] = (cfg_fastdiv() && Nf != 0.0f && std::fabs(Nf) < 0x1p28f) ? 1.0 / (double)Nf : 0.0;
        }
    }
    for (int j = cnt; j < kMaxK; ++j) {
        t.ptr[j] = nullptr;
        t.n[j] = 0;
        t.N[j] = 0;
        t.r[j] = 0.0;
    }
}

// numpy's conversion of a python int to float16 (round-to-nearest-even), kept in f32
// a python float / int as numpy's float16 weak scalar: ONE round-to-nearest-even from double (held in
// an f32; every half is exact in f32)
float to_half_value(double v) { return (float)(_Float16)v; }

int64_t grid_for(int64_t P, int E) {
    const int64_t strips = (P + E - 1) / E;
    return (strips + kBlock - 1) / kBlock;
}

int device_cus() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return cus > 0 ? cus : 256;
}

// The chip-wide store window of a single-launch FedOpt step (k_fedopt_cw), in 10-ns ticks of the
// reference clock, from the time one round of resident waves takes to stream its tiles at 6.4 TB/s
// (periods past ~1.5 rounds leave waves waiting for their window: 1.3-2x slower). Measured
// (profiles/r05_fedopt_window_product.log, 350 M params, every variant bit-exact):
//  - a launch that reads no optimizer state (a session's first round): period 0.65 round, window the
//    write share + 15 % of it: -8...-11 % at K = 32-64, -4...-5 % at K = 16;
//  - one that reads m and v (the steady state): period 0.35 round, window 15 %: -4...-9 % at K = 32,
//    -8...-10 % at K = 48 and 64 — but slower at K = 16 at every period tried, so only K >= 32.
// {0, 0}: no window — under 8 clients (under 32 with state), models under 2^24 elements, write
// shares over 25 %.
struct StoreWindow {
    uint32_t period = 0, w = 0;
};
template <typename Y, typename OLD, class PG, bool NT>
StoreWindow opt_store_window(const OptBuffers& b, int K, int64_t P) {
    const bool state = b.m_in_f64 >= 0 || b.v_in;
    if (K < (state ? 32 : 8) || P < ((int64_t)1 << 24)) return {};
    static std::atomic<int> blocks_per_cu{-1};            // resident workgroups per CU, per instantiation
    int nb = blocks_per_cu.load(std::memory_order_relaxed);
    if (nb < 0) {
        nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_fedopt_cw<Y, OLD, PG, NT>, kBlock, 0) != hipSuccess) nb = 0;
        blocks_per_cu.store(nb, std::memory_order_relaxed);
    }
    if (nb <= 0) return {};
    const double waves = (double)nb * (kBlock / 64) * device_cus();
    const double m_in = b.m_in_f64 == 1 ? 8 : b.m_in_f64 == 0 ? 4 : b.m_in_f64 < 0 ? 0 : 2;
    const double m_out = b.m_out_f64 == 1 ? 8 : b.m_out_f64 == 0 ? 4 : 2;
    const double rd = (double)K * sizeof(Y) + sizeof(OLD) + m_in + (b.v_in ? (b.v_in_f32 ? 4 : 8) : 0);
    const double wr = (b.out_f32 ? 4 : 8) + (b.v_out_f32 ? 4 : 8) + m_out;
    const double frac = wr / (rd + wr);
    if (frac > 0.25) return {};
    const double period = (state ? 0.35 : 0.65) * waves * 512.0 * (rd + wr) / 6.4e12 * 1e8;
    if (period < 1000 || period > 20000) return {};
    StoreWindow sw;
    sw.period = (uint32_t)period;
    sw.w = (uint32_t)(period * (state ? 0.15 : std::min(0.30, std::max(0.08, 1.15 * frac))));
    return sw;
}


// The store window of a first FedAvg launch (k_fedavg_pipe_win), in 10-ns ticks of the reference
// clock: period 0.45 of the time one round of resident workgroups streams its tiles at 6.4 TB/s,
// window 15 % — measured (profiles/r05_fedavg_window.log, 100 M fp32, bit-exact, two boxes) at
// K = 64: 0.24-0.47 round -5...-7 %, 0.6 round and longer +2...+22 %; K = 8: 0.34-0.42 round -6 %,
// 0.64 round 0 %; bf16 updates at K = 64 -5 %, at K = 8 (a 20 % write share) +4 %. {0, 0}: no window
// (write shares over 15 %, models under 2^24 elements, periods under 500 ticks).
struct AvgWindow {
    uint32_t period = 0, w = 0;
};
template <typename Y, typename X, class CP, int E, int S, bool NT, bool LT, int BLK, int NTS, int MAP>
AvgWindow avg_store_window(int K, int64_t P) {
    if (P < ((int64_t)1 << 24) || K < 2) return {};
    static std::atomic<int> blocks_per_cu{-1};
    int nb = blocks_per_cu.load(std::memory_order_relaxed);
    if (nb < 0) {
        nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_fedavg_pipe_win<Y, X, CP, E, S, true, false, NT, LT, BLK, NTS, MAP>,
                                                         BLK, 0) != hipSuccess)
            nb = 0;
        blocks_per_cu.store(nb, std::memory_order_relaxed);
    }
    if (nb <= 0) return {};
    if ((double)sizeof(X) / ((double)K * sizeof(Y) + sizeof(X)) > 0.15) return {};
    const double round_bytes = (double)nb * device_cus() * BLK * S * E * ((double)K * sizeof(Y) + sizeof(X));
    const double period = 0.45 * round_bytes / 6.4e12 * 1e8;
    if (period < 500 || period > 20000) return {};
    AvgWindow w;
    w.period = (uint32_t)period;
    w.w = (uint32_t)(0.15 * period);
    return w;
}

template <typename Y, typename X, class CP, int E, int S, bool NT, bool LT, int BLK = kBlock, int NTS = 0, int MAP = 0>
void launch_fedavg_pipe(X* a, const ClientTable<typename CP::S>& tab, int cnt, int64_t P, bool first, bool int_first,
                        hipStream_t st) {
    g_kernel = "k_fedavg_pipe";
    const int64_t strips = (P + E - 1) / E;
    int64_t ntiles = (strips + (int64_t)BLK * S - 1) / ((int64_t)BLK * S);
    if (cfg_grid_per_cu() > 0) {
        if constexpr (MAP != 0) return launch_fedavg_pipe<Y, X, CP, E, S, NT, LT, BLK, NTS, 0>(a, tab, cnt, P, first, int_first, st);
        ntiles = std::min<int64_t>(ntiles, (int64_t)cfg_grid_per_cu() * device_cus());
    }
    const dim3 grid((unsigned)ntiles);
    unsigned shm = 0;
    // the fp32 fold with a first launch (the BASELINE workload's shape): its stores in the chip-wide
    // window; other dtypes / continuation launches were not measured with one
    if constexpr (std::is_same<CP, CF32>::value && std::is_same<X, float>::value &&
                  ((std::is_same<Y, float>::value && S * E == 16) || (std::is_same<Y, bf16>::value && S * E == 32)) &&
                  BLK == kBlock && MAP == 0 && !LT && !NT && NTS == 1) {
        if (first && !int_first && cfg_grid_per_cu() == 0) {
            AvgWindow w = avg_store_window<Y, X, CP, E, S, NT, LT, BLK, NTS, MAP>(cnt, P);
            int wm = 0;
#ifdef FEDAGG_PROBES
            if (g_cfg.avg_win_period < 0 || g_cfg.wpe > 0 || g_cfg.lds_kib > 0) w = AvgWindow{};   // A/B and the other probes
            else if (g_cfg.avg_win_period > 0) {
                w = AvgWindow{(uint32_t)g_cfg.avg_win_period.load(), (uint32_t)g_cfg.avg_win_w.load()};
                wm = g_cfg.avg_win_mode.load();
            }
#endif
            if (w.period) {
                g_kernel = "k_fedavg_pipe_win";
                hipLaunchKernelGGL((k_fedavg_pipe_win<Y, X, CP, E, S, true, false, NT, LT, BLK, NTS, MAP>), grid, dim3(BLK), 0, st, a,
                                   tab, cnt, P, w.period, w.w, wm);
                return;
            }
        }
    }
#ifdef FEDAGG_PROBES
    shm = (unsigned)g_cfg.lds_kib * 1024u;     // occupancy probe: LDS the kernel never touches
    if constexpr (std::is_same<CP, CF32>::value && std::is_same<X, float>::value && S * E * (int)sizeof(Y) == 64 &&
                  BLK == kBlock && MAP == 0 && !LT && !NT && NTS == 1) {
        if (g_cfg.avg_win_period > 0 && !int_first && !first) {
            const uint32_t wl = (uint32_t)g_cfg.avg_win_period.load(), ww = (uint32_t)g_cfg.avg_win_w.load();
            hipLaunchKernelGGL((k_fedavg_pipe_win<Y, X, CP, E, S, false, false, NT, LT, BLK, NTS, MAP>), grid, dim3(BLK), shm, st, a, tab,
                               cnt, P, wl, ww, g_cfg.avg_win_mode.load());
            return;
        }
        const int w = g_cfg.wpe;
        if (w > 0 && !int_first) {
#define FA_WPE(W_)                                                                                                      \
    if (w == W_) {                                                                                                      \
        if (first) hipLaunchKernelGGL((k_fedavg_pipe_w<Y, X, CP, E, S, true, false, NT, LT, BLK, NTS, MAP, W_>), grid, dim3(BLK), shm, st, a, tab, cnt, P); \
        else hipLaunchKernelGGL((k_fedavg_pipe_w<Y, X, CP, E, S, false, false, NT, LT, BLK, NTS, MAP, W_>), grid, dim3(BLK), shm, st, a, tab, cnt, P); \
        return;                                                                                                         \
    }
            FA_WPE(5) FA_WPE(6) FA_WPE(8)
#undef FA_WPE
        }
    }
#endif
    if (first && int_first) {
        if constexpr (std::is_integral<Y>::value)
            hipLaunchKernelGGL((k_fedavg_pipe<Y, X, CP, E, S, true, true, NT, LT, BLK, NTS, MAP>), grid, dim3(BLK), shm, st, a, tab, cnt, P);
    } else if (first)
        hipLaunchKernelGGL((k_fedavg_pipe<Y, X, CP, E, S, true, false, NT, LT, BLK, NTS, MAP>), grid, dim3(BLK), shm, st, a, tab, cnt, P);
    else
        hipLaunchKernelGGL((k_fedavg_pipe<Y, X, CP, E, S, false, false, NT, LT, BLK, NTS, MAP>), grid, dim3(BLK), shm, st, a, tab, cnt, P);
}

template <typename Y, typename X, class CP, int E, int S, int U, bool NT>
void launch_fedavg_geom(X* a, const ClientTable<typename CP::S>& tab, int cnt, int64_t P, bool first, bool int_first,
                        hipStream_t st) {
    g_kernel = "k_fedavg";
    const int64_t strips = (P + E - 1) / E;
    const dim3 grid((unsigned)((strips + (int64_t)kBlock * S - 1) / ((int64_t)kBlock * S)));
    if (first && int_first) {
        if constexpr (std::is_integral<Y>::value)
            hipLaunchKernelGGL((k_fedavg<Y, X, CP, E, S, U, true, true, NT>), grid, dim3(kBlock), 0, st, a, tab, cnt, P);
    } else if (first)
        hipLaunchKernelGGL((k_fedavg<Y, X, CP, E, S, U, true, false, NT>), grid, dim3(kBlock), 0, st, a, tab, cnt, P);
    else
        hipLaunchKernelGGL((k_fedavg<Y, X, CP, E, S, U, false, false, NT>), grid, dim3(kBlock), 0, st, a, tab, cnt, P);
}

// Launch geometry by model size (profiles/r02_tile_probe.log). Every workgroup folds all K
// clients over one tile, so the grid must be many times the ~1,024 resident workgroups or its
// last partial wave decides the time. The pipelined 4-strip kernel (16 KiB of each client per
// tile) is the fastest once each client buffer is >= kPipeMinClientBytes (>= 10 K tiles: 0.74-0.75
// of peak at 64 x 100 M fp32 and bf16); below that, one 16-B strip per lane with 4 (fp32) or 8
// (narrower types, or K <= 8) clients loaded ahead — 4 KiB tiles — holds 0.65-0.80 where the
// 4-strip tiles drop to 0.25-0.55 (bf16 10 M: 0.27 -> 0.65; fp32 3 M x 64: 0.45 -> 0.67).
constexpr int64_t kPipeMinClientBytes = 160ll << 20;

template <typename Y>
inline bool pipe_pays(int64_t P) { return P * (int64_t)sizeof(Y) >= kPipeMinClientBytes; }

template <typename Y, typename X, class CP, int E>
void launch_fedavg_small(X* a, const ClientTable<typename CP::S>& tab, int cnt, int64_t P, bool first, bool int_first,
                         hipStream_t st);

template <class CP> struct is_sf_rule : std::false_type {};
template <typename Y, typename X> struct is_sf_rule<CWSUM<Y, X>> : std::true_type {};
template <typename T_> struct is_sf_rule<CRUN<T_>> : std::true_type {};

// The tunable geometries are instantiated for the fp32 hot path only; other dtypes use the default.
template <typename Y, typename X, class CP, int E>
void launch_fedavg_vec(X* a, const ClientTable<typename CP::S>& tab, int cnt, int64_t P, bool first, bool int_first,
                       hipStream_t st) {
    constexpr bool tunable = (std::is_same<Y, float>::value || std::is_same<Y, bf16>::value) && std::is_same<X, float>::value &&
                             std::is_same<CP, CF32>::value;
    if constexpr (is_sf_rule<CP>::value) {
        if (!pipe_pays<Y>(P)) return launch_fedavg_small<Y, X, CP, E>(a, tab, cnt, P, first, int_first, st);
        launch_fedavg_pipe<Y, X, CP, E, 4, false, false>(a, tab, cnt, P, first, int_first, st);
        return;
    }
    if constexpr (tunable) {
#ifdef FEDAGG_PROBES
        const int block_log = g_cfg.block_log, strips = g_cfg.strips, unroll = g_cfg.unroll, nt = g_cfg.nt;
        const int lanetab = g_cfg.lanetab, nt_store = g_cfg.nt_store, tilemap = g_cfg.tilemap;
        const int key = (block_log == 9 ? 20000 : block_log == 10 ? 30000 : 0) + lanetab * 10000 + strips * 100 +
                        unroll * 2 + nt;
        // the default settings select the product's size-dependent geometry (FA_TUNE_AUTO_GEOM 0 forces them)
        if (g_cfg.auto_geom && key == 4 * 100 + 0 && nt_store == 1 && tilemap == 0 && !pipe_pays<Y>(P))
            return launch_fedavg_small<Y, X, CP, E>(a, tab, cnt, P, first, int_first, st);
        if constexpr (sizeof(Y) < sizeof(X) && E % 2 == 0) {
            if (g_cfg.narrow && key == 4 * 100 + 0 && nt_store == 1 && tilemap == 0)
                return launch_fedavg_pipe<Y, X, CP, E / 2, 8, false, false, kBlock, 1>(a, tab, cnt, P, first, int_first, st);
        }
        switch (key) {
#define FA_GEOM(S_, U_, NT_) \
    case S_ * 100 + U_ * 2 + NT_: return launch_fedavg_geom<Y, X, CP, E, S_, U_, NT_>(a, tab, cnt, P, first, int_first, st);
            FA_GEOM(1, 4, 0) FA_GEOM(1, 8, 0) FA_GEOM(1, 16, 0) FA_GEOM(2, 4, 0) FA_GEOM(2, 8, 0) FA_GEOM(2, 16, 0)
            FA_GEOM(4, 1, 0) FA_GEOM(4, 2, 0) FA_GEOM(4, 4, 0) FA_GEOM(8, 1, 0) FA_GEOM(8, 2, 0) FA_GEOM(16, 1, 0)
            FA_GEOM(1, 8, 1) FA_GEOM(4, 2, 1) FA_GEOM(8, 1, 1)
            case 2 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 2, false, false>(a, tab, cnt, P, first, int_first, st);
            case 4 * 100 + 0:
                if (nt_store == 1 && tilemap > 0) {
                    switch (tilemap) {
#define FA_MAP(R_) \
    case R_: return launch_fedavg_pipe<Y, X, CP, E, 4, false, false, kBlock, 1, R_>(a, tab, cnt, P, first, int_first, st);
                        FA_MAP(2) FA_MAP(4) FA_MAP(8) FA_MAP(16) FA_MAP(32)
#undef FA_MAP
                        default: break;
                    }
                }
                if (nt_store == 1) return launch_fedavg_pipe<Y, X, CP, E, 4, false, false, kBlock, 1>(a, tab, cnt, P, first, int_first, st);
                if (nt_store == 2) return launch_fedavg_pipe<Y, X, CP, E, 4, false, false, kBlock, 2>(a, tab, cnt, P, first, int_first, st);
                return launch_fedavg_pipe<Y, X, CP, E, 4, false, false>(a, tab, cnt, P, first, int_first, st);
            case 8 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 8, false, false>(a, tab, cnt, P, first, int_first, st);
            case 4 * 100 + 1: return launch_fedavg_pipe<Y, X, CP, E, 4, true, false>(a, tab, cnt, P, first, int_first, st);
            case 20000 + 4 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 4, false, false, 512>(a, tab, cnt, P, first, int_first, st);
            case 30000 + 4 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 4, false, false, 1024>(a, tab, cnt, P, first, int_first, st);
            case 20000 + 8 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 8, false, false, 512>(a, tab, cnt, P, first, int_first, st);
            case 30000 + 2 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 2, false, false, 1024>(a, tab, cnt, P, first, int_first, st);
            case 10000 + 2 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 2, false, true>(a, tab, cnt, P, first, int_first, st);
            case 10000 + 4 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 4, false, true>(a, tab, cnt, P, first, int_first, st);
            case 10000 + 8 * 100 + 0: return launch_fedavg_pipe<Y, X, CP, E, 8, false, true>(a, tab, cnt, P, first, int_first, st);
#undef FA_GEOM
            default: break;
        }
#else
        if (!pipe_pays<Y>(P)) return launch_fedavg_small<Y, X, CP, E>(a, tab, cnt, P, first, int_first, st);
        // measured best on MI355X (profiles/r01_microbench.md): 4 x 16-B strips per lane, the next
        // client's strips in flight (pipelined), cached loads, non-temporal aggregate stores.
        // bf16 clients: strips of 4 elements (8-B loads, 16-B f32 stores), 8 per lane, so every wave
        // store is one contiguous 1 KiB — +3.5 % at K = 64, +7 % at K = 8 (profiles/r02_narrow_probe.log)
        if constexpr (sizeof(Y) < sizeof(X) && E % 2 == 0)
            return launch_fedavg_pipe<Y, X, CP, E / 2, 8, false, false, kBlock, 1>(a, tab, cnt, P, first, int_first, st);
        else
            return launch_fedavg_pipe<Y, X, CP, E, 4, false, false, kBlock, 1>(a, tab, cnt, P, first, int_first, st);
#endif
    }
    launch_fedavg_geom<Y, X, CP, E, 1, kUnroll, false>(a, tab, cnt, P, first, int_first, st);
}

template <typename Y, typename X, class CP, int E>
void launch_fedavg_small(X* a, const ClientTable<typename CP::S>& tab, int cnt, int64_t P, bool first, bool int_first,
                         hipStream_t st) {
    if (sizeof(Y) < 4 || cnt <= 8) launch_fedavg_geom<Y, X, CP, E, 1, 8, false>(a, tab, cnt, P, first, int_first, st);
    else launch_fedavg_geom<Y, X, CP, E, 1, 4, false>(a, tab, cnt, P, first, int_first, st);
}

template <typename Y, typename X, class CP>
int launch_fedavg(void* agg, const void* const* ups, const double* n, const double* N, int K, int64_t P,
                  int init, bool int_first, hipStream_t st) {
    constexpr int E16 = 16 / (int)sizeof(Y) > 0 ? 16 / (int)sizeof(Y) : 1;
    bool vec = aligned16(agg);
    for (int k = 0; k < K && vec; ++k) vec = aligned16(ups[k]);
    using S = typename CP::S;
    ClientTable<S> tab;
    int k0 = 0;
    bool first = init != 0;
    X* a = static_cast<X*>(agg);
    while (k0 < K) {
        const int cnt = (K - k0) < kMaxK ? (K - k0) : kMaxK;
        fill_table<S>(tab, ups, n, N, k0, cnt);
        if (std::is_same<CP, CF16>::value) {
            for (int j = 0; j < cnt; ++j) {
                tab.n[j] = (S)to_half_value(n[k0 + j]);
                tab.N[j] = (S)to_half_value(N[k0 + j]);
            }
        }
        if (vec) launch_fedavg_vec<Y, X, CP, E16>(a, tab, cnt, P, first, int_first, st);
        else launch_fedavg_geom<Y, X, CP, 1, 1, kUnroll, false>(a, tab, cnt, P, first, int_first, st);
        int rc = check_launch("fa_fedavg_fold: kernel launch");
        if (rc) return rc;
        first = false;
        k0 += cnt;
    }
    return FA_OK;
}

template <typename Y, typename OLD, class PG, int E, bool NT>
int launch_fedopt_one(const OptBuffers& b, const OptScalars& s, const ClientTable<typename PG::S>& tab, int cnt,
                      int64_t P, bool first, bool final_, hipStream_t st) {
    g_kernel = E == 4 ? "k_fedopt_c" : "k_fedopt";
    const dim3 grid((unsigned)grid_for(P, E));
#ifdef FEDAGG_PROBES
    // the probe variants exist for the configs[3] shapes only (fp32 updates over an fp32 or fp64
    // model, vector path); every other combination runs the product kernels in the probe build too
    constexpr bool probe_combo = E == 4 && std::is_same<Y, float>::value &&
                                 (std::is_same<OLD, float>::value || std::is_same<OLD, double>::value);
    if constexpr (probe_combo) {
        if (final_ && g_cfg.opt_g && std::is_same<OLD, double>::value) {
            if (b.m_out_f64 != 1 || b.v_out_f32 || b.out_f32 || !b.v_in || b.v_in_f32)
                return fail(FA_EINVAL, "fa_tune OPT_G probe: fp64 m / v / model out, fp64 v in");
            const int G = g_cfg.opt_g;
            const dim3 gg((unsigned)((P + 4 * 512 * G - 1) / (4 * 512 * G)));
            switch (G) {
#define FA_OPTG(G_) \
    case G_: if (first) hipLaunchKernelGGL((k_fedopt_cg<Y, OLD, PG, true, NT, G_>), gg, dim3(kBlock), 0, st, b, s, tab, cnt, P); \
             else hipLaunchKernelGGL((k_fedopt_cg<Y, OLD, PG, false, NT, G_>), gg, dim3(kBlock), 0, st, b, s, tab, cnt, P); break;
                FA_OPTG(1) FA_OPTG(2) FA_OPTG(4)
#undef FA_OPTG
                default: return fail(FA_EINVAL, "fa_tune OPT_G: 1, 2 or 4 tiles per wave");
            }
            return check_launch("fa_fedopt_step: kernel launch");
        }
        if (first && final_ && g_cfg.opt_burst) {
            if (b.m_out_f64 != 1) return fail(FA_EINVAL, "fa_tune OPT_BURST probe: fp64 m out");
            const int G = g_cfg.opt_burst;
            const dim3 gb((unsigned)((P + 4 * 512 * G - 1) / (4 * 512 * G)));   // a ragged last group is skipped
            switch (G) {
#define FA_BURST(G_) \
    case G_: hipLaunchKernelGGL((k_fedopt_mixg<Y, OLD, typename PG::S, NT, G_>), gb, dim3(kBlock), 0, st, b, tab, cnt, P); break;
                FA_BURST(1) FA_BURST(2) FA_BURST(4)
#undef FA_BURST
                default: return fail(FA_EINVAL, "fa_tune OPT_BURST: 1, 2 or 4 tiles per wave");
            }
            return check_launch("fa_fedopt_step: kernel launch");
        }
        if (first && final_ && g_cfg.opt_win_period > 0 && !g_cfg.opt_win_prod) {
            if (b.m_out_f64 != 1) return fail(FA_EINVAL, "fa_tune OPT_WIN probe: fp64 m out");
            const dim3 gw((unsigned)((P + 4 * 512 - 1) / (4 * 512)));   // a ragged last tile is skipped
            hipLaunchKernelGGL((k_fedopt_mixw<Y, OLD, typename PG::S, NT>), gw, dim3(kBlock), 0, st, b, tab, cnt, P,
                               (uint32_t)g_cfg.opt_win_period.load(), (uint32_t)g_cfg.opt_win_w.load(), g_cfg.opt_win_mode.load());
            return check_launch("fa_fedopt_step: kernel launch");
        }
        if (first && final_ && g_cfg.opt_mix) {
            const dim3 gm((unsigned)((P + 4 * 512 - 1) / (4 * 512)));   // a ragged last tile is skipped
            hipLaunchKernelGGL((k_fedopt_mix<Y, OLD, typename PG::S, NT>), gm, dim3(kBlock), 0, st, b, tab, cnt, P);
            return check_launch("fa_fedopt_step: kernel launch");
        }
        if (first && final_ && g_cfg.opt_nostore) {
            hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, true, true, NT, true>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
            return check_launch("fa_fedopt_step: kernel launch");
        }
        if (first && final_ && g_cfg.opt_coal == 1) {   // 2 pairs per lane (a 256-element wave tile)
            hipLaunchKernelGGL((k_fedopt_c<Y, OLD, PG, true, true, NT, 1, 2>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
            return check_launch("fa_fedopt_step: kernel launch");
        }
        if (first && final_ && !g_cfg.opt_coal) {    // the per-lane 4-element strip map (r01), for A/B
            if (g_cfg.opt_store == 1)
                hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, true, true, NT, false, 1>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
            else if (g_cfg.opt_store == 2)
                hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, true, true, NT, false, 2>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
            else
                hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, true, true, NT>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
            return check_launch("fa_fedopt_step: kernel launch");
        }
    }
#endif
    if constexpr (E == 4) {
        // wave-coalesced element map, 4 pairs per lane (512-element wave tiles), non-temporal state /
        // model stores: +3-6 % over the per-lane strip map on configs[3], bit-identical
        // (profiles/r02_fedopt_coal_*.log); every vector-path update dtype (bf16 /
        // fp16 updates: one dword per pair)
        const dim3 g4((unsigned)((P + 4 * 512 - 1) / (4 * 512)));
#ifdef FEDAGG_PROBES
        if constexpr (std::is_same<Y, bf16>::value && std::is_same<OLD, double>::value && std::is_same<PG, CF64>::value) {
            if (g_cfg.opt_quad) {                    // configs[4]'s wave kernels with the quad element map
                g_kernel = "k_fedopt_cq";
                if (first && final_) hipLaunchKernelGGL((k_fedopt_cq<Y, OLD, PG, true, true, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
                else if (first) hipLaunchKernelGGL((k_fedopt_cq<Y, OLD, PG, true, false, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
                else if (final_) hipLaunchKernelGGL((k_fedopt_cq<Y, OLD, PG, false, true, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
                else hipLaunchKernelGGL((k_fedopt_cq<Y, OLD, PG, false, false, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
                return check_launch("fa_fedopt_step: kernel launch");
            }
        }
        const unsigned shm = (unsigned)g_cfg.lds_kib * 1024u;
        if constexpr (probe_combo) {
        if (first && final_ && g_cfg.opt_mv) {
            if (P % (4 * 512) || b.m_in_f64 != 1 || b.m_out_f64 != 1 || !b.v_in)
                return fail(FA_EINVAL, "fa_tune OPT_MV probe: P %% 2048 == 0, fp64 m in and out, v given");
            hipLaunchKernelGGL((k_fedopt_c_mv<Y, OLD, PG, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
            return check_launch("fa_fedopt_step: kernel launch");
        }
        if (first && final_ && !(g_cfg.opt_win_period > 0 && g_cfg.opt_win_prod)) {   // (a window: below)
            switch (g_cfg.wpe) {
#define FA_WPE(W_) \
    case W_: hipLaunchKernelGGL((k_fedopt_c_w<Y, OLD, PG, true, true, NT, 1, 4, kUnroll / 2, W_>), g4, dim3(kBlock), shm, st, b, s, tab, cnt, P); \
        return check_launch("fa_fedopt_step: kernel launch");
                FA_WPE(6) FA_WPE(8)
#undef FA_WPE
                default:
                    if (shm) {
                        hipLaunchKernelGGL((k_fedopt_c<Y, OLD, PG, true, true, NT, 1, 4>), g4, dim3(kBlock), shm, st, b, s, tab, cnt, P);
                        return check_launch("fa_fedopt_step: kernel launch");
                    }
                    break;                                  // the product's own choice below
            }
        }
        }
#endif
        if (first && final_) {
            StoreWindow sw = opt_store_window<Y, OLD, PG, NT>(b, cnt, P);
#ifdef FEDAGG_PROBES
            if (g_cfg.opt_win_period < 0) sw = StoreWindow{};                                 // A/B: no window
            else if (g_cfg.opt_win_period > 0 && g_cfg.opt_win_prod) sw = StoreWindow{(uint32_t)g_cfg.opt_win_period.load(),
                                                                                          (uint32_t)g_cfg.opt_win_w.load()};
#endif
#ifdef FEDAGG_PROBES
            if constexpr (probe_combo) {
                if (sw.period && g_cfg.opt_win_prod == 1 && (g_cfg.wpe == 6 || g_cfg.wpe == 7)) {
                    if (g_cfg.wpe == 6)
                        hipLaunchKernelGGL((k_fedopt_cw_w<Y, OLD, PG, NT, 6>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P, sw.period, sw.w);
                    else
                        hipLaunchKernelGGL((k_fedopt_cw_w<Y, OLD, PG, NT, 7>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P, sw.period, sw.w);
                    return check_launch("fa_fedopt_step: kernel launch");
                }
                if (sw.period && g_cfg.opt_win_prod == 3) {
                    const dim3 g2((unsigned)((P + 4 * 256 - 1) / (4 * 256)));
                    hipLaunchKernelGGL((k_fedopt_cw2<Y, OLD, PG, NT>), g2, dim3(kBlock), 0, st, b, s, tab, cnt, P, sw.period, sw.w);
                    return check_launch("fa_fedopt_step: kernel launch");
                }
                if (sw.period && g_cfg.opt_win_prod == 2) {
                    if (b.m_out_f64 != 1 || b.v_out_f32 || b.out_f32 || (b.v_in && b.v_in_f32))
                        return fail(FA_EINVAL, "fa_tune OPT_WIN_PROD 2: fp64 m / v / model out");
                    hipLaunchKernelGGL((k_fedopt_cgw<Y, OLD, PG, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P, sw.period, sw.w);
                    return check_launch("fa_fedopt_step: kernel launch");
                }
            }
#endif
            if (sw.period) {
                g_kernel = "k_fedopt_cw";
                hipLaunchKernelGGL((k_fedopt_cw<Y, OLD, PG, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P, sw.period, sw.w);
                return check_launch("fa_fedopt_step: kernel launch");
            }
        }
#ifdef FEDAGG_PROBES
        if (!final_ && g_cfg.opt_win_period > 0 && g_cfg.opt_win_prod) {
            const uint32_t per = (uint32_t)g_cfg.opt_win_period.load(), w = (uint32_t)g_cfg.opt_win_w.load();
            if (first)
                hipLaunchKernelGGL((k_fedopt_cwp<Y, OLD, PG, true, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P, per, w);
            else
                hipLaunchKernelGGL((k_fedopt_cwp<Y, OLD, PG, false, NT>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P, per, w);
            return check_launch("fa_fedopt_step: kernel launch");
        }
#endif
        if (first && final_) hipLaunchKernelGGL((k_fedopt_c<Y, OLD, PG, true, true, NT, 1, 4>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
        else if (first) hipLaunchKernelGGL((k_fedopt_c<Y, OLD, PG, true, false, NT, 1, 4>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
        else if (final_) hipLaunchKernelGGL((k_fedopt_c<Y, OLD, PG, false, true, NT, 1, 4>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
        else hipLaunchKernelGGL((k_fedopt_c<Y, OLD, PG, false, false, NT, 1, 4>), g4, dim3(kBlock), 0, st, b, s, tab, cnt, P);
    } else {
        if (first && final_) hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, true, true, NT>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
        else if (first) hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, true, false, NT>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
        else if (final_) hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, false, true, NT>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
        else hipLaunchKernelGGL((k_fedopt<Y, OLD, PG, E, false, false, NT>), grid, dim3(kBlock), 0, st, b, s, tab, cnt, P);
    }
    return check_launch("fa_fedopt_step: kernel launch");
}

template <typename Y, typename OLD, class PG>
int launch_fedopt(const OptBuffers& b, const OptScalars& s, const void* const* ups, const double* n, const double* N,
                  int K, int64_t P, int flags, hipStream_t st) {
    bool vec = aligned16(b.old) && aligned16(b.pg) && aligned16(b.m_in) && aligned16(b.m_out) && aligned16(b.v_in) &&
               aligned16(b.v_out) && aligned16(b.out);
    for (int k = 0; k < K && vec; ++k) vec = aligned16(ups[k]);
    using S = typename PG::S;
    ClientTable<S> tab;
    bool first = (flags & FA_PG_FIRST) != 0;
    const bool final_all = (flags & FA_PG_FINAL) != 0;
    int k0 = 0;
    do {
        const int cnt = (K - k0) < kMaxK ? (K - k0) : kMaxK;
        fill_table<S>(tab, ups, n, N, k0, cnt);
        if constexpr (std::is_same<PG, CF16>::value) {
            for (int j = 0; j < cnt; ++j) {       // numpy casts the python n, N to the half dtype
                tab.n[j] = (S)to_half_value(n[k0 + j]);
                tab.N[j] = (S)to_half_value(N[k0 + j]);
            }
        }
        const bool last = k0 + cnt >= K;
        const bool fin = last && final_all;
#ifdef FEDAGG_PROBES
        if constexpr (std::is_same<Y, float>::value && (std::is_same<OLD, float>::value || std::is_same<OLD, double>::value))
        if (vec && !g_cfg.opt_nt) {
            int rc = launch_fedopt_one<Y, OLD, PG, 4, false>(b, s, tab, cnt, P, first, fin, st);
            if (rc) return rc;
            first = false;
            k0 += cnt;
            continue;
        }
#endif
        int rc = vec ? launch_fedopt_one<Y, OLD, PG, 4, true>(b, s, tab, cnt, P, first, fin, st)
                     : launch_fedopt_one<Y, OLD, PG, 1, false>(b, s, tab, cnt, P, first, fin, st);
        if (rc) return rc;
        first = false;
        k0 += cnt;
    } while (k0 < K);
    return FA_OK;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int fa_abi_version(void) { return FA_ABI_VERSION; }

const char* fa_last_error(void) { return g_err; }
const char* fa_last_kernel(void) { return g_kernel; }

int fa_promote(int a, int b) {
    auto fl = [](int d) { return d == FA_BF16 ? FA_F32 : d; };
    if (a == FA_NONE) return fl(b);
    if (b == FA_NONE) return fl(a);
    a = fl(a);
    b = fl(b);
    if (a == b) return a;
    if (a == FA_F64 || b == FA_F64) return FA_F64;
    if ((a == FA_F32 && b == FA_F16) || (a == FA_F16 && b == FA_F32)) return FA_F32;
    return FA_NONE;
}

int fa_fedavg_fold(void* agg, int agg_dtype, const void* const* updates, int upd_dtype, const double* n, const double* N,
                   int K, int64_t P, int init, void* stream) {
    g_err[0] = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (P < 0 || K < 0) return fail(FA_EINVAL, "fa_fedavg_fold: negative size (P=%lld, K=%d)", (long long)P, K);
    if (init && K < 1) return fail(FA_EINVAL, "fa_fedavg_fold: init requires K >= 1");
    if (K == 0 || P == 0) return FA_OK;
    if (!agg || !updates || !n || !N) return fail(FA_EINVAL, "fa_fedavg_fold: null pointer argument");
    for (int k = 0; k < K; ++k)
        if (!updates[k]) return fail(FA_EINVAL, "fa_fedavg_fold: updates[%d] is NULL", k);
    if (init && K == 1) {
        if (agg_dtype != upd_dtype) return fail(FA_EDTYPE, "fa_fedavg_fold: K=1 init is a copy; dtypes must match");
        hipError_t e = hipMemcpyAsync(agg, updates[0], (size_t)P * dt_size(upd_dtype), hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return fail(FA_EHIP, "fa_fedavg_fold: hipMemcpyAsync: %s", hipGetErrorString(e));
        return FA_OK;
    }
    const bool int_first = init && (upd_dtype == FA_I64 || upd_dtype == FA_I32);
    // the first fold of integer updates multiplies in the integer dtype: numpy does that for an int
    // num_examples only (a float one multiplies in float64: fa_elementwise FA_EW_IFOLD)
    if (int_first && !(n[1] == std::floor(n[1]) && std::fabs(n[1]) < 0x1p63))
        return fail(FA_EINVAL, "fa_fedavg_fold: integer updates need an integral n[1] (got %g); a float "
                               "num_examples folds through fa_elementwise(FA_EW_IFOLD)", n[1]);
    if (upd_dtype == FA_F32 && agg_dtype == FA_F32) return launch_fedavg<float, float, CF32>(agg, updates, n, N, K, P, init, false, st);
    if (upd_dtype == FA_BF16 && agg_dtype == FA_F32) return launch_fedavg<bf16, float, CF32>(agg, updates, n, N, K, P, init, false, st);
    if (upd_dtype == FA_F16 && agg_dtype == FA_F16) return launch_fedavg<f16, f16, CF16>(agg, updates, n, N, K, P, init, false, st);
    if (upd_dtype == FA_F64 && agg_dtype == FA_F64) return launch_fedavg<double, double, CF64>(agg, updates, n, N, K, P, init, false, st);
    if (upd_dtype == FA_F32 && agg_dtype == FA_F64) return launch_fedavg<float, double, CF64>(agg, updates, n, N, K, P, init, false, st);
    if (upd_dtype == FA_I64 && agg_dtype == FA_F64) return launch_fedavg<int64_t, double, CF64>(agg, updates, n, N, K, P, init, int_first, st);
    if (upd_dtype == FA_I32 && agg_dtype == FA_F64) return launch_fedavg<int32_t, double, CF64>(agg, updates, n, N, K, P, init, int_first, st);
    return fail(FA_EDTYPE, "fa_fedavg_fold: unsupported dtype pair (update %d, aggregate %d)", upd_dtype, agg_dtype);
}

// A small model's whole round in one call: the fold reads the packed updates and writes the model
// straight in page-locked host memory, through their device mappings, and the call returns with the
// model on the host. For mnist-sized models the copies, events and extra launches of the device path
// cost more than the bytes (configs[0]); the kernel and client table are fa_fedavg_fold's, so the bits
// are too.
int fa_fedavg_fold_host(void* agg, int agg_dtype, const void* const* updates, int upd_dtype, const double* n,
                        const double* N, int K, int64_t P, int init, void* stream) {
    g_err[0] = 0;
    if (P < 0 || K < 0) return fail(FA_EINVAL, "fa_fedavg_fold_host: negative size (P=%lld, K=%d)", (long long)P, K);
    if (K > kMaxK) return fail(FA_EINVAL, "fa_fedavg_fold_host: K=%d exceeds one launch (%d)", K, kMaxK);
    if (K == 0 || P == 0) return FA_OK;
    if (!agg || !updates) return fail(FA_EINVAL, "fa_fedavg_fold_host: null pointer argument");
    void* dev_agg = nullptr;
    const void* dev_upd[kMaxK];
    hipError_t e = hipHostGetDevicePointer(&dev_agg, agg, 0);
    for (int k = 0; e == hipSuccess && k < K; ++k) {
        void* d = nullptr;
        if (!updates[k]) return fail(FA_EINVAL, "fa_fedavg_fold_host: updates[%d] is NULL", k);
        e = hipHostGetDevicePointer(&d, const_cast<void*>(updates[k]), 0);
        dev_upd[k] = d;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(FA_EINVAL, "fa_fedavg_fold_host: %s (not page-locked host memory?)", hipGetErrorString(e));
    }
    const int rc = fa_fedavg_fold(dev_agg, agg_dtype, dev_upd, upd_dtype, n, N, K, P, init, stream);
    if (rc != FA_OK) return rc;
    e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(FA_EHIP, "fa_fedavg_fold_host: hipStreamSynchronize: %s", hipGetErrorString(e));
    return FA_OK;
}

int fa_weighted_sum(void* acc, int acc_dtype, const void* const* updates, int upd_dtype, const double* w, int K,
                    int64_t P, void* stream) {
    g_err[0] = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (P < 0 || K < 0) return fail(FA_EINVAL, "fa_weighted_sum: negative size (P=%lld, K=%d)", (long long)P, K);
    if (K == 0 || P == 0) return FA_OK;
    if (!acc || !updates || !w) return fail(FA_EINVAL, "fa_weighted_sum: null pointer argument");
    for (int k = 0; k < K; ++k)
        if (!updates[k]) return fail(FA_EINVAL, "fa_weighted_sum: updates[%d] is NULL", k);
    // the client table's N is unused by the rule; pass w so fill_table reads valid memory
    if (upd_dtype == FA_F32 && acc_dtype == FA_F32) return launch_fedavg<float, float, CWSUM<float, float>>(acc, updates, w, w, K, P, 0, false, st);
    if (upd_dtype == FA_F32 && acc_dtype == FA_F64) return launch_fedavg<float, double, CWSUM<float, double>>(acc, updates, w, w, K, P, 0, false, st);
    if (upd_dtype == FA_F64 && acc_dtype == FA_F64) return launch_fedavg<double, double, CWSUM<double, double>>(acc, updates, w, w, K, P, 0, false, st);
    if (upd_dtype == FA_F64 && acc_dtype == FA_F32) return launch_fedavg<double, float, CWSUM<double, float>>(acc, updates, w, w, K, P, 0, false, st);
    return fail(FA_EDTYPE, "fa_weighted_sum: unsupported dtype pair (update %d, accumulator %d)", upd_dtype, acc_dtype);
}

int fa_running_mean(void* g, int dtype, const void* m, double a, double b, double T, int64_t P, void* stream) {
    g_err[0] = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (P < 0) return fail(FA_EINVAL, "fa_running_mean: negative size");
    if (P == 0) return FA_OK;
    if (!g || !m) return fail(FA_EINVAL, "fa_running_mean: null pointer argument");
    const void* ups[1] = {m};
    const double bb[1] = {b}, TT[1] = {T};
    auto run = [&](auto tag) -> int {
        using T_ = decltype(tag);
        using CP = CRUN<T_>;
        constexpr int E = 16 / (int)sizeof(T_);
        ClientTable<double> tab;
        fill_table<double>(tab, ups, bb, TT, 0, 1);
        tab.r[0] = a;                                        // a = T - n rides in r[]
        T_* x = static_cast<T_*>(g);
        if (aligned16(g) && aligned16(m)) launch_fedavg_vec<T_, T_, CP, E>(x, tab, 1, P, false, false, st);
        else launch_fedavg_geom<T_, T_, CP, 1, 1, kUnroll, false>(x, tab, 1, P, false, false, st);
        return check_launch("fa_running_mean: kernel launch");
    };
    if (dtype == FA_F32) return run(float{});
    if (dtype == FA_F64) return run(double{});
    return fail(FA_EDTYPE, "fa_running_mean: unsupported dtype %d", dtype);
}

int fa_fedopt_step(const void* old, int old_dtype, const void* const* updates, int upd_dtype, const double* n,
                   const double* N, int K, void* pg, int flags, const void* m_in, int m_in_dtype, void* m_out,
                   const double* v_in, double* v_out, double* out, int serveropt, double lr, double beta1,
                   double beta2, double tau, int64_t P, void* stream) {
    // the reference's dtype flow: m as numpy promotes it, v and the model float64
    int pg_dt = (upd_dtype == FA_I32 || upd_dtype == FA_I64) ? FA_F64 : fa_promote(upd_dtype, old_dtype);
    const int m_out_dt = fa_promote(m_in ? m_in_dtype : FA_NONE, pg_dt);
    return fa_fedopt_step_ex(old, old_dtype, updates, upd_dtype, n, N, K, pg, flags, m_in, m_in_dtype, m_out,
                             m_out_dt, v_in, FA_F64, v_out, out, FA_F64, serveropt, lr, beta1, beta2, tau, P, stream);
}

int fa_fedopt_step_ex(const void* old, int old_dtype, const void* const* updates, int upd_dtype, const double* n,
                      const double* N, int K, void* pg, int flags, const void* m_in, int m_in_dtype, void* m_out,
                      int m_out_dtype, const void* v_in, int v_in_dtype, void* v_out, void* out, int state_dtype,
                      int serveropt, double lr, double beta1, double beta2, double tau, int64_t P, void* stream) {
    g_err[0] = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (P < 0 || K < 0) return fail(FA_EINVAL, "fa_fedopt_step: negative size");
    if (P == 0) return FA_OK;
    const bool first = flags & FA_PG_FIRST, final_ = flags & FA_PG_FINAL;
    if (first && K < 1) return fail(FA_EINVAL, "fa_fedopt_step: FA_PG_FIRST requires K >= 1");
    if (!old) return fail(FA_EINVAL, "fa_fedopt_step: old is NULL");
    if (K > 0 && (!updates || !n || !N)) return fail(FA_EINVAL, "fa_fedopt_step: null client table");
    for (int k = 0; k < K; ++k)
        if (!updates[k]) return fail(FA_EINVAL, "fa_fedopt_step: updates[%d] is NULL", k);
    if ((!first || !final_ || K > kMaxK) && !pg) return fail(FA_EINVAL, "fa_fedopt_step: pg workspace required");
    if (final_ && (!m_out || !v_out || !out)) return fail(FA_EINVAL, "fa_fedopt_step: null output buffer");
    if (serveropt < FA_ADAM || serveropt > FA_ADAGRAD) return fail(FA_EINVAL, "fa_fedopt_step: unsupported serveropt %d", serveropt);
    auto is_int = [](int d) { return d == FA_I32 || d == FA_I64; };
    if (old_dtype != FA_F32 && old_dtype != FA_F64 && old_dtype != FA_F16 && !is_int(old_dtype))
        return fail(FA_EDTYPE, "fa_fedopt_step: old dtype %d", old_dtype);
    if (upd_dtype != FA_F32 && upd_dtype != FA_F64 && upd_dtype != FA_BF16 && upd_dtype != FA_F16 && !is_int(upd_dtype))
        return fail(FA_EDTYPE, "fa_fedopt_step: update dtype %d", upd_dtype);
    if (is_int(old_dtype) && !is_int(upd_dtype))
        return fail(FA_EDTYPE, "fa_fedopt_step: integer global model with float updates is unsupported");
    // integer tensors: subtract = next*1.0 + old*(-1.0) turns them into float64 (numpy: int * python float)
    const int pg_dt = is_int(upd_dtype) ? FA_F64 : fa_promote(upd_dtype, old_dtype);
    if (m_in && m_in_dtype != FA_F32 && m_in_dtype != FA_F64 && m_in_dtype != FA_F16)
        return fail(FA_EDTYPE, "fa_fedopt_step: m dtype %d", m_in_dtype);
    if (!m_in) m_in_dtype = FA_NONE;
    if (state_dtype != FA_F64 && state_dtype != FA_F32)
        return fail(FA_EDTYPE, "fa_fedopt_step_ex: state dtype %d (F64: the reference's, F32: fp32 state)", state_dtype);
    if (v_in && v_in_dtype != FA_F64 && v_in_dtype != FA_F32)
        return fail(FA_EDTYPE, "fa_fedopt_step_ex: v dtype %d", v_in_dtype);
    // m as numpy promotes it; in the fp32-state mode m may instead be stored as f32 (rounded once)
    const int m_np = fa_promote(m_in_dtype, pg_dt);
    const int m_out_dt = m_out_dtype;
    if (final_ && m_out_dt != m_np && !(state_dtype == FA_F32 && m_out_dt == FA_F32))
        return fail(FA_EDTYPE, "fa_fedopt_step_ex: m_out dtype %d (numpy gives %d%s)", m_out_dt, m_np,
                    state_dtype == FA_F32 ? "; F32 in the fp32-state mode" : "");
    auto mcode = [](int d) { return d == FA_NONE ? -1 : d == FA_F64 ? 1 : d == FA_F16 ? 2 : 0; };

    OptBuffers b{old, pg, m_in, m_out, v_in, v_out, out, mcode(m_in_dtype), mcode(final_ ? m_out_dt : m_np),
                 v_in && v_in_dtype == FA_F32, state_dtype == FA_F32, state_dtype == FA_F32};
    OptScalars s;
    s.lr = lr;
    s.b1 = beta1;
    s.b2 = beta2;
    s.tau = tau;
    s.tau2 = std::pow(tau, 2.0);   // math.pow(tau, 2)
    s.c1 = 1.0 - beta1;
    s.c2 = 1.0 - beta2;
    s.nc2 = -(1.0 - beta2);
    s.b1f = (float)beta1;
    s.c1f = (float)s.c1;
    // fedopt adam: p*(1-beta2); p has the pg dtype
    s.c2f = (float)s.c2;
    s.b1h = to_half_value(beta1);
    s.c1h = to_half_value(s.c1);
    s.c2h = to_half_value(s.c2);
    s.opt = serveropt;

    if (upd_dtype == FA_F32 && old_dtype == FA_F32) return launch_fedopt<float, float, CF32>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_BF16 && old_dtype == FA_F32) return launch_fedopt<bf16, float, CF32>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_F32 && old_dtype == FA_F64) return launch_fedopt<float, double, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_F64 && old_dtype == FA_F64) return launch_fedopt<double, double, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_BF16 && old_dtype == FA_F64) return launch_fedopt<bf16, double, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_F64 && old_dtype == FA_F32) return launch_fedopt<double, float, CF64>(b, s, updates, n, N, K, P, flags, st);
    // float16 sessions (numpy's half loops for the pseudo-gradient while it is float16)
    if (upd_dtype == FA_F16 && old_dtype == FA_F16) return launch_fedopt<f16, f16, CF16>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_F16 && old_dtype == FA_F32) return launch_fedopt<f16, float, CF32>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_F16 && old_dtype == FA_F64) return launch_fedopt<f16, double, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_F32 && old_dtype == FA_F16) return launch_fedopt<float, f16, CF32>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_F64 && old_dtype == FA_F16) return launch_fedopt<double, f16, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_I64 && old_dtype == FA_I64) return launch_fedopt<int64_t, int64_t, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_I64 && old_dtype == FA_F64) return launch_fedopt<int64_t, double, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_I64 && old_dtype == FA_F32) return launch_fedopt<int64_t, float, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_I32 && old_dtype == FA_I32) return launch_fedopt<int32_t, int32_t, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_I32 && old_dtype == FA_F64) return launch_fedopt<int32_t, double, CF64>(b, s, updates, n, N, K, P, flags, st);
    if (upd_dtype == FA_I32 && old_dtype == FA_F32) return launch_fedopt<int32_t, float, CF64>(b, s, updates, n, N, K, P, flags, st);
    return fail(FA_EDTYPE, "fa_fedopt_step: unsupported dtype pair (update %d, old %d)", upd_dtype, old_dtype);
}

// A small model's whole FedOpt round in one call (the FedOpt form of fa_fedavg_fold_host): the global
// model, the packed updates and the new model in page-locked host memory, read and written through
// their device mappings; m / v in HBM. One FIRST | FINAL launch (the pseudo-gradient in registers,
// then the server step), then the stream wait.
int fa_fedopt_step_host(const void* old, int old_dtype, const void* const* updates, int upd_dtype, const double* n,
                        const double* N, int K, const void* m_in, int m_in_dtype, void* m_out, int m_out_dtype,
                        const void* v_in, int v_in_dtype, void* v_out, void* out, int state_dtype, int serveropt,
                        double lr, double beta1, double beta2, double tau, int64_t P, void* stream) {
    g_err[0] = 0;
    if (P < 0 || K < 1 || K > kMaxK)
        return fail(FA_EINVAL, "fa_fedopt_step_host: 1 <= K <= %d updates in one launch (K=%d, P=%lld)", kMaxK, K,
                    (long long)P);
    if (P == 0) return FA_OK;
    if (!old || !updates || !out) return fail(FA_EINVAL, "fa_fedopt_step_host: null pointer argument");
    void* dev_old = nullptr;
    void* dev_out = nullptr;
    const void* dev_upd[kMaxK];
    hipError_t e = hipHostGetDevicePointer(&dev_old, const_cast<void*>(old), 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dev_out, out, 0);
    for (int k = 0; e == hipSuccess && k < K; ++k) {
        void* d = nullptr;
        if (!updates[k]) return fail(FA_EINVAL, "fa_fedopt_step_host: updates[%d] is NULL", k);
        e = hipHostGetDevicePointer(&d, const_cast<void*>(updates[k]), 0);
        dev_upd[k] = d;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(FA_EINVAL, "fa_fedopt_step_host: %s (not page-locked host memory?)", hipGetErrorString(e));
    }
    const int rc = fa_fedopt_step_ex(dev_old, old_dtype, dev_upd, upd_dtype, n, N, K, nullptr, FA_PG_FIRST | FA_PG_FINAL,
                                     m_in, m_in_dtype, m_out, m_out_dtype, v_in, v_in_dtype, v_out, dev_out, state_dtype,
                                     serveropt, lr, beta1, beta2, tau, P, stream);
    if (rc != FA_OK) return rc;
    e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(FA_EHIP, "fa_fedopt_step_host: hipStreamSynchronize: %s", hipGetErrorString(e));
    return FA_OK;
}

int fa_elementwise(int op, void* out, int out_dtype, const void* x, int x_dtype, const void* y, int y_dtype,
                   double a, double b, int64_t P, void* stream) {
    g_err[0] = 0;
    if (P < 0 || !out || (op != FA_EW_FILL && !x)) return fail(FA_EINVAL, "fa_elementwise: bad arguments");
    if (op < FA_EW_AXPBY || op > FA_EW_NFOLD) return fail(FA_EINVAL, "fa_elementwise: unknown op %d", op);
    if (op == FA_EW_AXPBY && !y) return fail(FA_EINVAL, "fa_elementwise: AXPBY needs y");
    if (P == 0) return FA_OK;
    if (op == FA_EW_IPOW) {
        if (out_dtype != x_dtype)
            return fail(FA_EDTYPE, "fa_elementwise: IPOW returns its input's dtype");
        if (!(a >= 0.0) || a != std::floor(a) || a > 0x1p63)
            return fail(FA_EINVAL, "fa_elementwise: IPOW exponent must be a non-negative integer");
        const dim3 g((unsigned)std::min<int64_t>((P + kBlock - 1) / kBlock, 8192));
        hipStream_t sti = static_cast<hipStream_t>(stream);
        auto run = [&](auto tag) -> int {
            using T = decltype(tag);
            hipLaunchKernelGGL(k_ipow<T>, g, dim3(kBlock), 0, sti, static_cast<T*>(out), static_cast<const T*>(x),
                               (uint64_t)a, P);
            return check_launch("fa_elementwise");
        };
        switch (x_dtype) {
            case FA_I8: return run(int8_t{});
            case FA_I16: return run(int16_t{});
            case FA_I32: return run(int32_t{});
            case FA_I64: return run(int64_t{});
            case FA_U8: return run(uint8_t{});
            case FA_U16: return run(uint16_t{});
            case FA_U32: return run(uint32_t{});
            case FA_U64: return run(uint64_t{});
            default: return fail(FA_EDTYPE, "fa_elementwise: IPOW takes an integer array, got dtype %d", x_dtype);
        }
    }
    if (op == FA_EW_IFOLD || op == FA_EW_NFOLD) {
        if (!y || out_dtype != FA_F64 || x_dtype != y_dtype)
            return fail(FA_EDTYPE, "fa_elementwise: IFOLD / NFOLD take two arrays of one integer dtype and return float64");
        if (op == FA_EW_NFOLD && !(std::fabs(a) < 0x1p53 && a == std::floor(a)))
            return fail(FA_EINVAL, "fa_elementwise: NFOLD num_examples must be an integer below 2^53 in magnitude");
        const dim3 g((unsigned)std::min<int64_t>((P + kBlock - 1) / kBlock, 8192));
        hipStream_t sti = static_cast<hipStream_t>(stream);
        auto run = [&](auto tag) -> int {
            using T = decltype(tag);
            using U = typename std::make_unsigned<T>::type;
            if (op == FA_EW_IFOLD)
                hipLaunchKernelGGL(k_ifold<T>, g, dim3(kBlock), 0, sti, static_cast<double*>(out),
                                   static_cast<const T*>(x), static_cast<const T*>(y), a, b, P);
            else
                hipLaunchKernelGGL(k_nfold<T>, g, dim3(kBlock), 0, sti, static_cast<double*>(out),
                                   static_cast<const T*>(x), static_cast<const T*>(y), (T)(U)(int64_t)a, b, P);
            return check_launch("fa_elementwise");
        };
        switch (x_dtype) {
            case FA_I8: return run(int8_t{});
            case FA_I16: return run(int16_t{});
            case FA_I32: return run(int32_t{});
            case FA_I64: return run(int64_t{});
            case FA_U8: return run(uint8_t{});
            case FA_U16: return run(uint16_t{});
            case FA_U32: return run(uint32_t{});
            case FA_U64: return run(uint64_t{});
            default: return fail(FA_EDTYPE, "fa_elementwise: IFOLD / NFOLD need an integer dtype, got %d", x_dtype);
        }
    }
    if (op == FA_EW_AXPBY && x_dtype == FA_F16 && y_dtype == FA_F16 && out_dtype == FA_F16) {
        const dim3 g((unsigned)std::min<int64_t>((P + kBlock - 1) / kBlock, 8192));
        hipLaunchKernelGGL(k_axpby_half, g, dim3(kBlock), 0, static_cast<hipStream_t>(stream), static_cast<f16*>(out),
                           static_cast<const f16*>(x), static_cast<const f16*>(y), to_half_value(a), to_half_value(b), P);
        return check_launch("fa_elementwise");
    }
    auto isf = [](int d) { return d == FA_F32 || d == FA_F64; };
    if (op == FA_EW_FILL) x_dtype = out_dtype;
    if (!y) y_dtype = x_dtype;
    if (!isf(out_dtype) || !isf(x_dtype) || !isf(y_dtype)) return fail(FA_EDTYPE, "fa_elementwise: f32/f64 only");
    const int want = (op == FA_EW_FILL) ? out_dtype
                     : (op == FA_EW_AXPBY || ((op == FA_EW_MUL || op == FA_EW_DIV) && y)) ? fa_promote(x_dtype, y_dtype)
                     : x_dtype;
    if (out_dtype != want) return fail(FA_EDTYPE, "fa_elementwise: output dtype must be %d", want);
    const dim3 grid((unsigned)std::min<int64_t>((P + kBlock - 1) / kBlock, 8192));
    hipStream_t st = static_cast<hipStream_t>(stream);
#define FA_EW(TX, TY, TO) \
    hipLaunchKernelGGL((k_elementwise<TX, TY, TO>), grid, dim3(kBlock), 0, st, op, static_cast<TO*>(out), \
                       static_cast<const TX*>(x), static_cast<const TY*>(y), a, b, P)
    const bool x32 = x_dtype == FA_F32, y32 = y_dtype == FA_F32, o32 = out_dtype == FA_F32;
    if (x32 && y32 && o32) FA_EW(float, float, float);
    else if (x32 && y32) FA_EW(float, float, double);
    else if (x32) FA_EW(float, double, double);
    else if (y32) FA_EW(double, float, double);
    else FA_EW(double, double, double);
#undef FA_EW
    return check_launch("fa_elementwise");
}

int64_t fa_norm1_work(int64_t rows, int64_t cols, int matrix) {
    return matrix ? std::max<int64_t>(cols, 1) : kNormBlocks;
}

int fa_norm1(double* out, const void* x, int dtype, int64_t rows, int64_t cols, int matrix, double* work,
             void* stream) {
    g_err[0] = 0;
    if (!out || !work || rows < 0 || cols < 0 || (rows * cols > 0 && !x)) return fail(FA_EINVAL, "fa_norm1: bad arguments");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t P = rows * cols;
    auto run = [&](auto tag) -> int {
        using T = decltype(tag);
        const T* xp = static_cast<const T*>(x);
        if (matrix) {
            if (cols > 0)
                hipLaunchKernelGGL(k_colabssum<T>, dim3((unsigned)std::min<int64_t>((cols + kBlock - 1) / kBlock, 4096)),
                                   dim3(kBlock), 0, st, xp, rows, cols, work);
            hipLaunchKernelGGL(k_final_reduce, dim3(1), dim3(kBlock), 0, st, work, cols, 1, out);
        } else {
            hipLaunchKernelGGL(k_abssum_partial<T>, dim3(kNormBlocks), dim3(kBlock), 0, st, xp, P, work);
            hipLaunchKernelGGL(k_final_reduce, dim3(1), dim3(kBlock), 0, st, work, (int64_t)kNormBlocks, 0, out);
        }
        return check_launch("fa_norm1");
    };
    switch (dtype) {
        case FA_F32: return run(float{});
        case FA_F64: return run(double{});
        case FA_I32: return run(int32_t{});
        case FA_I64: return run(int64_t{});
        case FA_I8: return run(int8_t{});
        case FA_I16: return run(int16_t{});
        case FA_U8: return run(uint8_t{});
        case FA_U16: return run(uint16_t{});
        case FA_U32: return run(uint32_t{});
        case FA_U64: return run(uint64_t{});
        default: return fail(FA_EDTYPE, "fa_norm1: dtype %d", dtype);
    }
}

int fa_cast(void* out, int out_dtype, const void* in, int in_dtype, int ndim, const int64_t* out_shape,
            const int64_t* in_strides, void* stream) {
    g_err[0] = 0;
    if (!out_shape || !in_strides) return fail(FA_EINVAL, "fa_cast: null shape or strides");
    if (ndim < 1 || ndim > kCastMaxDim) return fail(FA_EINVAL, "fa_cast: ndim must be 1..%d, got %d", kCastMaxDim, ndim);
    CastGeom g;
    g.ndim = ndim;
    int64_t P = 1, cstride = 1;
    bool bc = false;
    for (int d = ndim - 1; d >= 0; --d) {
        if (out_shape[d] < 0) return fail(FA_EINVAL, "fa_cast: negative dimension");
        g.shape[d] = out_shape[d];
        g.stride[d] = in_strides[d];
        if (out_shape[d] != 1 && in_strides[d] != cstride) bc = true;   // not the contiguous identity map
        cstride *= out_shape[d];
    }
    for (int d = 0; d < ndim; ++d) P *= out_shape[d];
    if (P == 0) return FA_OK;
    if (!out || !in) return fail(FA_EINVAL, "fa_cast: null buffer");
    const dim3 grid((unsigned)std::min<int64_t>((P + kBlock - 1) / kBlock, 16384));
    hipStream_t st = static_cast<hipStream_t>(stream);
#define FA_CAST(DI, TI, DO, TO)                                                                                     \
    if (in_dtype == DI && out_dtype == DO) {                                                                        \
        if (bc) hipLaunchKernelGGL((k_cast<TI, TO, true>), grid, dim3(kBlock), 0, st, static_cast<TO*>(out),        \
                                   static_cast<const TI*>(in), g, P);                                                \
        else hipLaunchKernelGGL((k_cast<TI, TO, false>), grid, dim3(kBlock), 0, st, static_cast<TO*>(out),          \
                                static_cast<const TI*>(in), g, P);                                                   \
        return check_launch("fa_cast");                                                                             \
    }
    FA_CAST(FA_F32, float, FA_F32, float)
    FA_CAST(FA_F64, double, FA_F64, double)
    FA_CAST(FA_F32, float, FA_F16, f16)      // narrowing float casts (numpy astype: round to nearest even):
    FA_CAST(FA_F64, double, FA_F32, float)   // the result of a float16 / float32 helper op computed wider
    FA_CAST(FA_F16, f16, FA_F16, f16)
    FA_CAST(FA_BF16, bf16, FA_BF16, bf16)
    FA_CAST(FA_I32, int32_t, FA_I32, int32_t)
    FA_CAST(FA_I64, int64_t, FA_I64, int64_t)
    FA_CAST(FA_F16, f16, FA_F32, float)
    FA_CAST(FA_F16, f16, FA_F64, double)
    FA_CAST(FA_BF16, bf16, FA_F32, float)
    FA_CAST(FA_BF16, bf16, FA_F64, double)
    FA_CAST(FA_F32, float, FA_F64, double)
    FA_CAST(FA_I32, int32_t, FA_I64, int64_t)
    FA_CAST(FA_I32, int32_t, FA_F64, double)
    FA_CAST(FA_I64, int64_t, FA_F64, double)
    // narrow / unsigned integers: identity (broadcast) and numpy's safe widenings
    FA_CAST(FA_I8, int8_t, FA_I8, int8_t)
    FA_CAST(FA_I8, int8_t, FA_I16, int16_t)
    FA_CAST(FA_I8, int8_t, FA_I32, int32_t)
    FA_CAST(FA_I8, int8_t, FA_I64, int64_t)
    FA_CAST(FA_I8, int8_t, FA_F16, f16)
    FA_CAST(FA_I8, int8_t, FA_F32, float)
    FA_CAST(FA_I8, int8_t, FA_F64, double)
    FA_CAST(FA_U8, uint8_t, FA_U8, uint8_t)
    FA_CAST(FA_U8, uint8_t, FA_I16, int16_t)
    FA_CAST(FA_U8, uint8_t, FA_U16, uint16_t)
    FA_CAST(FA_U8, uint8_t, FA_I32, int32_t)
    FA_CAST(FA_U8, uint8_t, FA_U32, uint32_t)
    FA_CAST(FA_U8, uint8_t, FA_I64, int64_t)
    FA_CAST(FA_U8, uint8_t, FA_U64, uint64_t)
    FA_CAST(FA_U8, uint8_t, FA_F16, f16)
    FA_CAST(FA_U8, uint8_t, FA_F32, float)
    FA_CAST(FA_U8, uint8_t, FA_F64, double)
    FA_CAST(FA_I16, int16_t, FA_I16, int16_t)
    FA_CAST(FA_I16, int16_t, FA_I32, int32_t)
    FA_CAST(FA_I16, int16_t, FA_I64, int64_t)
    FA_CAST(FA_I16, int16_t, FA_F32, float)
    FA_CAST(FA_I16, int16_t, FA_F64, double)
    FA_CAST(FA_U16, uint16_t, FA_U16, uint16_t)
    FA_CAST(FA_U16, uint16_t, FA_I32, int32_t)
    FA_CAST(FA_U16, uint16_t, FA_U32, uint32_t)
    FA_CAST(FA_U16, uint16_t, FA_I64, int64_t)
    FA_CAST(FA_U16, uint16_t, FA_U64, uint64_t)
    FA_CAST(FA_U16, uint16_t, FA_F32, float)
    FA_CAST(FA_U16, uint16_t, FA_F64, double)
    FA_CAST(FA_U32, uint32_t, FA_U32, uint32_t)
    FA_CAST(FA_U32, uint32_t, FA_I64, int64_t)
    FA_CAST(FA_U32, uint32_t, FA_U64, uint64_t)
    FA_CAST(FA_U32, uint32_t, FA_F64, double)
    FA_CAST(FA_U64, uint64_t, FA_U64, uint64_t)
    FA_CAST(FA_U64, uint64_t, FA_F64, double)
#undef FA_CAST
    return fail(FA_EDTYPE, "fa_cast: unsupported conversion %d -> %d", in_dtype, out_dtype);
}

// ----------------------------------------------------------------------------
// peer transport of the parameter-sliced all-gather (sharded.P2PAllGather,
// multidev.allgather_devices): IPC mappings of the peers' model buffers and DMA copies into them
// ----------------------------------------------------------------------------
static_assert(sizeof(hipIpcMemHandle_t) <= FA_IPC_HANDLE_BYTES, "IPC handle size");

int fa_ipc_get_handle(const void* dptr, void* handle, uint64_t* offset) {
    g_err[0] = 0;
    if (!dptr || !handle || !offset) return fail(FA_EINVAL, "fa_ipc_get_handle: null argument");
    // a handle names a whole allocation (a caching allocator hands out pieces of one): export the
    // allocation's base and the piece's offset in it
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(dptr));
    if (e != hipSuccess) return fail(FA_EHIP, "fa_ipc_get_handle: hipMemGetAddressRange: %s", hipGetErrorString(e));
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, base);
    if (e != hipSuccess) return fail(FA_EHIP, "fa_ipc_get_handle: hipIpcGetMemHandle: %s", hipGetErrorString(e));
    std::memset(handle, 0, FA_IPC_HANDLE_BYTES);
    std::memcpy(handle, &h, sizeof(h));
    *offset = (uint64_t)(static_cast<const char*>(dptr) - static_cast<const char*>(base));
    return FA_OK;
}

int fa_ipc_open(const void* handle, uint64_t offset, void** base, void** dptr) {
    g_err[0] = 0;
    if (!handle || !base || !dptr) return fail(FA_EINVAL, "fa_ipc_open: null argument");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    void* b = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return fail(FA_EHIP, "fa_ipc_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
    *base = b;
    *dptr = static_cast<char*>(b) + offset;
    return FA_OK;
}

int fa_ipc_close(void* base) {
    g_err[0] = 0;
    if (!base) return FA_OK;
    hipError_t e = hipIpcCloseMemHandle(base);
    if (e != hipSuccess) return fail(FA_EHIP, "fa_ipc_close: %s", hipGetErrorString(e));
    return FA_OK;
}

int fa_copy_async(void* dst, const void* src, int64_t bytes, void* stream) {
    g_err[0] = 0;
    if (bytes < 0 || (bytes > 0 && (!dst || !src))) return fail(FA_EINVAL, "fa_copy_async: bad arguments");
    if (bytes == 0) return FA_OK;
    hipError_t e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(FA_EHIP, "fa_copy_async: %s", hipGetErrorString(e));
    return FA_OK;
}

int fa_fedavg_fold_push(float* agg, const void* const* updates, const double* n, const double* N, int K, int64_t P,
                        int init, void* const* dsts, int ndst, uint32_t* release_rec, void* stream) {
    g_err[0] = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (P < 0 || K < 0 || ndst < 0 || ndst > kPushMax)
        return fail(FA_EINVAL, "fa_fedavg_fold_push: bad sizes (P=%lld, K=%d, ndst=%d <= %d)", (long long)P, K, ndst,
                    kPushMax);
    if (init && K < 1) return fail(FA_EINVAL, "fa_fedavg_fold_push: init requires K >= 1");
    if (K == 0 || P == 0) return FA_OK;
    if (!agg || !updates || !n || !N || (ndst > 0 && !dsts)) return fail(FA_EINVAL, "fa_fedavg_fold_push: null pointer argument");
    if (!aligned16(agg)) return fail(FA_EINVAL, "fa_fedavg_fold_push: agg not 16-B aligned");
    PushTable t{};
    for (int d = 0; d < ndst; ++d) {
        if (!dsts[d] || !aligned16(dsts[d])) return fail(FA_EINVAL, "fa_fedavg_fold_push: destination %d null or not 16-B aligned", d);
        t.dst[d] = static_cast<u32x4*>(dsts[d]);
    }
    for (int k = 0; k < K; ++k)
        if (!updates[k] || !aligned16(updates[k])) return fail(FA_EINVAL, "fa_fedavg_fold_push: updates[%d] null or not 16-B aligned", k);
    // clients beyond one kernarg table fold first (plain launches); the last table's launch pushes
    const int last0 = ((K - 1) / kMaxK) * kMaxK;
    if (last0 > 0) {
        const int rc = fa_fedavg_fold(agg, FA_F32, updates, FA_F32, n, N, last0, P, init, stream);
        if (rc) return rc;
    }
    ClientTable<CF32::S> tab;
    const int cnt = K - last0;
    fill_table<CF32::S>(tab, updates, n, N, last0, cnt);
    const bool first = init && last0 == 0;
    const dim3 grid((unsigned)((P + 4 * (int64_t)kBlock - 1) / (4 * (int64_t)kBlock)));
    if (cnt <= 8) {
        if (first) hipLaunchKernelGGL((k_fedavg_push<8, true>), grid, dim3(kBlock), 0, st, agg, tab, cnt, P, t, ndst);
        else hipLaunchKernelGGL((k_fedavg_push<8, false>), grid, dim3(kBlock), 0, st, agg, tab, cnt, P, t, ndst);
    } else {
        if (first) hipLaunchKernelGGL((k_fedavg_push<4, true>), grid, dim3(kBlock), 0, st, agg, tab, cnt, P, t, ndst);
        else hipLaunchKernelGGL((k_fedavg_push<4, false>), grid, dim3(kBlock), 0, st, agg, tab, cnt, P, t, ndst);
    }
    const int rc = check_launch("fa_fedavg_fold_push: kernel launch");
    return rc ? rc : (ndst > 0 ? launch_release(st, release_rec) : FA_OK);
}

int fa_push(void* const* dsts, int ndst, const void* src, int64_t bytes, uint32_t* release_rec, void* stream) {
    g_err[0] = 0;
    if (ndst < 0 || ndst > kPushMax || bytes < 0 || (bytes > 0 && (!src || (ndst > 0 && !dsts))))
        return fail(FA_EINVAL, "fa_push: bad arguments (at most %d destinations)", kPushMax);
    if (bytes == 0 || ndst == 0) return FA_OK;
    PushTable t{};
    for (int d = 0; d < ndst; ++d) {
        if (!dsts[d]) return fail(FA_EINVAL, "fa_push: destination %d is null", d);
        if (reinterpret_cast<uintptr_t>(dsts[d]) % 16) return fail(FA_EINVAL, "fa_push: destination %d not 16-B aligned", d);
        t.dst[d] = static_cast<u32x4*>(dsts[d]);
    }
    if (reinterpret_cast<uintptr_t>(src) % 16) return fail(FA_EINVAL, "fa_push: source not 16-B aligned");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t n16 = bytes / 16;
    const int rem = (int)(bytes % 16);
    if (n16 > 0) {
        // link-bound, not HBM-bound: a few hundred workgroups keep every link's writes in flight and
        // leave most of the chip to the fold running beside it
        const int64_t need = (n16 + (int64_t)kBlock * kPushWords - 1) / ((int64_t)kBlock * kPushWords);
        const int grid = (int)std::min<int64_t>(need, 512);
        hipLaunchKernelGGL(k_push, dim3(grid), dim3(kBlock), 0, st, t, ndst, static_cast<const u32x4*>(src), n16);
    }
    if (rem > 0)
        hipLaunchKernelGGL(k_push_tail, dim3(1), dim3(64), 0, st, t, ndst, static_cast<const uint8_t*>(src), n16 * 16,
                           rem);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FA_EHIP, "fa_push: %s", hipGetErrorString(e));
    return launch_release(st, release_rec);
}

int fa_device_xccs(int dev, int* n) {
    g_err[0] = 0;
    if (!n) return fail(FA_EINVAL, "fa_device_xccs: null argument");
    return device_xccs(dev, n);
}

int fa_host_device_ptr(const void* host, void** dptr) {
    g_err[0] = 0;
    if (!host || !dptr) return fail(FA_EINVAL, "fa_host_device_ptr: null argument");
    void* d = nullptr;
    hipError_t e = hipHostGetDevicePointer(&d, const_cast<void*>(host), 0);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(FA_EHIP, "fa_host_device_ptr: %s (not page-locked host memory?)", hipGetErrorString(e));
    }
    *dptr = d;
    return FA_OK;
}

int fa_host_register(void* p, int64_t bytes) {
    g_err[0] = 0;
    if (!p || bytes <= 0) return fail(FA_EINVAL, "fa_host_register: bad arguments");
    hipError_t e = hipHostRegister(p, (size_t)bytes, hipHostRegisterPortable);
    if (e != hipSuccess) return fail(FA_EHIP, "fa_host_register: %s", hipGetErrorString(e));
    return FA_OK;
}

int fa_host_unregister(void* p) {
    g_err[0] = 0;
    if (!p) return FA_OK;
    hipError_t e = hipHostUnregister(p);
    if (e != hipSuccess) return fail(FA_EHIP, "fa_host_unregister: %s", hipGetErrorString(e));
    return FA_OK;
}

int fa_peer_enable(int dev, int peer) {
    g_err[0] = 0;
    if (dev == peer) return FA_OK;
    int can = 0;
    hipError_t e = hipDeviceCanAccessPeer(&can, dev, peer);
    if (e != hipSuccess) return fail(FA_EHIP, "fa_peer_enable: hipDeviceCanAccessPeer: %s", hipGetErrorString(e));
    if (!can) return fail(FA_EHIP, "fa_peer_enable: device %d cannot access device %d", dev, peer);
    int cur = 0;
    (void)hipGetDevice(&cur);
    e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipDeviceEnablePeerAccess(peer, 0);
    (void)hipSetDevice(cur);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        return FA_OK;
    }
    if (e != hipSuccess) return fail(FA_EHIP, "fa_peer_enable(%d -> %d): %s", dev, peer, hipGetErrorString(e));
    return FA_OK;
}

#ifdef FEDAGG_PROBES
int fa_tune(int knob, int value) {
    g_err[0] = 0;
    switch (knob) {
        case FA_TUNE_STRIPS:
            if (value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
                return fail(FA_EINVAL, "fa_tune: strips must be 1, 2, 4, 8 or 16");
            g_cfg.strips = value;
            return FA_OK;
        case FA_TUNE_UNROLL:
            if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
                return fail(FA_EINVAL, "fa_tune: unroll must be 0 (pipelined), 1, 2, 4, 8 or 16");
            g_cfg.unroll = value;
            return FA_OK;
        case FA_TUNE_NT:
            g_cfg.nt = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_SUM_NOSTORE:
            g_cfg.sum_nostore = value != 0;
            return FA_OK;
        case FA_TUNE_NT_STORE:
            if (value < 0 || value > 2) return fail(FA_EINVAL, "fa_tune: store mode 0 (plain), 1 (nt) or 2 (sc1)");
            g_cfg.nt_store = value;
            return FA_OK;
        case FA_TUNE_BLOCK:
            if (value != 256 && value != 512 && value != 1024) return fail(FA_EINVAL, "fa_tune: block 256, 512 or 1024");
            g_cfg.block_log = value == 256 ? 8 : value == 512 ? 9 : 10;
            return FA_OK;
        case FA_TUNE_READ:
            if (value != 4 && value != 8 && value != 16) return fail(FA_EINVAL, "fa_tune: read probe depth 4, 8 or 16");
            g_cfg.read_per_lane = value;
            return FA_OK;
        case FA_TUNE_GRID:
            if (value < 0 || value > 64) return fail(FA_EINVAL, "fa_tune: grid blocks per CU must be 0..64");
            g_cfg.grid_per_cu = value;
            return FA_OK;
        case FA_TUNE_TILEMAP:
            if (value != 0 && value != 2 && value != 4 && value != 8 && value != 16 && value != 32)
                return fail(FA_EINVAL, "fa_tune: tile map 0 (identity) or runs of 2, 4, 8, 16, 32 tiles per XCD");
            g_cfg.tilemap = value;
            return FA_OK;
        case FA_TUNE_LANETAB:
            g_cfg.lanetab = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_FASTDIV:
            g_cfg.fastdiv = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_FASTDIV64:
            g_cfg.fastdiv64 = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_OPT_NT:
            g_cfg.opt_nt = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_OPT_NOSTORE:
            g_cfg.opt_nostore = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_OPT_COAL:
            if (value < 0 || value > 2)
                return fail(FA_EINVAL, "fa_tune: FedOpt map 0 (strip), 1 (coalesced, 2 pairs/lane), 2 (4 pairs/lane: product)");
            g_cfg.opt_coal = value;
            return FA_OK;
        case FA_TUNE_OPT_STORE:
            if (value < 0 || value > 2) return fail(FA_EINVAL, "fa_tune: FedOpt store mode 0 (plain), 1 (nt) or 2 (sc1)");
            g_cfg.opt_store = value;
            return FA_OK;
        case FA_TUNE_NARROW:
            g_cfg.narrow = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_LDS:
            if (value < 0 || value > 64) return fail(FA_EINVAL, "fa_tune: occupancy-probe LDS 0..64 KiB per workgroup");
            g_cfg.lds_kib = value;
            return FA_OK;
        case FA_TUNE_AUTO_GEOM:
            g_cfg.auto_geom = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_OPT_MV:
            g_cfg.opt_mv = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_OPT_MIX:
            g_cfg.opt_mix = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_OPT_G:
            if (value != 0 && value != 1 && value != 2 && value != 4)
                return fail(FA_EINVAL, "fa_tune: burst-store product probe 0 (off), 1, 2 or 4 tiles per wave");
            g_cfg.opt_g = value;
            return FA_OK;
        case FA_TUNE_OPT_WIN_PERIOD:
            if (value != 0 && value != -1 && (value < 64 || value > (1 << 24)))
                return fail(FA_EINVAL, "fa_tune: store-window period 64 .. 2^24 ticks of 10 ns (0 = the product's own, -1 = none)");
            g_cfg.opt_win_period = value;
            return FA_OK;
        case FA_TUNE_OPT_WIN_W:
            if (value < 0) return fail(FA_EINVAL, "fa_tune: store-window length in ticks >= 0");
            g_cfg.opt_win_w = value;
            return FA_OK;
        case FA_TUNE_OPT_WIN_MODE:
            if (value < 0 || value > 2) return fail(FA_EINVAL, "fa_tune: store-window mode 0, 1 or 2");
            g_cfg.opt_win_mode = value;
            return FA_OK;
        case FA_TUNE_OPT_WIN_PROD:
            if (value < 0 || value > 3)
                return fail(FA_EINVAL, "fa_tune: OPT_WIN_PROD 0 (pattern probe), 1 (k_fedopt_cw), 2 (k_fedopt_cgw), 3 (k_fedopt_cw2)");
            g_cfg.opt_win_prod = value;
            return FA_OK;
        case FA_TUNE_OPT_QUAD:
            g_cfg.opt_quad = value ? 1 : 0;
            return FA_OK;
        case FA_TUNE_AVG_WIN_PERIOD:
            if (value != 0 && value != -1 && (value < 64 || value > (1 << 24)))
                return fail(FA_EINVAL, "fa_tune: store-window period 64 .. 2^24 ticks of 10 ns (0 = the product's own, -1 = none)");
            g_cfg.avg_win_period = value;
            return FA_OK;
        case FA_TUNE_AVG_WIN_W:
            if (value < 0) return fail(FA_EINVAL, "fa_tune: store-window length in ticks >= 0");
            g_cfg.avg_win_w = value;
            return FA_OK;
        case FA_TUNE_AVG_WIN_MODE:
            if (value < 0 || value > 2) return fail(FA_EINVAL, "fa_tune: store-window mode 0, 1 or 2");
            g_cfg.avg_win_mode = value;
            return FA_OK;
        case FA_TUNE_OPT_BURST:
            if (value != 0 && value != 1 && value != 2 && value != 4)
                return fail(FA_EINVAL, "fa_tune: burst-store probe 0 (off), 1, 2 or 4 tiles per wave");
            g_cfg.opt_burst = value;
            return FA_OK;
        case FA_TUNE_WPE:
            if (value != 0 && value != 5 && value != 6 && value != 7 && value != 8)
                return fail(FA_EINVAL, "fa_tune: waves per SIMD 0 (compiler's choice), 5, 6, 7 or 8");
            g_cfg.wpe = value;
            return FA_OK;
        default:
            return fail(FA_EINVAL, "fa_tune: unknown knob %d", knob);
    }
}

int fa_stream_sum(float* out, const float* const* bufs, int K, int64_t P, void* stream) {
    g_err[0] = 0;
    if (K < 1 || K > kMaxK || P < 0 || !out || !bufs) return fail(FA_EINVAL, "fa_stream_sum: bad arguments");
    bool vec = aligned16(out);
    for (int k = 0; k < K; ++k) vec = vec && bufs[k] && aligned16(bufs[k]);
    if (!vec) return fail(FA_EINVAL, "fa_stream_sum: buffers must be 16-B aligned");
    ClientTable<float> tab;
    std::vector<double> ones(K, 1.0);
    fill_table<float>(tab, reinterpret_cast<const void* const*>(bufs), ones.data(), ones.data(), 0, K);
    if (g_cfg.sum_nostore)
        launch_fedavg_pipe<float, float, CADDNW, 4, 4, false, false>(out, tab, K, P, true, false, static_cast<hipStream_t>(stream));
    else if (g_cfg.nt_store == 1)
        launch_fedavg_pipe<float, float, CADD, 4, 4, false, false, kBlock, 1>(out, tab, K, P, true, false, static_cast<hipStream_t>(stream));
    else if (g_cfg.nt_store == 2)
        launch_fedavg_pipe<float, float, CADD, 4, 4, false, false, kBlock, 2>(out, tab, K, P, true, false, static_cast<hipStream_t>(stream));
    else
        launch_fedavg_pipe<float, float, CADD, 4, 4, false, false>(out, tab, K, P, true, false, static_cast<hipStream_t>(stream));
    return check_launch("fa_stream_sum");
}

int fa_stream_copy(void* dst, const void* src, int64_t bytes, void* stream) {
    g_err[0] = 0;
    if (bytes < 0 || (bytes & 15) || !aligned16(dst) || !aligned16(src))
        return fail(FA_EINVAL, "fa_stream_copy: bytes must be a multiple of 16 and buffers 16-B aligned");
    const int64_t n16 = bytes / 16;
    if (!n16) return FA_OK;
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)((n16 + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), static_cast<u32x4*>(dst), static_cast<const u32x4*>(src), n16);
    return check_launch("fa_stream_copy");
}

int64_t fa_stream_read_blocks(int64_t bytes) {
    const int64_t n16 = bytes / 16;
    const int64_t per = (int64_t)kBlock * kReadPerLane;
    return (n16 + per - 1) / per;
}

int fa_stream_read(const void* src, int64_t bytes, void* sink, void* stream) {
    g_err[0] = 0;
    if (bytes < 0 || (bytes & 15) || !aligned16(src) || !aligned16(sink))
        return fail(FA_EINVAL, "fa_stream_read: bytes must be a multiple of 16 and buffers 16-B aligned");
    const int64_t blocks = fa_stream_read_blocks(bytes);
    if (!blocks) return FA_OK;
    const int64_t n16 = bytes / 16;
    const dim3 blk(kBlock);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const u32x4* s4 = static_cast<const u32x4*>(src);
    u32x4* k4 = static_cast<u32x4*>(sink);
    // loads in flight per lane (fa_tune FA_TUNE_UNROLL reused for this probe: 4, 8 or 16)
    switch (g_cfg.read_per_lane) {
        case 4: hipLaunchKernelGGL(k_stream_read<4>, dim3((unsigned)((n16 + kBlock * 4 - 1) / (kBlock * 4))), blk, 0, st, s4, n16, k4); break;
        case 8: hipLaunchKernelGGL(k_stream_read<8>, dim3((unsigned)((n16 + kBlock * 8 - 1) / (kBlock * 8))), blk, 0, st, s4, n16, k4); break;
        default: hipLaunchKernelGGL(k_stream_read<16>, dim3((unsigned)blocks), blk, 0, st, s4, n16, k4); break;
    }
    return check_launch("fa_stream_read");
}

#endif  // FEDAGG_PROBES

}  // extern "C"
