/*
 * fedagg.h — C ABI of the MI355X (gfx950) aggregation library `libfedagg.so`.
 *
 * This is the drop-in boundary for FEDn's combiner-side aggregation hot path
 * (SURVEY.md §8(b)). Every entry point takes plain pointers, sizes and a
 * hipStream_t passed as `void*`; no torch or numpy types cross it. Buffers are
 * owned by the caller (device memory, e.g. PyTorch-ROCm tensors); the library
 * allocates nothing persistent. Every function returns 0 on success or a
 * positive FA_E* status; `fa_last_error()` then holds a message (thread-local).
 *
 * Reference interfaces each entry point replaces (paths relative to the FEDn
 * checkout, v0.33.0):
 *   fa_fedavg_fold   numpyhelper.Helper.increment_average
 *                    fedn/utils/helpers/plugins/numpyhelper.py:18-32, applied in
 *                    queue order by fedavg.Aggregator.combine_models
 *                    fedn/network/combiner/aggregators/fedavg.py:47-71, and by
 *                    Control.reduce fedn/network/controller/control.py:678-682
 *   fa_fedopt_step   the pseudo-gradient loop + server optimizer of
 *                    fedopt.Aggregator.combine_models
 *                    fedn/network/combiner/aggregators/fedopt.py:74-118 with
 *                    serveropt_adam   fedopt.py:151-185
 *                    serveropt_yogi   fedopt.py:187-223
 *                    serveropt_adagrad fedopt.py:225-258
 *                    and the helper primitives numpyhelper.py:34-142 they call.
 *
 * Numerics contract: results are bit-identical to the numpy reference for the
 * dtypes it defines (IEEE-754 op-by-op replay of the same expression order, no
 * FMA contraction, correctly rounded division and square root). bf16 inputs have
 * no numpy counterpart: they are defined as the fp32 path on the exactly
 * upcast values.
 */
#ifndef FEDAGG_H
#define FEDAGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_ABI_VERSION 8

/* element type codes */
enum fa_dtype {
    FA_NONE = -1, /* "array is None" (FedOpt state before the first round) */
    FA_F32 = 0,
    FA_F64 = 1,
    FA_BF16 = 2,
    FA_F16 = 3,
    FA_I32 = 4,
    FA_I64 = 5,
    /* narrow / unsigned integers: accepted by fa_cast and the FA_EW_IFOLD / FA_EW_NFOLD folds only
       (models with such tensors are aggregated by the per-tensor path, fedn_amd/mixed.py) */
    FA_I8 = 6,
    FA_I16 = 7,
    FA_U8 = 8,
    FA_U16 = 9,
    FA_U32 = 10,
    FA_U64 = 11
};

/* status codes */
enum fa_status {
    FA_OK = 0,
    FA_EINVAL = 1,  /* bad argument (null pointer, negative size, K out of range) */
    FA_EDTYPE = 2,  /* unsupported dtype combination */
    FA_EHIP = 3     /* a HIP runtime call or kernel launch failed */
};

/* server optimizers, fedopt.py:141-145 */
enum fa_serveropt { FA_ADAM = 0, FA_YOGI = 1, FA_ADAGRAD = 2 };

/* fa_fedopt_step flags */
#define FA_PG_FIRST 1 /* pseudo-gradient starts from updates[0] - old (fedopt.py:89-91); else read from pg */
#define FA_PG_FINAL 2 /* apply the server step and write m_out, v_out, out; else write pg   */

int fa_abi_version(void);
const char* fa_last_error(void);
/* ABI 8: the kernel family the calling thread's last fold / FedOpt launch ran ("k_fedavg",
 * "k_fedavg_pipe", "k_fedavg_pipe_win", "k_fedopt", "k_fedopt_c", "k_fedopt_cw"; "" before any), so a
 * benchmark reports the kernel that ran — e.g. whether the store window was used — not a guess. */
const char* fa_last_kernel(void);

/*
 * FedAvg incremental weighted fold (numpyhelper.py:32):
 *     x <- x + (n_k * (y_k - x)) / N_k        for k in queue order
 *
 * agg      device buffer, P elements of agg_dtype (the running model)
 * updates  HOST array of K DEVICE pointers, each P elements of upd_dtype
 * n, N     HOST arrays of K doubles: num_examples of update k and the running
 *          total including it (fedavg.py:62), exact integers
 * init     1: agg := updates[0] (the `model = model_next` alias, fedavg.py:65-66),
 *             then fold k = 1..K-1;  0: fold k = 0..K-1 into the existing agg
 * stream   hipStream_t (NULL = default stream)
 *
 * dtype pairs (upd, agg) and the compute type numpy would use:
 *   (F32,F32)->f32  (BF16,F32)->f32  (F16,F16)->f16  (F64,F64)->f64
 *   (F32,F64)->f64  (I64,F64)/(I32,F64)->int then f64 (numpy true_divide)
 * With init=1 and K=1 the result is a plain copy and agg_dtype must equal upd_dtype.
 * Integer updates with init=1: n[1] must be integral (numpy multiplies the first integer difference
 * in the integer dtype only for an int num_examples; see FA_EW_IFOLD for a float one).
 */
int fa_fedavg_fold(void* agg, int agg_dtype,
                   const void* const* updates, int upd_dtype,
                   const double* n, const double* N, int K,
                   int64_t P, int init, void* stream);

/*
 * fa_fedavg_fold_host (ABI 8): fa_fedavg_fold for a small model whose round never leaves the host
 * (configs[0]: FEDn's mnist-pytorch example, fedavg.py:47-83 over 52,650 parameters). agg and every
 * updates[k] are PAGE-LOCKED HOST addresses (e.g. the pinned arena the updates were packed into and a
 * pinned result block); the kernel reads and writes them over PCIe through their device mappings
 * (hipHostGetDevicePointer), and the call returns once `stream` has drained, with the model in agg.
 * No H2D / D2H copy and no event: the round's GPU work is one launch and one wait. Same kernel,
 * client table and dtype pairs as fa_fedavg_fold, so the same bits. K <= 64 (one launch).
 * FA_EINVAL for memory that is not page-locked.
 */
int fa_fedavg_fold_host(void* agg, int agg_dtype, const void* const* updates, int upd_dtype,
                        const double* n, const double* N, int K, int64_t P, int init, void* stream);

/*
 * fa_fedopt_step_host (ABI 8): the FedOpt round of a small model in one call — fa_fedopt_step_ex with
 * flags FA_PG_FIRST | FA_PG_FINAL and no pg workspace, where `old`, every updates[k] and `out` are
 * PAGE-LOCKED HOST addresses (the global model and the updates packed into a pinned arena, a pinned
 * result block), mapped inside; m_in / m_out / v_in / v_out are device buffers as in
 * fa_fedopt_step_ex (the session's state stays in HBM). Returns once `stream` has drained. 1 <= K <= 64.
 */
int fa_fedopt_step_host(const void* old, int old_dtype, const void* const* updates, int upd_dtype,
                        const double* n, const double* N, int K,
                        const void* m_in, int m_in_dtype, void* m_out, int m_out_dtype,
                        const void* v_in, int v_in_dtype, void* v_out, void* out, int state_dtype,
                        int serveropt, double lr, double beta1, double beta2, double tau, int64_t P, void* stream);

/*
 * FedOpt (fedopt.py:74-118, 151-258), fused: pseudo-gradient running mean over the
 * K updates followed (FA_PG_FINAL) by one Adam / Yogi / AdaGrad server step.
 *
 * old       device, P elements of old_dtype (F32 | F64 | F16 | I32 | I64): the global model the
 *           clients trained from (fedopt.py:90)
 * updates   HOST array of K DEVICE pointers (F32 | BF16 | F16 | F64 | I32 | I64); a float16
 *           pseudo-gradient (F16 updates over an F16 model) is computed with numpy's half loops
 *           (every op rounded to half, python scalars cast to half); integer tensors
 *           (e.g. BatchNorm counters) become float64 exactly as numpy's int * 1.0 does.
 *           upd_dtype is required even when K = 0: it fixes the pg dtype.
 * n, N      HOST arrays of K doubles (num_examples, running total)
 * pg        device workspace, P elements of pg dtype = promote(upd, old) (F64 for integer
 *           updates); read when
 *           !FA_PG_FIRST, written when !FA_PG_FINAL (and used internally when
 *           K exceeds one launch); may be NULL when FIRST|FINAL and K <= 64
 * m_in      device, P elements of m_in_dtype (F16 | F32 | F64), or NULL with m_in_dtype = FA_NONE
 * m_out     device, dtype promote(m_in, pg) (pg dtype when m is None); may alias m_in
 *           when the dtypes are equal
 * v_in      device f64, or NULL (v is None -> ones * tau**2, fedopt.py:170-171)
 * v_out     device f64; may alias v_in
 * out       device f64 (the new global model, fedopt.py:183)
 * serveropt FA_ADAM | FA_YOGI | FA_ADAGRAD; lr, beta1, beta2, tau as in fedopt.py:53-59
 */
int fa_fedopt_step(const void* old, int old_dtype,
                   const void* const* updates, int upd_dtype,
                   const double* n, const double* N, int K,
                   void* pg, int flags,
                   const void* m_in, int m_in_dtype, void* m_out,
                   const double* v_in, double* v_out, double* out,
                   int serveropt, double lr, double beta1, double beta2, double tau,
                   int64_t P, void* stream);

/*
 * fa_fedopt_step with the storage dtypes of the server state explicit: the reference's flow
 * (state_dtype F64; m_out_dtype = numpy's promote(m_in, pg)) or the fp32-STATE mode (state_dtype
 * F32): v_out and out are float32 and m_out may be F32. Same arithmetic as the reference step on the
 * values it is given (f64 server step, numpy's dtype rules for m and the pseudo-gradient); each
 * stored value is the f64 result rounded once to f32, and f32 state is widened exactly on load.
 * HBM bytes per round in that mode with fp32 updates, old, m, v: P*(4K + 24) instead of
 * P*(4K + 48) (plug-in fedn_amd.aggregators.fedopt_f32state).
 * v_in_dtype: F64 or F32 (either mode may read either: a session can switch).
 */
int fa_fedopt_step_ex(const void* old, int old_dtype,
                      const void* const* updates, int upd_dtype,
                      const double* n, const double* N, int K,
                      void* pg, int flags,
                      const void* m_in, int m_in_dtype, void* m_out, int m_out_dtype,
                      const void* v_in, int v_in_dtype, void* v_out, void* out, int state_dtype,
                      int serveropt, double lr, double beta1, double beta2, double tau,
                      int64_t P, void* stream);

/*
 * Server-function aggregation rules (hooks.py:109-143): the two formulas the reference ships
 * as examples of user aggregation code, on device buffers with numpy's rounding.
 *
 * fa_weighted_sum replaces the loop of examples/server-functions/server_functions.py:58-67
 *     for each client k in order:  acc[i] += updates[k][i] * w[k]
 *   the product in the update dtype (w is a weak python scalar), the sum in
 *   promote(acc, update), stored in the accumulator dtype. acc is read (start from zeros for
 *   the example's np.zeros_like). The final `/ total_weight` is fa_elementwise(FA_EW_DIV).
 *   acc_dtype, upd_dtype in {F32, F64}; w: HOST array of K doubles; any K (chunked by 64).
 *
 * fa_running_mean replaces examples/server-functions/sf_incremental_aggregation.py:36-37
 *     g[i] = (g[i] * a + m[i] * b) / T      with a = T - n, b = n, T = running total
 *   in place, g and m of the same dtype (F32 or F64); every scalar cast to that dtype.
 */
int fa_weighted_sum(void* acc, int acc_dtype, const void* const* updates, int upd_dtype,
                    const double* w, int K, int64_t P, void* stream);
int fa_running_mean(void* g, int dtype, const void* m, double a, double b, double T,
                    int64_t P, void* stream);

/*
 * numpyhelper primitives (numpyhelper.py:34-142) on device buffers, numpy rounding (python
 * scalars a, b are weak: x*a is computed in x's dtype, then promoted). F32 / F64, and AXPBY on
 * three F16 arrays (numpy's half loops: a, b cast to half, every op rounded to half).
 *   FA_EW_AXPBY   out = x*a + y*b                 numpyhelper.add / subtract (b -> -b)
 *   FA_EW_MUL     out = x*y, or x*a if y == NULL   numpyhelper.multiply
 *   FA_EW_DIV     out = x/y, or x/a if y == NULL   numpyhelper.divide
 *   FA_EW_SQRT    out = sqrt(x)                    numpyhelper.sqrt
 *   FA_EW_SQUARE  out = x*x                        numpyhelper.power(m, 2)
 *   FA_EW_SIGN    out = sign(x) (+-1, 0, NaN)      numpyhelper.sign
 *   FA_EW_FILL    out = 1.0*a (x unused)           numpyhelper.ones
 *   FA_EW_POW     out = x**a (float a)             numpyhelper.power(m, a); f32 computed as the f64
 *                                                  power rounded once (numpy's own float power is its
 *                                                  host libm's / SIMD library's: not bit-reproducible
 *                                                  across hosts; parity: 1e-6 relative, f64 1e-15)
 *   FA_EW_IPOW    out = x**a, x any integer dtype (I8..I64, U8..U64), a a non-negative integer:
 *                 exponentiation by squaring with wrapping products, out_dtype = x_dtype (numpy's
 *                 integer power)
 *   FA_EW_IFOLD   out = x + ((y - x)*a)/b, x and y of one integer dtype (I8..I64, U8..U64), out
 *                 F64: numpyhelper.increment_average (numpyhelper.py:32) on integer arrays with a
 *                 python-float num_examples a and total b — the difference wraps in the integer
 *                 dtype, then float64 multiply, divide and add, each rounded once
 *   FA_EW_NFOLD   out = x + T((y - x)*a)/b, x and y of one integer dtype T (I8, I16, U8, U16, U32,
 *                 U64, I32, I64), out F64: the same fold with a python-INT num_examples a (integral,
 *                 |a| < 2^53; numpy refuses an a outside T's range, and so must the caller) —
 *                 difference and product wrap in T, then the float64 divide by b and add
 * out_dtype must be the numpy result dtype of the op.
 */
enum fa_ew_op { FA_EW_AXPBY = 0, FA_EW_MUL = 1, FA_EW_DIV = 2, FA_EW_SQRT = 3, FA_EW_SQUARE = 4, FA_EW_SIGN = 5,
                FA_EW_FILL = 6, FA_EW_POW = 7, FA_EW_IPOW = 8, FA_EW_IFOLD = 9,
                FA_EW_NFOLD = 10 };
int fa_elementwise(int op, void* out, int out_dtype, const void* x, int x_dtype, const void* y, int y_dtype,
                   double a, double b, int64_t P, void* stream);

/*
 * numpyhelper.norm (numpyhelper.py:106-117) for one tensor: np.linalg.norm(x, 1), i.e. sum |x| of a
 * vector (matrix = 0; rows*cols elements) or the max column sum of |x| of a C-order rows x cols
 * matrix (matrix = 1). x: F32 | F64 | any integer dtype (numpy: astype(float) first). Accumulated in
 * f64 in a fixed order (numpy sums f32
 * pairwise in f32: parity 1e-6 relative). out: DEVICE double (written on `stream`); work: DEVICE
 * scratch of fa_norm1_work(rows, cols, matrix) doubles.
 */
int64_t fa_norm1_work(int64_t rows, int64_t cols, int matrix);
int fa_norm1(double* out, const void* x, int dtype, int64_t rows, int64_t cols, int matrix, double* work,
             void* stream);

/* dtype promotion used by the two entry points above (numpy result_type for the
 * pairs this library supports; bf16 promotes as f32). Returns FA_NONE if unsupported. */
int fa_promote(int a, int b);

/*
 * Broadcast + widening conversion, the implicit step numpy takes before a binary ufunc whose
 * operands differ in dtype or (broadcastable) shape — e.g. numpyhelper.py:32 folding a float64
 * client into a float32 model, an int64 model with a float32 client, or a (1,) tensor against
 * (n,). Used by the per-tensor path of the plug-ins (fedn_amd/mixed.py) when client updates
 * differ from the running model (fedavg.py:68, fedopt.py:91-94, control.py:682).
 *
 *   out[i] = convert(in[j(i)])      i over the ndim-dimensional C-order index space out_shape,
 *                                   j(i) = sum_d i_d * in_strides[d] (element strides; 0 along
 *                                   broadcast dimensions)
 * Conversions (numpy's casting of the value): identity for every dtype; F16/BF16 -> F32/F64 and
 * F32 -> F64 (exact); I32 -> I64 (exact); I32/I64 -> F64 (round to nearest even); I8 / I16 / U8 /
 * U16 / U32 / U64 to every integer or float dtype numpy casts them to safely (U64 -> F64 rounds to
 * nearest even, the rest are exact); and two narrowing float casts, F32 -> F16 and F64 -> F32, rounded
 * to nearest even as numpy's astype (the result of a helper op computed in a wider float: a single
 * correctly rounded op then rounded again equals the op rounded once, since 24 >= 2*11+2 and
 * 53 >= 2*24+2). Other narrowing conversions are refused (FA_EDTYPE). 1 <= ndim <= 8; out is contiguous.
 */
int fa_cast(void* out, int out_dtype, const void* in, int in_dtype, int ndim, const int64_t* out_shape,
            const int64_t* in_strides, void* stream);

/*
 * Peer transport of the parameter-sliced all-gather ("prefer ... direct (all 7
 * links)"; the gathered model's consumer is roundhandler.py:465-468). Replaces the transport of
 * RCCL's ncclAllGather for fedn_amd/sharded.py P2PAllGather (one process per GPU) and
 * fedn_amd/multidev.py allgather_devices (one process, several GPUs): every rank copies its folded
 * slice straight into each peer's model buffer, one copy stream per peer (one xGMI link each).
 *
 * fa_ipc_get_handle  FA_IPC_HANDLE_BYTES of handle for the allocation that holds dptr, and dptr's
 *                    byte offset in it (a caching allocator hands out pieces of one allocation)
 * fa_ipc_open        map another process's handle: *base = the mapping (pass it to fa_ipc_close),
 *                    *dptr = base + offset
 * fa_ipc_close       unmap a mapping fa_ipc_open returned
 * fa_copy_async      bytes from src to dst on stream; any two device pointers of this process
 *                    (IPC mappings and other devices' buffers included): the DMA engines move them
 * fa_push            bytes from src to each of ndst (<= 16) destinations on stream, by a kernel: the
 *                    source is read once and every destination (IPC mappings of the peers' model
 *                    buffers, or in-process peers' buffers) written by vector stores — each over its
 *                    own link, all at once; 16-B aligned pointers. The alternative to one
 *                    fa_copy_async per peer that the all-gather picks between (sharded.P2PAllGather;
 *                    replaces the all-gather consumed at roundhandler.py:465-468)
 * fa_fedavg_fold_push  fa_fedavg_fold (fp32 updates, fp32 aggregate, 16-B aligned buffers) whose kernel
 *                    also stores every finished element to each of ndst (<= 16) destinations: the
 *                    fold and the all-gather push in ONE pass (sharded.P2PAllGather engine "fused";
 *                    the peers' buffers IPC-mapped or in-process). agg is this rank's own copy.
 *   release_rec      (fa_push, fa_fedavg_fold_push; ABI 7) after a grid that stored into peers, a
 *                    release grid writes every XCD's L2 back at system scope. HIP does not promise
 *                    which XCDs a grid's workgroups run on, so each release workgroup records its
 *                    XCD (HW_REG_XCC_ID) in release_rec: FA_RELEASE_WORDS uint32 of caller-owned
 *                    DEVICE memory, zeroed once before the first call and then passed to every call
 *                    on one stream. Per release launch, the last workgroup compares the number of
 *                    distinct XCDs covered with the device's XCD count (IDs are counted, not matched
 *                    against 0 .. n - 1: a partition mode may report physical indices) and
 *                    increments FA_REL_MISSES on a gap; FA_REL_LAUNCHES counts the launches checked,
 *                    FA_REL_SEEN is the union of the XCDs seen and FA_REL_EXPECT the mask
 *                    (1 << n) - 1 of the device's XCD count. The caller reads the record at a
 *                    synchronisation point and must treat MISSES > 0 as a failed exchange. NULL:
 *                    release without the record (in-process peers behind a device synchronize).
 * fa_device_xccs     *n = the number of XCDs (each with its own L2) of device dev
 * fa_peer_enable     let device dev read / write device peer's memory directly (in-process);
 *                    already enabled is not an error
 * fa_host_register   page-lock host memory the caller mapped (the node's shared host model that
 *                    every rank D2H's its slice into: sharded.HostGather), so DMA reaches it directly;
 * fa_host_unregister undo it before the caller unmaps
 * fa_host_device_ptr the device address of page-locked host memory (hipHostGetDevicePointer): a
 *                    small round's fold reads its clients from the pinned arena and writes the
 *                    model into the caller's pinned block over PCIe, with no H2D / D2H copy
 *                    (staging.FedAvgPipeline.result); an error for pageable memory
 */
#define FA_IPC_HANDLE_BYTES 64
#define FA_RELEASE_WORDS 8
enum fa_release_word { FA_REL_MASK = 0, FA_REL_ARRIVED = 1, FA_REL_LAUNCHES = 2, FA_REL_MISSES = 3, FA_REL_SEEN = 4,
                       FA_REL_EXPECT = 5 };
int fa_ipc_get_handle(const void* dptr, void* handle, uint64_t* offset);
int fa_ipc_open(const void* handle, uint64_t offset, void** base, void** dptr);
int fa_ipc_close(void* base);
int fa_copy_async(void* dst, const void* src, int64_t bytes, void* stream);
int fa_push(void* const* dsts, int ndst, const void* src, int64_t bytes, uint32_t* release_rec, void* stream);
int fa_fedavg_fold_push(float* agg, const void* const* updates, const double* n, const double* N, int K, int64_t P,
                        int init, void* const* dsts, int ndst, uint32_t* release_rec, void* stream);
int fa_device_xccs(int dev, int* n);
int fa_peer_enable(int dev, int peer);
int fa_host_register(void* p, int64_t bytes);
int fa_host_unregister(void* p);
int fa_host_device_ptr(const void* host, void** dptr);

#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_H */
