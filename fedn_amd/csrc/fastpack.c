/* _fastpack: admission + pack of one small host update in ONE native call (CPython extension).
 *
 * The per-update work of the plug-ins' small-model path (staging._Pipeline.put_small): FEDn hands
 * the aggregator each update as a list of numpy arrays (fedavg.py:47-68 via load_model_update,
 * updatehandler.py:93-117); a round whose updates all have the first update's exact layout folds
 * them in one multi-client launch from a pinned arena. Deciding that an update has that layout
 * (one exact (shape, dtype) test per tensor, C-contiguous) and queueing its copies into the arena
 * took ~14 us of Python per update (ctypes pointers, argument arrays), more than numpy's own fold
 * of a 52,650-param mnist update (~23 us). Here it is one C call: the test reads the array structs
 * directly and the copies go to libfednpz's gather thread (fnpz_gather_start, reached through the
 * function address the caller passes), so the Python thread moves on to the next update.
 *
 *   plan(specs) -> capsule       specs: one (shape tuple, dtype, dst byte offset) per tensor
 *   admit(plan, arrays, dst_addr, gather_start_addr, threads, buf_addr, buf_len) -> int
 *       > 0  the gather ticket (wait on it with fnpz_gather_wait before reading dst)
 *         0  admitted, nothing to copy (only empty tensors)
 *        -1  not this layout (wrong length / type / shape / dtype, or not C-contiguous): the
 *            caller takes its general path, which raises numpy's error where numpy would
 *        -2  the gather queue refused the job (fnpz_last_error says why: e.g. FNPZ_ENOSPC, a
 *            destination outside [buf_addr, buf_addr + buf_len), the pinned buffer it packs into)
 * The caller keeps ``arrays`` referenced until the ticket is done.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_2_0_API_VERSION
#include <numpy/arrayobject.h>
#include <stdint.h>
#include <string.h>

typedef int64_t (*gather_start_fn)(int n, void* const* dsts, const void* const* srcs, const int64_t* nbytes,
                                   int threads, const void* dst_lo, int64_t dst_len);

typedef struct {
    int ndim;
    npy_intp shape[NPY_MAXDIMS];
    PyArray_Descr* dtype; /* owned reference */
    int64_t dst_off;
    int64_t nbytes;
} Tensor;

typedef struct {
    Py_ssize_t n;
    Tensor t[];
} Plan;

#define MAX_STACK 64

static void plan_free(PyObject* cap) {
    Plan* p = (Plan*)PyCapsule_GetPointer(cap, "fedn_amd._fastpack.plan");
    if (!p) return;
    for (Py_ssize_t i = 0; i < p->n; ++i) Py_XDECREF(p->t[i].dtype);
    PyMem_Free(p);
}

static PyObject* fp_plan(PyObject* self, PyObject* args) {
    PyObject* specs;
    if (!PyArg_ParseTuple(args, "O!", &PyList_Type, &specs)) return NULL;
    Py_ssize_t n = PyList_GET_SIZE(specs);
    Plan* p = (Plan*)PyMem_Calloc(1, sizeof(Plan) + (size_t)n * sizeof(Tensor));
    if (!p) return PyErr_NoMemory();
    p->n = n;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *shape, *dt;
        long long off;
        if (!PyArg_ParseTuple(PyList_GET_ITEM(specs, i), "O!OL", &PyTuple_Type, &shape, &dt, &off)) goto fail;
        Tensor* t = &p->t[i];
        t->ndim = (int)PyTuple_GET_SIZE(shape);
        if (t->ndim > NPY_MAXDIMS) {
            PyErr_SetString(PyExc_ValueError, "too many dimensions");
            goto fail;
        }
        npy_intp count = 1;
        for (int d = 0; d < t->ndim; ++d) {
            t->shape[d] = (npy_intp)PyLong_AsSsize_t(PyTuple_GET_ITEM(shape, d));
            if (t->shape[d] < 0) {
                if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "negative dimension");
                goto fail;
            }
            count *= t->shape[d];
        }
        if (!PyArray_DescrConverter(dt, &t->dtype)) goto fail;
        t->dst_off = off;
        t->nbytes = (int64_t)count * (int64_t)PyDataType_ELSIZE(t->dtype);
    }
    PyObject* cap = PyCapsule_New(p, "fedn_amd._fastpack.plan", plan_free);
    if (!cap) goto fail;
    return cap;
fail:
    for (Py_ssize_t i = 0; i < n; ++i) Py_XDECREF(p->t[i].dtype);
    PyMem_Free(p);
    return NULL;
}

static inline int same_dtype(PyArray_Descr* a, PyArray_Descr* b) {
    return a == b || PyArray_EquivTypes(a, b);
}

static PyObject* fp_admit(PyObject* self, PyObject* args) {
    PyObject *cap, *arrays;
    unsigned long long dst, fn, buf;
    long long buf_len;
    int threads;
    if (!PyArg_ParseTuple(args, "OOKKiKL", &cap, &arrays, &dst, &fn, &threads, &buf, &buf_len)) return NULL;
    Plan* p = (Plan*)PyCapsule_GetPointer(cap, "fedn_amd._fastpack.plan");
    if (!p) return NULL;
    if (!PyList_CheckExact(arrays) || PyList_GET_SIZE(arrays) != p->n) return PyLong_FromLong(-1);
    void* dsts_s[MAX_STACK];
    const void* srcs_s[MAX_STACK];
    int64_t nb_s[MAX_STACK];
    void** dsts = dsts_s;
    const void** srcs = srcs_s;
    int64_t* nb = nb_s;
    if (p->n > MAX_STACK) {
        dsts = (void**)PyMem_Malloc(sizeof(void*) * p->n);
        srcs = (const void**)PyMem_Malloc(sizeof(void*) * p->n);
        nb = (int64_t*)PyMem_Malloc(sizeof(int64_t) * p->n);
        if (!dsts || !srcs || !nb) {
            PyMem_Free(dsts), PyMem_Free(srcs), PyMem_Free(nb);
            return PyErr_NoMemory();
        }
    }
    long rc = 0;
    int k = 0;
    for (Py_ssize_t i = 0; i < p->n; ++i) {
        PyObject* o = PyList_GET_ITEM(arrays, i);
        const Tensor* t = &p->t[i];
        if (Py_TYPE(o) != &PyArray_Type) { rc = -1; break; }     /* exactly numpy.ndarray, as fast_host */
        PyArrayObject* a = (PyArrayObject*)o;
        if (PyArray_NDIM(a) != t->ndim || !PyArray_IS_C_CONTIGUOUS(a)) { rc = -1; break; }
        const npy_intp* sh = PyArray_DIMS(a);
        int ok = 1;
        for (int d = 0; d < t->ndim; ++d) ok &= sh[d] == t->shape[d];
        if (!ok || !same_dtype(PyArray_DESCR(a), t->dtype)) { rc = -1; break; }
        if (t->nbytes) {
            dsts[k] = (void*)(uintptr_t)(dst + (unsigned long long)t->dst_off);
            srcs[k] = PyArray_DATA(a);
            nb[k] = t->nbytes;
            ++k;
        }
    }
    if (rc == 0 && k > 0) {
        int64_t ticket = ((gather_start_fn)(uintptr_t)fn)(k, dsts, srcs, nb, threads < 1 ? 1 : threads,
                                                           (const void*)(uintptr_t)buf, (int64_t)buf_len);
        rc = ticket > 0 ? (long)ticket : -2;
    }
    if (dsts != dsts_s) PyMem_Free(dsts), PyMem_Free(srcs), PyMem_Free(nb);
    return PyLong_FromLong(rc);
}

/* ---- a small model's round end: pack wait + fold + wait in one call (smallround.py) --------------
 *
 *   fold_plan([(agg_dtype, upd_dtype, byte_offset, elems), ...]) -> capsule   one entry per dtype group
 *   fold_host(fold_plan, fold_addr, wait_addr, ticket, arena_addr, stride, K, out_addr, n, N, stream)
 *       -> status
 * fold_host waits for the gather ticket (the updates' packs into the pinned arena, fnpz_gather_wait),
 * then for each group calls fa_fedavg_fold_host (include/fedagg.h: the fold of K pinned host updates
 * into pinned host memory, synchronous) with updates[k] = arena + k * stride + offset, the result at
 * out + offset; n / N are sequences of K floats (n[0] = 0, N[0] = 1: agg := the first update). The GIL
 * is released throughout. Returns fa_fedavg_fold_host's status (0 = the model is in out), or -1 if
 * the pack failed (fnpz_last_error says why). */
typedef int (*fold_host_fn)(void* agg, int agg_dtype, const void* const* updates, int upd_dtype, const double* n,
                            const double* N, int K, int64_t P, int init, void* stream);
typedef int (*gather_wait_fn)(int64_t ticket);

typedef struct {
    int agg_dtype, upd_dtype;
    int64_t off, elems;
} Group;

typedef struct {
    Py_ssize_t n;
    Group g[];
} FoldPlan;

#define MAX_FOLD_K 64

static void fold_plan_free(PyObject* cap) {
    PyMem_Free(PyCapsule_GetPointer(cap, "fedn_amd._fastpack.fold_plan"));
}

static PyObject* fp_fold_plan(PyObject* self, PyObject* args) {
    PyObject* specs;
    if (!PyArg_ParseTuple(args, "O!", &PyList_Type, &specs)) return NULL;
    Py_ssize_t n = PyList_GET_SIZE(specs);
    FoldPlan* p = (FoldPlan*)PyMem_Calloc(1, sizeof(FoldPlan) + (size_t)n * sizeof(Group));
    if (!p) return PyErr_NoMemory();
    p->n = n;
    for (Py_ssize_t i = 0; i < n; ++i) {
        long long off, elems;
        if (!PyArg_ParseTuple(PyList_GET_ITEM(specs, i), "iiLL", &p->g[i].agg_dtype, &p->g[i].upd_dtype, &off, &elems)) {
            PyMem_Free(p);
            return NULL;
        }
        if (off < 0 || elems < 0) {
            PyMem_Free(p);
            PyErr_SetString(PyExc_ValueError, "negative offset or size");
            return NULL;
        }
        p->g[i].off = off;
        p->g[i].elems = elems;
    }
    PyObject* cap = PyCapsule_New(p, "fedn_amd._fastpack.fold_plan", fold_plan_free);
    if (!cap) PyMem_Free(p);
    return cap;
}

static int read_doubles(PyObject* seq, double* out, Py_ssize_t K) {
    PyObject* f = PySequence_Fast(seq, "n and N must be sequences");
    if (!f) return -1;
    if (PySequence_Fast_GET_SIZE(f) != K) {
        Py_DECREF(f);
        PyErr_SetString(PyExc_ValueError, "n and N need one entry per update");
        return -1;
    }
    for (Py_ssize_t k = 0; k < K; ++k) {
        out[k] = PyFloat_AsDouble(PySequence_Fast_GET_ITEM(f, k));
        if (out[k] == -1.0 && PyErr_Occurred()) {
            Py_DECREF(f);
            return -1;
        }
    }
    Py_DECREF(f);
    return 0;
}

static PyObject* fp_fold_host(PyObject* self, PyObject* args) {
    PyObject *cap, *ns, *Ns;
    unsigned long long fold, wait, arena, out, stream;
    long long ticket, stride;
    int K;
    if (!PyArg_ParseTuple(args, "OKKLKLiKOOK", &cap, &fold, &wait, &ticket, &arena, &stride, &K, &out, &ns, &Ns,
                          &stream))
        return NULL;
    FoldPlan* p = (FoldPlan*)PyCapsule_GetPointer(cap, "fedn_amd._fastpack.fold_plan");
    if (!p) return NULL;
    if (K < 1 || K > MAX_FOLD_K || stride < 0 || !arena || !out || !fold) {
        PyErr_SetString(PyExc_ValueError, "fold_host: bad arguments");
        return NULL;
    }
    double n[MAX_FOLD_K], N[MAX_FOLD_K];
    if (read_doubles(ns, n, K) || read_doubles(Ns, N, K)) return NULL;
    int rc = 0;
    Py_BEGIN_ALLOW_THREADS
    if (ticket > 0 && wait) rc = ((gather_wait_fn)(uintptr_t)wait)((int64_t)ticket) ? -1 : 0;
    for (Py_ssize_t i = 0; rc == 0 && i < p->n; ++i) {
        const Group* g = &p->g[i];
        if (!g->elems) continue;
        const void* ups[MAX_FOLD_K];
        for (int k = 0; k < K; ++k) ups[k] = (const void*)(uintptr_t)(arena + (unsigned long long)k * stride + g->off);
        rc = ((fold_host_fn)(uintptr_t)fold)((void*)(uintptr_t)(out + g->off), g->agg_dtype, ups, g->upd_dtype, n, N, K,
                                              g->elems, 1, (void*)(uintptr_t)stream);
    }
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

/*   fedopt_host(fn, wait, ticket, old, arena, stride, K, upd_dtype, old_dtype, P, out, n, N, stream,
 *               (m_in, m_in_dtype, m_out, m_out_dtype, v_in, v_in_dtype, v_out, state_dtype),
 *               serveropt, lr, beta1, beta2, tau) -> status
 * A small model's FedOpt round (one dtype group): the global model packed into the pinned block at
 * ``old`` and the K updates at arena slots 0..K-1; waits for the packs (``ticket``: the last), then fa_fedopt_step_host (include/fedagg.h: FIRST |
 * FINAL, the new model into pinned ``out``, m / v device buffers) — the GIL released throughout.
 * -1 if the pack failed (fnpz_last_error says why). */
typedef int (*fedopt_host_fn)(const void* old, int old_dtype, const void* const* updates, int upd_dtype,
                              const double* n, const double* N, int K, const void* m_in, int m_in_dtype, void* m_out,
                              int m_out_dtype, const void* v_in, int v_in_dtype, void* v_out, void* out,
                              int state_dtype, int serveropt, double lr, double beta1, double beta2, double tau,
                              int64_t P, void* stream);

static PyObject* fp_fedopt_host(PyObject* self, PyObject* args) {
    PyObject *ns, *Ns;
    unsigned long long fn, wait, old, arena, out, stream, m_in, m_out, v_in, v_out;
    long long ticket, stride, P;
    int K, upd_dt, old_dt, m_in_dt, m_out_dt, v_in_dt, state_dt, opt;
    double lr, b1, b2, tau;
    if (!PyArg_ParseTuple(args, "KKLKKLiiiLKOOK(KiKiKiKi)idddd", &fn, &wait, &ticket, &old, &arena, &stride, &K, &upd_dt,
                          &old_dt, &P, &out, &ns, &Ns, &stream, &m_in, &m_in_dt, &m_out, &m_out_dt, &v_in, &v_in_dt,
                          &v_out, &state_dt, &opt, &lr, &b1, &b2, &tau))
        return NULL;
    if (K < 1 || K > MAX_FOLD_K || stride < 0 || P < 0 || !old || !arena || !out || !fn) {
        PyErr_SetString(PyExc_ValueError, "fedopt_host: bad arguments");
        return NULL;
    }
    double n[MAX_FOLD_K], N[MAX_FOLD_K];
    if (read_doubles(ns, n, K) || read_doubles(Ns, N, K)) return NULL;
    const void* ups[MAX_FOLD_K];
    for (int k = 0; k < K; ++k) ups[k] = (const void*)(uintptr_t)(arena + (unsigned long long)k * stride);
    int rc = 0;
    Py_BEGIN_ALLOW_THREADS
    if (ticket > 0 && wait) rc = ((gather_wait_fn)(uintptr_t)wait)((int64_t)ticket) ? -1 : 0;
    if (rc == 0)
        rc = ((fedopt_host_fn)(uintptr_t)fn)((const void*)(uintptr_t)old, old_dt, ups, upd_dt, n, N, K,
                                             (const void*)(uintptr_t)m_in, m_in_dt, (void*)(uintptr_t)m_out, m_out_dt,
                                             (const void*)(uintptr_t)v_in, v_in_dt, (void*)(uintptr_t)v_out,
                                             (void*)(uintptr_t)out, state_dt, opt, lr, b1, b2, tau, (int64_t)P,
                                             (void*)(uintptr_t)stream);
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

/*   views(plan, base) -> list    the model's arrays as views of ``base`` (a C-contiguous numpy array whose
 * bytes hold the packed layout ``plan`` describes: the admission plan), each keeping ``base`` alive */
static PyObject* fp_views(PyObject* self, PyObject* args) {
    PyObject *cap, *base;
    if (!PyArg_ParseTuple(args, "OO!", &cap, &PyArray_Type, &base)) return NULL;
    Plan* p = (Plan*)PyCapsule_GetPointer(cap, "fedn_amd._fastpack.plan");
    if (!p) return NULL;
    PyArrayObject* b = (PyArrayObject*)base;
    if (!PyArray_IS_C_CONTIGUOUS(b)) {
        PyErr_SetString(PyExc_ValueError, "views: base must be C-contiguous");
        return NULL;
    }
    const int64_t cap_bytes = (int64_t)PyArray_NBYTES(b);
    char* data = (char*)PyArray_DATA(b);
    PyObject* out = PyList_New(p->n);
    if (!out) return NULL;
    for (Py_ssize_t i = 0; i < p->n; ++i) {
        const Tensor* t = &p->t[i];
        if (t->dst_off < 0 || t->dst_off + t->nbytes > cap_bytes) {
            Py_DECREF(out);
            PyErr_SetString(PyExc_ValueError, "views: the plan does not fit the base array");
            return NULL;
        }
        Py_INCREF(t->dtype);   /* stolen by PyArray_NewFromDescr */
        PyObject* v = PyArray_NewFromDescr(&PyArray_Type, t->dtype, t->ndim, (npy_intp*)t->shape, NULL,
                                           data + t->dst_off, NPY_ARRAY_CARRAY, NULL);
        if (!v) {
            Py_DECREF(out);
            return NULL;
        }
        Py_INCREF(base);
        if (PyArray_SetBaseObject((PyArrayObject*)v, base) < 0) {
            Py_DECREF(v);
            Py_DECREF(out);
            return NULL;
        }
        PyList_SET_ITEM(out, i, v);
    }
    return out;
}

static PyMethodDef methods[] = {
    {"fold_plan", fp_fold_plan, METH_VARARGS, "fold_plan([(agg_dtype, upd_dtype, byte_offset, elems), ...]) -> capsule"},
    {"fold_host", fp_fold_host, METH_VARARGS,
     "fold_host(fold_plan, fold_addr, wait_addr, ticket, arena_addr, stride, K, out_addr, n, N, stream) -> status"},
    {"views", fp_views, METH_VARARGS, "views(plan, base) -> list of arrays viewing base"},
    {"fedopt_host", fp_fedopt_host, METH_VARARGS,
     "fedopt_host(fn, wait, ticket, old, arena, stride, K, upd_dtype, old_dtype, P, out, n, N, stream, state, serveropt, "
     "lr, beta1, beta2, tau) -> status"},
    {"plan", fp_plan, METH_VARARGS, "plan([(shape, dtype, dst_offset), ...]) -> capsule"},
    {"admit", fp_admit, METH_VARARGS,
     "admit(plan, arrays, dst_addr, gather_start_addr, threads, buf_addr, buf_len) -> ticket | 0 | -1 (not this "
     "layout) | -2"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fastpack", NULL, -1, methods};

PyMODINIT_FUNC PyInit__fastpack(void) {
    import_array();
    return PyModule_Create(&module);
}
