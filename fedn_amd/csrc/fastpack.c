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

static PyMethodDef methods[] = {
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
