/* hoststage.c — the host half of a small model's ingress, native (CPython extension fedscale_amd._hoststage).
 *
 * A small model's upload (config 1: FEMNIST CNN, 8 arrays, 98 KB) is copied entry by entry into the pinned
 * staging mirror the round's kernel reads over PCIe (ClientStaging bulk path).  In Python each entry costs a shape
 * check, a dtype check and a numpy assignment (~0.5 us on the MI355X host for arrays whose copy takes ~0.3 us);
 * here one call validates and copies the whole upload.  Semantics are the Python loop's (bucket.py
 * ClientStaging._put_bulk_views): entry i must be a plain C-contiguous numpy array of the destination's shape and
 * dtype in native byte order; at the first entry that is not, nothing more is written and its index is returned,
 * so the caller finishes that upload in Python (which converts or raises exactly as before).  -1: all copied.
 * No reference counterpart (the reference aggregates uploads as numpy arrays on the CPU, aggregator.py:497-503).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <emmintrin.h>
#include <stdint.h>
#include <string.h>

/* Non-temporal copies (the default): the staged rows are read by the GPU over PCIe (zero-copy) right after they are
 * written, so they go straight to DRAM with streaming stores instead of being left dirty in this core's cache for the
 * device's reads to snoop; one sfence per call orders them before the launch that follows.  0: plain memcpy. */
static int g_nt = 1;

static void copy_nt(char* d, const char* s, size_t n) {
  if (n < 1024) {
    memcpy(d, s, n);
    return;
  }
  const size_t head = (16 - ((uintptr_t)d & 15)) & 15;
  memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  const size_t blocks = n / 64;
  for (size_t i = 0; i < blocks; ++i) {
    const __m128i a = _mm_loadu_si128((const __m128i*)(s + 0));
    const __m128i b = _mm_loadu_si128((const __m128i*)(s + 16));
    const __m128i c = _mm_loadu_si128((const __m128i*)(s + 32));
    const __m128i e = _mm_loadu_si128((const __m128i*)(s + 48));
    _mm_stream_si128((__m128i*)(d + 0), a);
    _mm_stream_si128((__m128i*)(d + 16), b);
    _mm_stream_si128((__m128i*)(d + 32), c);
    _mm_stream_si128((__m128i*)(d + 48), e);
    d += 64;
    s += 64;
  }
  memcpy(d, s, n - blocks * 64);
}

#ifndef HS_BUILD_ID
#define HS_BUILD_ID "unknown"
#endif

/* the result of a stage() call: every streaming store made so far is ordered before anything that follows */
static PyObject* stop(Py_ssize_t i) {
  if (g_nt) _mm_sfence();
  return PyLong_FromSsize_t(i);
}

/* stage(values, dsts) -> int: copy values[i] into dsts[i] for every i (both lists of equal length) */
static PyObject* hs_stage(PyObject* self, PyObject* args) {
  PyObject *values, *dsts;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!", &PyList_Type, &values, &PyList_Type, &dsts)) return NULL;
  const Py_ssize_t n = PyList_GET_SIZE(dsts);
  if (PyList_GET_SIZE(values) != n) {
    PyErr_SetString(PyExc_ValueError, "stage: values and destinations differ in length");
    return NULL;
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* a = PyList_GET_ITEM(values, i);
    PyObject* d = PyList_GET_ITEM(dsts, i);
    if (!PyArray_CheckExact(a) || !PyArray_CheckExact(d)) return stop(i);
    PyArrayObject* x = (PyArrayObject*)a;
    PyArrayObject* y = (PyArrayObject*)d;
    const int nd = PyArray_NDIM(y);
    if (PyArray_NDIM(x) != nd || PyArray_TYPE(x) != PyArray_TYPE(y) || !PyArray_ISNOTSWAPPED(x) ||
        !PyArray_IS_C_CONTIGUOUS(x) || !PyArray_IS_C_CONTIGUOUS(y) || !PyArray_ISWRITEABLE(y))
      return stop(i);
    const npy_intp* xs = PyArray_DIMS(x);
    const npy_intp* ys = PyArray_DIMS(y);
    for (int k = 0; k < nd; ++k)
      if (xs[k] != ys[k]) return stop(i);
    const npy_intp nbytes = PyArray_NBYTES(y);
    if (nbytes) {
      if (g_nt)
        copy_nt((char*)PyArray_DATA(y), (const char*)PyArray_DATA(x), (size_t)nbytes);
      else
        memcpy(PyArray_DATA(y), PyArray_DATA(x), (size_t)nbytes);
    }
  }
  return stop(-1);
}

/* set_nt(on) -> previous setting (A/B of the copy policy) */
static PyObject* hs_set_nt(PyObject* self, PyObject* args) {
  int on;
  (void)self;
  if (!PyArg_ParseTuple(args, "p", &on)) return NULL;
  const int prev = g_nt;
  g_nt = on;
  return PyBool_FromLong(prev);
}

static PyObject* hs_build_id(PyObject* self, PyObject* noargs) {
  (void)self;
  (void)noargs;
  return PyUnicode_FromString(HS_BUILD_ID);
}

static PyMethodDef hs_methods[] = {
    {"stage", hs_stage, METH_VARARGS, "stage(values, dsts) -> -1, or the index of the first entry left to Python"},
    {"set_nt", hs_set_nt, METH_VARARGS, "set_nt(on) -> previous: streaming (non-temporal) copies on or off"},
    {"build_id", hs_build_id, METH_NOARGS, "the build id of this module's source (fedscale_amd/buildinfo.py)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef hs_module = {PyModuleDef_HEAD_INIT, "_hoststage", NULL, -1, hs_methods, NULL, NULL, NULL,
                                       NULL};

PyMODINIT_FUNC PyInit__hoststage(void) {
  import_array();
  return PyModule_Create(&hs_module);
}
