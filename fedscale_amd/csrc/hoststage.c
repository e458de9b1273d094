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
#include <string.h>

#ifndef HS_BUILD_ID
#define HS_BUILD_ID "unknown"
#endif

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
    if (!PyArray_CheckExact(a) || !PyArray_CheckExact(d)) return PyLong_FromSsize_t(i);
    PyArrayObject* x = (PyArrayObject*)a;
    PyArrayObject* y = (PyArrayObject*)d;
    const int nd = PyArray_NDIM(y);
    if (PyArray_NDIM(x) != nd || PyArray_TYPE(x) != PyArray_TYPE(y) || !PyArray_ISNOTSWAPPED(x) ||
        !PyArray_IS_C_CONTIGUOUS(x) || !PyArray_IS_C_CONTIGUOUS(y) || !PyArray_ISWRITEABLE(y))
      return PyLong_FromSsize_t(i);
    const npy_intp* xs = PyArray_DIMS(x);
    const npy_intp* ys = PyArray_DIMS(y);
    for (int k = 0; k < nd; ++k)
      if (xs[k] != ys[k]) return PyLong_FromSsize_t(i);
    const npy_intp nbytes = PyArray_NBYTES(y);
    if (nbytes) memcpy(PyArray_DATA(y), PyArray_DATA(x), (size_t)nbytes);
  }
  return PyLong_FromLong(-1);
}

static PyObject* hs_build_id(PyObject* self, PyObject* noargs) {
  (void)self;
  (void)noargs;
  return PyUnicode_FromString(HS_BUILD_ID);
}

static PyMethodDef hs_methods[] = {
    {"stage", hs_stage, METH_VARARGS, "stage(values, dsts) -> -1, or the index of the first entry left to Python"},
    {"build_id", hs_build_id, METH_NOARGS, "the build id of this module's source (fedscale_amd/buildinfo.py)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef hs_module = {PyModuleDef_HEAD_INIT, "_hoststage", NULL, -1, hs_methods, NULL, NULL, NULL,
                                       NULL};

PyMODINIT_FUNC PyInit__hoststage(void) {
  import_array();
  return PyModule_Create(&hs_module);
}
