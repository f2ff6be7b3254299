/* _mtfast: a CPython extension that calls the library's generic tensor entry points
 * (mt_tensor_map / _zip / _reduce, mt_matmul_f32: include/minitorch_hip.h) with the shapes and
 * strides as Python tuples, converted on the C stack. It replaces ctypes on the host path of
 * every minitorch op on the HIP backend: a ctypes call with fourteen typed arguments and six
 * cached int64 arrays costs ≈ 3.2 µs of host time against ≈ 0.4 µs here, and a config-5 training
 * step makes ≈ 230 of them. No link-time dependency on the library: minitorch/_hip.py hands over
 * the entry points' addresses from the loaded libminitorch_hip.so (bind), so both always refer
 * to the same library and the HIP code runs exactly as through ctypes.
 * Built by the package Makefile (gcc, Python headers); optional: without it the ops keep ctypes. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

#define MAXD 16

typedef int (*map_fn)(int, float*, const int64_t*, const int64_t*, int, const float*, const int64_t*,
                      const int64_t*, int, void*);
typedef int (*zip_fn)(int, float*, const int64_t*, const int64_t*, int, const float*, const int64_t*,
                      const int64_t*, int, const float*, const int64_t*, const int64_t*, int, void*);
typedef int (*reduce_fn)(int, float*, const int64_t*, const int64_t*, const float*, const int64_t*,
                         const int64_t*, int, int, float, void*);
typedef int (*matmul_fn)(float*, const float*, const float*, int64_t, int64_t, int64_t, int64_t,
                         const int64_t*, const int64_t*, const int64_t*, void*);

static map_fn p_map = NULL;
static zip_fn p_zip = NULL;
static reduce_fn p_reduce = NULL;
static matmul_fn p_matmul = NULL;

/* a tuple of ints into out[0..n); returns n, or -1 with a Python error set */
static int tup(PyObject* t, int64_t* out) {
  if (!PyTuple_Check(t)) {
    PyErr_SetString(PyExc_TypeError, "_mtfast: shapes and strides are tuples of ints");
    return -1;
  }
  const Py_ssize_t n = PyTuple_GET_SIZE(t);
  if (n > MAXD) {
    PyErr_SetString(PyExc_ValueError, "_mtfast: more than 16 dims");
    return -1;
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    out[i] = PyLong_AsLongLong(PyTuple_GET_ITEM(t, i));
    if (out[i] == -1 && PyErr_Occurred()) return -1;
  }
  return (int)n;
}

static void* ptr_of(PyObject* o) { return PyLong_AsVoidPtr(o); }

static PyObject* bind(PyObject* self, PyObject* args) {
  PyObject *m, *z, *r, *mm;
  (void)self;
  if (!PyArg_ParseTuple(args, "OOOO", &m, &z, &r, &mm)) return NULL;
  p_map = (map_fn)ptr_of(m);
  p_zip = (zip_fn)ptr_of(z);
  p_reduce = (reduce_fn)ptr_of(r);
  p_matmul = (matmul_fn)ptr_of(mm);
  if (PyErr_Occurred()) return NULL;
  Py_RETURN_NONE;
}

/* a shape tuple and its strides tuple must have the same length (the library is passed only
   the shape's rank, so shorter strides would be read past their end) */
#define SAME_RANK(x, y, what)                                                              \
  if ((x) != (y))                                                                          \
    return PyErr_Format(PyExc_ValueError, "_mtfast: %s shape has %d dims, strides %d", what, \
                        (x), (y));

#define NEED(p)                                                              \
  if (!(p)) {                                                                \
    PyErr_SetString(PyExc_RuntimeError, "_mtfast: entry points not bound"); \
    return NULL;                                                             \
  }

/* map(fid, out, oshape, ostrides, a, ashape, astrides, stream) -> status */
static PyObject* fmap(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  NEED(p_map);
  if (n != 8) return PyErr_Format(PyExc_TypeError, "_mtfast.map takes 8 arguments");
  int64_t os[MAXD], ost[MAXD], as[MAXD], ast[MAXD];
  const int od = tup(a[2], os), od2 = tup(a[3], ost), ad = tup(a[5], as), ad2 = tup(a[6], ast);
  if (od < 0 || od2 < 0 || ad < 0 || ad2 < 0) return NULL;
  SAME_RANK(od, od2, "out");
  SAME_RANK(ad, ad2, "input");
  const int fid = (int)PyLong_AsLong(a[0]);
  float* out = (float*)ptr_of(a[1]);
  const float* in = (const float*)ptr_of(a[4]);
  void* st = ptr_of(a[7]);
  if (PyErr_Occurred()) return NULL;
  return PyLong_FromLong(p_map(fid, out, os, ost, od, in, as, ast, ad, st));
}

/* zip(fid, out, oshape, ostrides, a, ashape, astrides, b, bshape, bstrides, stream) -> status */
static PyObject* fzip(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  NEED(p_zip);
  if (n != 11) return PyErr_Format(PyExc_TypeError, "_mtfast.zip takes 11 arguments");
  int64_t os[MAXD], ost[MAXD], as[MAXD], ast[MAXD], bs[MAXD], bst[MAXD];
  const int od = tup(a[2], os), od2 = tup(a[3], ost), ad = tup(a[5], as), ad2 = tup(a[6], ast);
  const int bd = tup(a[8], bs), bd2 = tup(a[9], bst);
  if (od < 0 || od2 < 0 || ad < 0 || ad2 < 0 || bd < 0 || bd2 < 0) return NULL;
  SAME_RANK(od, od2, "out");
  SAME_RANK(ad, ad2, "a");
  SAME_RANK(bd, bd2, "b");
  const int fid = (int)PyLong_AsLong(a[0]);
  float* out = (float*)ptr_of(a[1]);
  const float* x = (const float*)ptr_of(a[4]);
  const float* y = (const float*)ptr_of(a[7]);
  void* st = ptr_of(a[10]);
  if (PyErr_Occurred()) return NULL;
  return PyLong_FromLong(p_zip(fid, out, os, ost, od, x, as, ast, ad, y, bs, bst, bd, st));
}

/* reduce(fid, out, oshape, ostrides, a, ashape, astrides, dim, start, stream) -> status */
static PyObject* freduce(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  NEED(p_reduce);
  if (n != 10) return PyErr_Format(PyExc_TypeError, "_mtfast.reduce takes 10 arguments");
  int64_t os[MAXD], ost[MAXD], as[MAXD], ast[MAXD];
  const int od = tup(a[2], os), od2 = tup(a[3], ost), ad = tup(a[5], as), ad2 = tup(a[6], ast);
  if (od < 0 || od2 < 0 || ad < 0 || ad2 < 0) return NULL;
  SAME_RANK(od, od2, "out");
  SAME_RANK(ad, ad2, "input");
  const int fid = (int)PyLong_AsLong(a[0]);
  float* out = (float*)ptr_of(a[1]);
  const float* in = (const float*)ptr_of(a[4]);
  const int dim = (int)PyLong_AsLong(a[7]);
  const float start = (float)PyFloat_AsDouble(a[8]);
  void* st = ptr_of(a[9]);
  if (PyErr_Occurred()) return NULL;
  return PyLong_FromLong(p_reduce(fid, out, os, ost, in, as, ast, ad, dim, start, st));
}

/* matmul(c, a, b, batch, M, N, K, sa, sb, sc, stream) -> status; strides are 3-tuples */
static PyObject* fmatmul(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  NEED(p_matmul);
  if (n != 11) return PyErr_Format(PyExc_TypeError, "_mtfast.matmul takes 11 arguments");
  int64_t sa[MAXD], sb[MAXD], sc[MAXD];
  if (tup(a[7], sa) != 3 || tup(a[8], sb) != 3 || tup(a[9], sc) != 3) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "_mtfast.matmul: strides are (batch, row, col)");
    return NULL;
  }
  float* c = (float*)ptr_of(a[0]);
  const float* x = (const float*)ptr_of(a[1]);
  const float* y = (const float*)ptr_of(a[2]);
  const int64_t batch = PyLong_AsLongLong(a[3]), M = PyLong_AsLongLong(a[4]), N = PyLong_AsLongLong(a[5]),
                K = PyLong_AsLongLong(a[6]);
  void* st = ptr_of(a[10]);
  if (PyErr_Occurred()) return NULL;
  return PyLong_FromLong(p_matmul(c, x, y, batch, M, N, K, sa, sb, sc, st));
}

static PyMethodDef methods[] = {
    {"bind", bind, METH_VARARGS, "bind(map, zip, reduce, matmul): the entry points' addresses"},
    {"map", (PyCFunction)(void (*)(void))fmap, METH_FASTCALL, "mt_tensor_map"},
    {"zip", (PyCFunction)(void (*)(void))fzip, METH_FASTCALL, "mt_tensor_zip"},
    {"reduce", (PyCFunction)(void (*)(void))freduce, METH_FASTCALL, "mt_tensor_reduce"},
    {"matmul", (PyCFunction)(void (*)(void))fmatmul, METH_FASTCALL, "mt_matmul_f32"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_mtfast", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__mtfast(void) { return PyModule_Create(&mod); }
